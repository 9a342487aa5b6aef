#!/bin/bash
# 2048^3 2x2x2 block rank 3/8 (fake rank, copy-engine traffic real): 20 timed solves after 8 warmups per schedule
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/sdma2048
for v in "--no-overlap" "--transport sdma" "--transport sdma --no-overlap"; do
  tag=$(echo "$v" | tr -d ' -')
  echo "== 2048 fake 3/8 2x2x2 $v"
  timeout -k 10 200 ./bin/wave3d 2048 0.00025 20 1 --fake-rank 3/8 --decomp 2x2x2 --repeat 20 --warmup 8 --quiet $v \
    --json gpurun_out/sdma2048/$tag.json | grep "Total time" || exit 1
done
