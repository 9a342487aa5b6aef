#!/bin/bash
# kernel traces of the 512^3 2x2x2 block rank 3/8 (fake rank), overlapped and sequential -> gpurun_out/blktrace/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
rm -rf gpurun_out/blktrace; mkdir -p gpurun_out/blktrace
for v in ovl seq; do
  extra=""; [ $v = seq ] && extra="--no-overlap"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/blktrace/$v -o run -- \
    ./bin/wave3d 512 0.001 20 1 --fake-rank 3/8 --decomp 2x2x2 --repeat 4 --warmup 2 --quiet $extra \
    > gpurun_out/blktrace/$v.log 2>&1 || exit 1
done
