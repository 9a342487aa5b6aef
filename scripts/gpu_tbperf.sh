#!/bin/bash
# LDS S-step kernel change: GPU tests (bit-exactness), kernel sweep at 512³, CLI at the reference config, deep-tb ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/tune_leapfrog.py --tb --json gpurun_out/tune_tb.json > gpurun_out/tune_tb.log 2>&1 &&
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 20 --warmup 3 > gpurun_out/cli512.log 2>&1 &&
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 --timers --trace gpurun_out/trace1.jsonl --quiet >> gpurun_out/cli512.log 2>&1 &&
for cfg in 1/2 1/4 1/8; do
  timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 --quiet --fake-rank $cfg >> gpurun_out/cli512.log 2>&1 || exit 1
done
