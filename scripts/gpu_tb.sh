#!/bin/bash
# Deep temporal blocking: numerics vs CPU steps, then the kernel sweep at 512³.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "leapfrog_tb" > gpurun_out/pytest_tb.log 2>&1 &&
timeout -k 10 300 python tools/tune_leapfrog.py --tb --json gpurun_out/tune_tb.json > gpurun_out/tune_tb.log 2>&1
