#!/bin/bash
# GPU tests + reference-config CLI run + bench line (each step time-limited, chain stops at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 > gpurun_out/cli512.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
