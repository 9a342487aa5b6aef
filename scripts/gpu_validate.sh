#!/bin/bash
# One GPU-box validation pass: smoke, CLI at the reference config, GPU tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
step smoke && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
step cli && timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 > gpurun_out/cli512.log 2>&1 &&
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 --no-graph --timers >> gpurun_out/cli512.log 2>&1 &&
step pytest && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
step bench && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 &&
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 > gpurun_out/prof.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
