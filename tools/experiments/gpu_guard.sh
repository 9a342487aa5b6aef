#!/bin/bash
# The stream-capture guard's one-time GPU check: the production topology (mode 0), then the round-4 split (mode 2,
# refused by the guard), each in its own process and under its own time limit; then the GPU test suite.
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for m in 0 2; do
  timeout -k 5 60 python -u -c "
import sys
from mpi_cuda_amd._native import load
C = load()
print('mode $m:', C.capture_guard_selftest($m), flush=True)
if $m == 2:
    print('mode 0 after the refusal:', C.capture_guard_selftest(0), flush=True)
" > gpurun_out/guard_selftest_m$m.log 2>&1
  rc=$?; cat gpurun_out/guard_selftest_m$m.log; [ $rc -eq 0 ] || exit 1
done
bash tools/experiments/gpu_ab_tests.sh
