#!/bin/bash
# TB kernel A/B: bit-exactness tests of every workgroup size, then the pass-cost sweep (tools/tune_leapfrog.py --tb).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "leapfrog_tb" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tb.log 2>&1 &&
timeout -k 10 300 python tools/tune_leapfrog.py --tb --json gpurun_out/tune_tb.json > gpurun_out/tune_tb.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
