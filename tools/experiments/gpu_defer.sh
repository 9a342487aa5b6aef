#!/bin/bash
# Deferred own-wave stores A/B (build/ab/wave3d_storeall: every wave stores, at the stage), the kernel + new tests,
# the full GPU suite, then the capture-topology probe (the round-4 split topology last: it may crash on the host).
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh abn ./build/ab/wave3d_storeall ./bin/wave3d || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl_cli.py tests/test_gpu_sdma.py \
  -x -v --timeout 240 --timeout-method thread -k "p2 or leapfrog_tb or block_p2 or bench or traffic" \
  > gpurun_out/pytest_new.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu.sh test || exit 1
p=./build/probes/capture_probe3
for m in 0 1 3 4; do timeout -k 5 60 $p $m 4 > gpurun_out/capture_probe3_m$m.log 2>&1 || { cat gpurun_out/capture_probe3_m$m.log; exit 1; }; tail -1 gpurun_out/capture_probe3_m$m.log; done
timeout -k 5 60 $p 2 4 1 > gpurun_out/capture_probe3_m2_eager.log 2>&1 || exit 1
tail -1 gpurun_out/capture_probe3_m2_eager.log
timeout -k 5 60 $p 2 4 > gpurun_out/capture_probe3_m2.log 2>&1
echo "mode 2 captured: exit $?"; tail -3 gpurun_out/capture_probe3_m2.log
