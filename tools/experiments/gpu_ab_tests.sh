#!/bin/bash
# Same-box A/B of the CLI builds named in $AB_BINS (scripts/gpu.sh abn), the new/changed GPU tests ($AB_K: a pytest -k
# expression), the full GPU suite, then the capture-topology probe (the round-4 split topology last: it may crash on
# the host, and the script ends there).
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${AB_BINS:-}" ]; then bash scripts/gpu.sh abn $AB_BINS || exit 1; fi
if [ -n "${AB_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$AB_K" \
    > gpurun_out/pytest_new.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit 1
fi
if [ -z "${AB_NO_SUITE:-}" ]; then bash scripts/gpu.sh test || exit 1; fi
if [ -n "${AB_PROBE:-}" ]; then
  p=./build/probes/capture_probe3
  for m in 0 1 3 4; do timeout -k 5 60 $p $m 4 > gpurun_out/capture_probe3_m$m.log 2>&1 || { cat gpurun_out/capture_probe3_m$m.log; exit 1; }; tail -1 gpurun_out/capture_probe3_m$m.log; done
  timeout -k 5 60 $p 2 4 1 > gpurun_out/capture_probe3_m2_eager.log 2>&1 || exit 1
  tail -1 gpurun_out/capture_probe3_m2_eager.log
  timeout -k 5 60 $p 2 4 > gpurun_out/capture_probe3_m2.log 2>&1
  echo "mode 2 captured: exit $?"; tail -3 gpurun_out/capture_probe3_m2.log
fi
