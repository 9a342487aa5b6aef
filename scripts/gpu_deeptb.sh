#!/bin/bash
# deep-tb (LDS S-step passes on slab ranks): loopback bit-exactness tests, then per-rank schedules of 512³ K=20
# timed alone on one GPU (--fake-rank, no transport) against the previous slab schedules.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/deeptb.log
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread \
  -k "deep_tb or schedule_modes or deep_halo" > gpurun_out/pytest_deeptb.log 2>&1 || exit 1
for cfg in "0/2" "1/2" "1/4" "0/8" "1/8" "1/16"; do
  for opt in "" "--no-tb" "--no-overlap"; do
    echo "== fake-rank $cfg slab $opt" >> $out
    timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 --quiet --fake-rank $cfg --decomp slab $opt >> $out 2>&1 || exit 1
  done
done
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 --quiet --fake-rank 1/8 --decomp slab --timers >> $out 2>&1
