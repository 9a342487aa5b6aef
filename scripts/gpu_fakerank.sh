#!/bin/bash
# Per-rank compute schedule of multi-GPU decompositions, timed alone on one GPU (no transport): upper bound for
# strong scaling before communication costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fakerank.log
: > $out
for cfg in "1/2 slab" "1/4 slab" "1/8 slab" "3/8 slab" "0/8 2x2x2" "0/4 2x2x1" "1/2 slab --no-overlap" "1/8 slab --no-overlap" "1/8 slab --no-graph"; do
  set -- $cfg
  echo "== fake-rank $1 decomp $2 ${3:-}" >> $out
  timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 --quiet --fake-rank $1 --decomp $2 ${3:-} >> $out 2>&1 || exit 1
done
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 --quiet --fake-rank 1/8 --decomp slab --timers >> $out 2>&1
