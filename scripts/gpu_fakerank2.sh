#!/bin/bash
# Fused-kernel tiling sweep on per-rank decompositions (fake ranks, no transport) and on the single-rank solve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fakerank2.log
: > $out
for fr in "1/8" "1/4" "1/2" "none"; do
  for rows in 1 2; do
    for tgt in 0 2048 4096 6144 8192 12288; do
      if [ "$fr" = none ]; then extra=""; else extra="--fake-rank $fr --decomp slab"; fi
      echo "== $fr rows $rows target $tgt" >> $out
      timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 8 --warmup 2 --quiet $extra --t2-rows $rows --t2-target $tgt >> $out 2>&1 || exit 1
    done
  done
done
