#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/occ.log
: > $out
for occ in 0 3 0 3; do
  for tgt in 0 8192; do
    echo "== occ $occ target $tgt" >> $out
    timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 --quiet --t2-occ $occ --t2-target $tgt >> $out 2>&1 || exit 1
  done
done
