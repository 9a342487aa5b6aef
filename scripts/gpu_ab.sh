#!/bin/bash
# Same-box A/B of the 512³ K=20 solve: bin/wave3d_old (previous build) vs bin/wave3d, interleaved, best of 20 each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
for r in 1 2 3 4; do
  for v in old new; do
    bin=./bin/wave3d; [ "$v" = old ] && bin=./bin/wave3d_old
    echo "== $r $v" >> $out
    timeout -k 10 60 $bin 512 0.001 20 1 --repeat 20 --warmup 3 --quiet 2>&1 | grep -E "Total time" >> $out || exit 1
  done
done
