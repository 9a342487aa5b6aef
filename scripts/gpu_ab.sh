#!/bin/bash
# Same-box A/B of the 512³ K=20 solve: bin/wave3d_old (previous kernel build) vs bin/wave3d variants, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
for r in 1 2 3; do
  for v in "old" "new" "new --tb-threads 1024" "new --tb-threads 768"; do
    set -- $v
    bin=./bin/wave3d; [ "$1" = old ] && bin=./bin/wave3d_old
    shift
    echo "== $r $v" >> $out
    timeout -k 10 60 $bin 512 0.001 20 1 --repeat 20 --warmup 3 "$@" 2>&1 | grep -E "Total time|Throughput" >> $out || exit 1
  done
done
