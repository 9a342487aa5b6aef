#!/bin/bash
# Price the RCCL halo exchange with real traffic on one MI355X: a fake rank (--fake-rank R/P)
# runs its production schedule alone; --fake-traffic sends and receives its exact message set to itself over a one-rank
# RCCL communicator, so RCCL's copy kernels take CUs and HBM bandwidth next to the passes as on a node (the xGMI hop
# itself is not priced). Sequential (--no-overlap) and overlapped schedules, with and without CUs reserved for RCCL;
# the copy-engine transport beside them. Then one kernel trace of an overlapped case (RCCL kernels vs the passes).
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/traffic.log
: > "$out"
run() {  # label, args...
  local label=$1; shift
  echo "== $label :: $*" >> "$out"
  timeout -k 5 150 ./bin/wave3d "$@" --repeat 7 --warmup 2 --quiet >> "$out" 2>&1 || { echo "FAILED $label" >> "$out"; return 1; }
}
for fr in 512:0.001:0/2:slab 512:0.001:1/8:slab 512:0.001:3/8:2x2x2 2048:0.00025:3/8:2x2x2; do
  IFS=: read -r N tau r dec <<< "$fr"
  base=("$N" "$tau" 20 1 --fake-rank "$r" --decomp "$dec")
  run "N=$N $r $dec compute only (no exchange), seq"    "${base[@]}" --no-overlap || exit 1
  run "N=$N $r $dec rccl traffic, seq"                   "${base[@]}" --no-overlap --fake-traffic || exit 1
  run "N=$N $r $dec rccl traffic, overlap"               "${base[@]}" --fake-traffic || exit 1
  run "N=$N $r $dec rccl traffic, overlap, 16 CUs kept"  "${base[@]}" --fake-traffic --reserve-cus 16 || exit 1
  run "N=$N $r $dec rccl traffic, overlap, 32 CUs kept"  "${base[@]}" --fake-traffic --reserve-cus 32 || exit 1
  run "N=$N $r $dec copy engines, overlap"               "${base[@]}" --transport sdma || exit 1
done
grep -E "^==|Total time|FAILED" "$out"
for c in "0/2 slab" "1/8 slab" "3/8 2x2x2"; do
  set -- $c
  d="gpurun_out/trace_traffic_${1/\//of}_$2"
  rm -rf "$d"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- \
    ./bin/wave3d 512 0.001 20 1 --fake-rank "$1" --decomp "$2" --fake-traffic --repeat 5 --warmup 1 --quiet \
    > /dev/null 2>&1 || exit 1
  echo "== trace $c (overlap, rccl traffic)"
  python3 tools/trace_overlap.py "$d" | head -8
done
# raw TCC read counters of the reference config (FETCH_SIZE of 128-byte requests: TCC_BUBBLE)
rm -rf gpurun_out/pmc_tcc1 gpurun_out/pmc_tcc2
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum \
  --kernel-trace --output-format csv -d gpurun_out/pmc_tcc1 -o run -- ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 \
  --quiet > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_WRREQ_sum \
  --kernel-trace --output-format csv -d gpurun_out/pmc_tcc2 -o run -- ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 \
  --quiet > /dev/null 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_tcc1 gpurun_out/pmc_tcc2 | grep -v "__amd" > gpurun_out/pmc_tcc.md
cat gpurun_out/pmc_tcc.md
