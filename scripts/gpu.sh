#!/bin/bash
# One parametrised GPU-box driver (replaces the round-1 scratch scripts/gpu_*.sh). Every step that touches the GPU runs
# under its own time limit and the steps are chained with &&: the first failure, fault or timeout ends the call.
#
#   scripts/gpu.sh test [pytest -k expr]     pytest -m gpu (one process, per-test timeout) -> gpurun_out/pytest_gpu.log
#   scripts/gpu.sh bench [bench.py args]     1-GPU bench.py line                            -> gpurun_out/bench.log
#   scripts/gpu.sh prof [wave3d args]        rocprofv3 kernel trace + stats of the 512^3 CLI solve -> gpurun_out/prof/
#   scripts/gpu.sh profbench [bench args]    rocprofv3 kernel trace + stats of bench.py     -> gpurun_out/profbench/
#   scripts/gpu.sh pmc "<counters>" [wave3d args]  one PMC pass (counters of one block budget) -> gpurun_out/pmc/
#   scripts/gpu.sh cli [wave3d args]         the reference-config CLI run (512 0.001 20 1)   -> gpurun_out/cli.log
#   scripts/gpu.sh fakerank                  per-rank solve times (--fake-rank) of the slab schedules: RCCL overlap /
#                                            sequential, push overlap / sequential, 512^3 ranks 1/8 + 1/2, 2048^3 3/8;
#                                            2x2x2 blocks (overlap / sequential) at 512^3 and 2048^3, rank 3/8
#   scripts/gpu.sh fakesweep                 512^3 compute-only scaling projection (one rank of P, P = 1/2/4/8)
#   scripts/gpu.sh ab [wave3d args]          same-box A/B: build/ab/wave3d_base vs bin/wave3d -> gpurun_out/ab.log
#   scripts/gpu.sh transports                per-rank solve times (--fake-rank) of sequential / RCCL-overlap / copy-engine
#                                            (sdma) schedules: 512^3 slab 1/8 + 1/2, 2x2x2 blocks at 512^3 and 2048^3
#                                            -> gpurun_out/transports.log
#   scripts/gpu.sh attrib                    LDS-pass kernel times: production, no checks, 768 threads, experiment builds
#                                            build/ab/wave3d_noload / _nostore -> gpurun_out/attrib.txt
#   scripts/gpu.sh abn BIN...               same-box interleaved A/B/n of any binaries + their kernel stats -> abn.log
#   scripts/gpu.sh sdmatail                  per-solve times of the copy-engine fake ranks + a copy/kernel trace -> sdmatail/
#   scripts/gpu.sh probe                     tools/probes/sdma_probe (copy engines, memops, capture) -> gpurun_out/probe.log
#   scripts/gpu.sh all                       test && cli && bench && profbench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what=${1:-all}
shift || true

run_test() {
  local k=()
  [ $# -gt 0 ] && k=(-k "$*")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${k[@]}" \
    > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  return $rc
}
run_bench() {
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench.log 2>&1
  local rc=$?
  tail -2 gpurun_out/bench.log
  return $rc
}
run_cli() {
  timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 2 "$@" > gpurun_out/cli.log 2>&1
  local rc=$?
  tail -4 gpurun_out/cli.log
  return $rc
}
run_prof() {
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 "$@" > gpurun_out/prof.log 2>&1
}
run_profbench() {
  rm -rf gpurun_out/profbench
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profbench -o run -- \
    python3 bench.py --steps 5 --warmup 2 "$@" > gpurun_out/profbench.log 2>&1
}
run_pmc() {
  local counters=$1
  shift
  rm -rf gpurun_out/pmc
  timeout -s KILL 90 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d gpurun_out/pmc -o run -- \
    ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 "$@" > gpurun_out/pmc.log 2>&1
}

run_fakerank() {
  local fr v
  for fr in 512:0.001:1/8 512:0.001:1/2 2048:0.00025:3/8; do
    IFS=: read -r N tau r <<< "$fr"
    for v in "" "--no-overlap" "--transport push" "--transport push --no-overlap"; do
      echo "== N=$N fake $r $v"
      timeout -k 5 120 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$r" --repeat 5 --warmup 2 --quiet $v \
        | grep "Total time" || return 1
    done
  done
  for fr in 512:0.001:3/8 2048:0.00025:3/8; do  # 3-D blocks 2x2x2: overlap / sequential
    IFS=: read -r N tau r <<< "$fr"
    for v in "" "--no-overlap"; do
      echo "== N=$N fake $r --decomp 2x2x2 $v"
      timeout -k 5 120 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$r" --decomp 2x2x2 --repeat 5 --warmup 2 --quiet $v \
        | grep "Total time" || return 1
    done
  done
}

# same-box A/B of the reference-config CLI: build/ab/wave3d_base (a copy of an earlier build) against bin/wave3d,
# interleaved rounds of best-of-20 solves
# (W3D_AB_NEW_ARGS: extra arguments for bin/wave3d only, e.g. a new option the base build does not know)
run_ab() {
  local r b extra
  for r in 1 2 3; do
    for b in build/ab/wave3d_base bin/wave3d; do
      extra=""
      [ "$b" = bin/wave3d ] && extra="${W3D_AB_NEW_ARGS:-}"
      echo "== round $r $b $extra"
      timeout -k 5 120 "$b" 512 0.001 20 1 --repeat 20 --warmup 2 --quiet $extra "$@" | grep -i "time" || return 1
    done
  done
}

# same-box A/B/n of the reference-config CLI over any binaries: interleaved rounds of best-of-20 solves, then the
# rocprofv3 kernel stats of each (leapfrog passes, avg / min us) -> gpurun_out/abn.log
# (a spec BIN@ARGS passes ARGS to that binary only, e.g. bin/wave3d@--tb-threads,768 — commas become spaces)
run_abn() {
  local r b n spec extra
  for r in 1 2 3; do
    for spec in "$@"; do
      b=${spec%%@*}; extra=""; [ "$spec" != "$b" ] && extra=${spec#*@}; extra=${extra//,/ }
      echo "== round $r $b $extra"
      timeout -k 5 120 "$b" 512 0.001 20 1 --repeat 20 --warmup 2 --quiet $extra | grep -i "total time" || return 1
    done
  done
  for spec in "$@"; do
    b=${spec%%@*}; extra=""; [ "$spec" != "$b" ] && extra=${spec#*@}; extra=${extra//,/ }
    n=$(basename "$b")$(echo "$extra" | tr -d ' -')
    rm -rf "gpurun_out/abn/$n"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/abn/$n" -o run -- \
      "$b" 512 0.001 20 1 --repeat 10 --warmup 2 --quiet $extra > /dev/null 2>&1 || return 1
    echo "== kernels $n"
    python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abn/$n/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'leapfrog' in r['Name']:
            print(r['Name'].split('(')[0][-60:], r['Calls'], 'avg', round(float(r['AverageNs'])/1e3,1), 'min', round(float(r['MinNs'])/1e3,1))
for f in glob.glob('gpurun_out/abn/$n/**/run_kernel_trace.csv', recursive=True):
    seen=set()
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name'].split('(')[0][-50:]
        if 'leapfrog' in k and k not in seen:
            seen.add(k); print('  regs', k, 'vgpr', r['VGPR_Count'], 'agpr', r.get('Accum_VGPR_Count'), 'sgpr', r['SGPR_Count'], 'scratch', r['Scratch_Size'], 'lds', r['LDS_Block_Size'])
"
  done
}

# perf attribution of the LDS passes: rocprofv3 kernel stats of the production solve, the same solve without error
# checks, and the experiment builds build/ab/wave3d_<variant> (W3D_EXTRA_DEFS=-DW3D_EXPERIMENT_<VARIANT>, results
# wrong) -> gpurun_out/attrib/<name>/ and gpurun_out/attrib.txt
run_attrib() {
  local name bin extra
  rm -rf gpurun_out/attrib
  mkdir -p gpurun_out/attrib
  : > gpurun_out/attrib.txt
  for spec in "base:build/ab/wave3d_base:" "prod:bin/wave3d:" "nocheck:bin/wave3d:--check-every 100" "t768:bin/wave3d:--tb-threads 768" \
              "noload:build/ab/wave3d_noload:" "nostore:build/ab/wave3d_nostore:" "static:build/ab/wave3d_static:" "plainstore:build/ab/wave3d_plainstore:"; do
    IFS=: read -r name bin extra <<< "$spec"
    [ -x "$bin" ] || continue
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attrib/$name -o run -- \
      "$bin" 512 0.001 20 1 --repeat 10 --warmup 2 --quiet $extra > gpurun_out/attrib/$name.log 2>&1 || return 1
    echo "== $name $extra" >> gpurun_out/attrib.txt
    python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/attrib/$name/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'leapfrog' in r['Name']:
            print(r['Name'].split('(')[0][-60:], r['Calls'], 'avg', round(float(r['AverageNs'])/1e3,1), 'min', round(float(r['MinNs'])/1e3,1))
" >> gpurun_out/attrib.txt
  done
  cat gpurun_out/attrib.txt
}

# compute-only strong-scaling projection of the 512^3 solve: one rank of P timed alone (--fake-rank, no transport
# traffic) for the sequential slab and block schedules; one JSON line per point -> gpurun_out/fakesweep.jsonl.
# (round 6: solve_s = the bench.py measure, a block of 20 graph replays enqueued back to back — --bench-steps, which
# multi-rank RCCL runs now pipeline too; repeat_best_s = the best of 10 solves with a host round trip each, as before;
# every point after ≈ 130 ms of untimed solves — 40 × P of them — so the 1-GPU solve and the short fake-rank solves are
# timed at the same settled clock: the power controller's transient after a burst from idle lasts ≈ 15 one-GPU solves,
# profiles/r6/clock/)
run_fakesweep() {
  local P dec r j out=gpurun_out/fakesweep.jsonl
  : > "$out"
  timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --repeat 10 --warmup 40 --bench-steps 20 --quiet --json /tmp/fs.json \
    > /dev/null || return 1
  python3 -c "import json;d=json.load(open('/tmp/fs.json'));print(json.dumps({'P':1,'decomp':'1x1x1','rank':0,'solve_s':d['bench_s']/d['bench_steps'],'repeat_best_s':d['solve_s']}))" >> "$out" || return 1
  for P in 2 4 8; do
    for dec in slab block; do
      [ "$dec" = block ] && [ "$P" -lt 4 ] && continue
      for r in 0 1; do
        timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r/$P" --decomp "$dec" --no-overlap --repeat 10 \
          --warmup $((40 * P)) --bench-steps 20 --quiet --json /tmp/fs.json > /dev/null || return 1
        python3 -c "import json,sys;d=json.load(open('/tmp/fs.json'));print(json.dumps({'P':$P,'decomp':'x'.join(map(str,d['dims'])),'schedule':'$dec-seq','rank':$r,'solve_s':d['bench_s']/d['bench_steps'],'repeat_best_s':d['solve_s']}))" >> "$out" || return 1
        timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r/$P" --decomp "$dec" --no-overlap --fake-traffic \
          --repeat 10 --warmup $((40 * P)) --bench-steps 20 --quiet --json /tmp/fs.json > /dev/null || return 1
        python3 -c "import json,sys;d=json.load(open('/tmp/fs.json'));print(json.dumps({'P':$P,'decomp':'x'.join(map(str,d['dims'])),'schedule':'$dec-seq-rccltraffic','rank':$r,'solve_s':d['bench_s']/d['bench_steps'],'repeat_best_s':d['solve_s']}))" >> "$out" || return 1
      done
    done
  done
  # (round 4) the same ranks WITH their copy-engine traffic, mean of 20 solves after 8 warmups ("sdma" schedules: a
  # second, pessimistic curve — one GPU's engines carry what a node's links would)
  local v tag
  for P in 2 4 8; do
    for spec in "slab:--transport sdma:slab-sdma" "slab:--transport sdma --no-overlap:slab-sdma-seq" \
                "block:--transport sdma --no-overlap:block-sdma-seq"; do
      IFS=: read -r dec v tag <<< "$spec"
      [ "$dec" = block ] && [ "$P" -lt 4 ] && continue
      for r in 0 1; do
        timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r/$P" --decomp "$dec" $v --repeat 20 \
          --warmup 8 --quiet --json /tmp/fs.json > /dev/null || return 1
        python3 -c "import json,sys;d=json.load(open('/tmp/fs.json'));print(json.dumps({'P':$P,'decomp':'x'.join(map(str,d['dims'])),'schedule':'$tag','rank':$r,'solve_s':d['mean_s'],'best_s':d['solve_s']}))" >> "$out" || return 1
      done
    done
  done
  cat "$out"
}

run_transports() {
  local fr v
  local vs=("--no-overlap" "" "--transport sdma" "--transport sdma --no-overlap")
  [ -n "${W3D_TRANSPORTS_VARIANTS:-}" ] && IFS=';' read -r -a vs <<< "$W3D_TRANSPORTS_VARIANTS"
  for fr in 512:0.001:1/8:slab 512:0.001:0/2:slab 512:0.001:3/8:2x2x2 2048:0.00025:3/8:2x2x2; do
    IFS=: read -r N tau r dec <<< "$fr"
    for v in "${vs[@]}"; do
      echo "== N=$N fake $r --decomp $dec $v"
      timeout -k 5 120 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$r" --decomp "$dec" --repeat 7 --warmup 2 --quiet $v \
        | grep -E "Total time|Throughput" || return 1
    done
  done
}
# SDMA tail study: per-solve times of the copy-engine fake ranks (--json solve_times_s), then
# a kernel + memory-copy trace of 12 back-to-back solves of the 512^3 slab rank 1/8 -> gpurun_out/sdmatail/
run_sdmatail() {
  local d=gpurun_out/sdmatail fr v tag
  rm -rf "$d"
  mkdir -p "$d"
  for fr in 512:0.001:1/8:slab 512:0.001:3/8:2x2x2; do
    IFS=: read -r N tau r dec <<< "$fr"
    for v in "--transport sdma" "--transport sdma --no-overlap" "--no-overlap"; do
      tag="$(echo "$N-$r-$dec-$v" | tr ' /' '_-')"
      echo "== N=$N fake $r --decomp $dec $v"
      timeout -k 5 120 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$r" --decomp "$dec" --repeat 20 --warmup 2 --quiet $v \
        --json "$d/$tag.json" | grep -E "Total time" || return 1
      python3 -c "import json;t=json.load(open('$d/$tag.json'))['solve_times_s'];print(' '.join('%.2f'%(x*1e3) for x in t))"
    done
  done
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$d/trace" -o run -- \
    ./bin/wave3d 512 0.001 20 1 --fake-rank 1/8 --decomp slab --transport sdma --repeat 10 --warmup 2 --quiet \
    --json "$d/trace.json" > "$d/trace.log" 2>&1 || return 1
  python3 tools/trace_overlap.py "$d/trace" --json "$d/trace.json" --solves 12
}
run_probe() {
  [ -x build/sdma_probe ] || { echo "build/sdma_probe missing" >&2; return 1; }
  timeout -k 10 120 build/sdma_probe > gpurun_out/probe.log 2>&1
  local rc=$?
  cat gpurun_out/probe.log
  return $rc
}

case "$what" in
  transports) run_transports > gpurun_out/transports.log 2>&1; rc=$?; cat gpurun_out/transports.log; exit $rc ;;
  sdmatail) run_sdmatail > gpurun_out/sdmatail.log 2>&1; rc=$?; cat gpurun_out/sdmatail.log; exit $rc ;;
  probe) run_probe ;;
  fakesweep) run_fakesweep ;;
  ab) run_ab "$@" > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log; exit $rc ;;
  abn) run_abn "$@" > gpurun_out/abn.log 2>&1; rc=$?; cat gpurun_out/abn.log; exit $rc ;;
  test) run_test "$@" ;;
  bench) run_bench "$@" ;;
  cli) run_cli "$@" ;;
  prof) run_prof "$@" ;;
  profbench) run_profbench "$@" ;;
  pmc) run_pmc "$@" ;;
  attrib) run_attrib ;;
  fakerank) run_fakerank > gpurun_out/fakerank.log 2>&1; rc=$?; cat gpurun_out/fakerank.log; exit $rc ;;
  all) run_test && run_cli && run_bench && run_profbench ;;
  *) echo "unknown step $what" >&2; exit 2 ;;
esac
