#!/bin/bash
# Reference-style CPU sweeps (report.pdf p.7-11, p.20-26): grids x OpenMP threads (the sequential / OpenMP programs)
# and x processes (the MPI program: native `wave3d --cpu --np P`, one process per rank over shared memory; MPI+OpenMP:
# P processes x T threads). Best of REPEAT solves per point. Writes JSON lines to $OUT, prints the tables, draws the
# speedup / efficiency figure next to it.
#   scripts/run_cpu_sweep.sh [OUT=cpu_sweep.jsonl] [GRIDS="128 256"] [THREADS="1 2 4 8"] [RANKS="1 2 4 8"]
#                            [HYBRID="2x2 2x4 4x2"] [REPEAT=3]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-cpu_sweep.jsonl}; GRIDS=${GRIDS:-"128 256"}; THREADS=${THREADS:-"1 2 4 8"}; RANKS=${RANKS:-"1 2 4 8"}
HYBRID=${HYBRID:-"2x2 2x4 4x2"}; REPEAT=${REPEAT:-3}
[ -x bin/wave3d ] || python tools/build.py
: > "$OUT"
tag() {  # tag <json> <mode> <workers>: add the sweep coordinates to one result line
  python - "$@" >> "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); d["mode"] = sys.argv[2]; d["workers"] = int(sys.argv[3]); print(json.dumps(d))
PY
}
for g in $GRIDS; do
  echo "Running test with grid size ${g}^3"
  for t in $THREADS; do
    bin/wave3d "$g" 0.001 20 --cpu --threads "$t" --repeat "$REPEAT" --quiet --json /tmp/w3d_cpu.json > /dev/null
    tag /tmp/w3d_cpu.json openmp "$t"
  done
  for p in $RANKS; do
    if [ "$p" = 1 ]; then
      bin/wave3d "$g" 0.001 20 --cpu --threads 1 --repeat "$REPEAT" --quiet --json /tmp/w3d_mpi.json > /dev/null
    else
      bin/wave3d "$g" 0.001 20 --cpu --np "$p" --threads 1 --repeat "$REPEAT" --quiet --json /tmp/w3d_mpi.json > /dev/null
    fi
    tag /tmp/w3d_mpi.json mpi "$p"
  done
  for h in $HYBRID; do
    p=${h%x*}; t=${h#*x}
    bin/wave3d "$g" 0.001 20 --cpu --np "$p" --threads "$t" --repeat "$REPEAT" --quiet --json /tmp/w3d_hyb.json > /dev/null
    tag /tmp/w3d_hyb.json "mpi+openmp(${p}x${t})" $((p * t))
  done
done
python tools/scaling_report.py "$OUT" --plot "${OUT%.jsonl}.png"
