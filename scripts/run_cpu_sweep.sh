#!/bin/bash
# Reference-style CPU sweeps (report.pdf p.7-11, p.20-26): grids {128,256,512} x OpenMP threads (sequential/OpenMP
# programs) and x ranks over torch.distributed gloo (MPI / MPI+OpenMP programs). Writes JSON lines to $OUT.
#   scripts/run_cpu_sweep.sh [OUT=cpu_sweep.jsonl] [GRIDS="128 256"] [THREADS="1 2 4 8"] [RANKS="1 2 4"]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-cpu_sweep.jsonl}; GRIDS=${GRIDS:-"128 256"}; THREADS=${THREADS:-"1 2 4 8"}; RANKS=${RANKS:-"1 2 4"}
[ -x bin/wave3d ] || python tools/build.py
: > "$OUT"
for g in $GRIDS; do
  echo "Running test with grid size ${g}^3"
  for t in $THREADS; do
    bin/wave3d "$g" 0.001 20 --cpu --threads "$t" --quiet --json /tmp/w3d_cpu.json > /dev/null
    python - "$t" >> "$OUT" <<'PY'
import json, sys
d = json.load(open("/tmp/w3d_cpu.json")); d["mode"] = "openmp"; d["workers"] = int(sys.argv[1]); print(json.dumps(d))
PY
  done
  for p in $RANKS; do
    OMP_NUM_THREADS=1 python -m torch.distributed.run --nproc-per-node "$p" --master-addr 127.0.0.1 \
      --master-port $((29700 + p)) -m mpi_cuda_amd "$g" 0.001 20 --backend cpu --transport torch --threads 1 \
      --quiet --json /tmp/w3d_mpi.json > /dev/null
    python - "$p" >> "$OUT" <<'PY'
import json, sys
d = json.load(open("/tmp/w3d_mpi.json")); d["mode"] = "ranks"; d["workers"] = int(sys.argv[1]); print(json.dumps(d))
PY
  done
done
python tools/scaling_report.py "$OUT"
