#!/bin/bash
# Reference-style GPU run (cf. the reference's LSF script: `mpirun -np 2 ./mpigpu-1 512 0.001 20 1`, report.pdf p.15).
#   scripts/run_gpu.sh [NGPU] [N] [TAU] [K] [L] [extra wave3d args...]
# One rank per GPU of this node, RCCL over xGMI; uses the native CLI's built-in launcher (no MPI needed).
set -euo pipefail
cd "$(dirname "$0")/.."
NGPU=${1:-1}; N=${2:-512}; TAU=${3:-0.001}; K=${4:-20}; L=${5:-1}
shift $(( $# < 5 ? $# : 5 ))
[ -x bin/wave3d ] || python tools/build.py
echo "Running test with grid size ${N}^3 on ${NGPU} GPU(s)"
exec bin/wave3d "$N" "$TAU" "$K" "$L" --np "$NGPU" "$@"
