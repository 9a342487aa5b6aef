#!/bin/bash
# Strong-scaling sweep of the headline benchmark (512^3, K=20) at 1/2/4/8 GPUs of one node via bench.py (one rank per
# GPU, torch.distributed.run), plus the 2048^3 block-decomposed weak point. JSON lines -> $OUT, table -> stdout.
#   scripts/run_scaling.sh [OUT=scaling.jsonl] [GPUS="1 2 4 8"]
set -uo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-scaling.jsonl}; GPUS=${GPUS:-"1 2 4 8"}
: > "$OUT"
for n in $GPUS; do
  if [ "$n" = 1 ]; then
    timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 --out "$OUT" || exit $?
  else
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus "$n" --steps 20 --warmup 3 --out "$OUT" || exit $?
  fi
done
python tools/scaling_report.py "$OUT"
# 2048^3 fp64 (stable tau: the CFL limit at L=1 is 2.8e-4) on all 8 GPUs (BASELINE config 5); 3 timed
# solves. The schedule is autotuned with the copy-engine candidates included (--autotune-sdma): the only 2048^3
# exchange measured with real traffic is the copy-engine one (2x2x2 block rank, profiles/r3/sdma_transport.md), and
# RCCL's copy kernels need CUs the LDS passes hold; the autotune still times the RCCL block/slab schedules next to it
# and keeps the fastest whose log and fields match.
if echo " $GPUS " | grep -q " 8 "; then
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29599 bench.py --gpus 8 --N 2048 --tau 2.5e-4 --autotune-sdma --steps 3 --warmup 2 \
    --out "${OUT%.jsonl}_2048.jsonl" || exit $?
fi
