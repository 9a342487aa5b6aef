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
