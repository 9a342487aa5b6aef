#!/bin/bash
# Python Solver(runtime="process") vs the native CLI, same job shape (2 ranks sharing the GPU, copy engines, no RCCL),
# 512^3 K=20: per-solve times -> gpurun_out/proc_parity.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export W3D_SHARE_GPUS=1 W3D_TIMEOUT_S=60
for round in 1 2; do
  echo "== round $round CLI --np 2 --no-rccl --transport sdma"
  timeout -k 10 180 ./bin/wave3d 512 0.001 20 1 --np 2 --no-rccl --transport sdma --warmup 8 --repeat 20 --quiet \
    --json gpurun_out/proc_cli.json | grep "Total time" || exit 1
  python3 -c "import json,statistics as s;t=json.load(open('gpurun_out/proc_cli.json'))['solve_times_s'][8:];print('cli median %.6f mean %.6f'%(s.median(t),s.mean(t)))" || exit 1
  echo "== round $round Python Solver(runtime=process)"
  timeout -k 10 300 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    tools/proc_runtime_bench.py --N 512 --transport sdma --no-rccl --reps 20 --warmup 8 || exit 1
done
