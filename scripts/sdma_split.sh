#!/bin/bash
# slab copy-engine ranks with each face's two field copies on two streams (W3D_SDMA_SPLIT=1) vs one stream per face:
# 512^3 slab rank 1/8 (fake rank), 40 timed solves after 8 warmups; and a 2-process bit-exactness check at N=96
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sdmasplit
for r in 1 2; do
  for sp in 0 1; do
    for v in "" "--no-overlap"; do
      tag="split$sp${v:+-seq}-r$r"
      echo "== round $r split=$sp $v"
      W3D_SDMA_SPLIT=$sp timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --fake-rank 1/8 --transport sdma $v --repeat 40 \
        --warmup 8 --quiet --json gpurun_out/sdmasplit/$tag.json | grep "Total time" || exit 1
    done
  done
done
W3D_SDMA_SPLIT=1 W3D_SHARE_GPUS=1 W3D_TIMEOUT_S=30 timeout -k 10 120 ./bin/wave3d 96 0.001 20 1 --np 2 --no-rccl \
  --transport sdma --warmup 2 --repeat 20 --verify-repeat --quiet --json gpurun_out/sdmasplit/np2.json || exit 1
timeout -k 10 60 ./bin/wave3d 96 0.001 20 1 --quiet --json gpurun_out/sdmasplit/one.json || exit 1
python3 -c "
import json
a=json.load(open('gpurun_out/sdmasplit/np2.json'))['steps']; b=json.load(open('gpurun_out/sdmasplit/one.json'))['steps']
print('np2 split log == 1-GPU log:', all(x[0]==y[0] and abs(x[1]-y[1])<=1e-12*y[1] and abs(x[2]-y[2])<=1e-9*y[2] for x,y in zip(a,b)) and len(a)==len(b))
"
