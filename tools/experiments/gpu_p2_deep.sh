#!/bin/bash
# Deep-prefetch A/B of the pair-tiled pass + the GPU test suite + slab ranks at S = 4 vs 5 (fake ranks, RCCL traffic).
#   build/ab/wave3d_base   : -DP2_DEEP=0 -DP2_COND_QUEUE (the first round-5 kernel)
#   build/ab/wave3d_nodeep : -DP2_DEEP=0 (unconditional queue writes only)
#   bin/wave3d             : deep prefetch (production)
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh abn ./build/ab/wave3d_base ./build/ab/wave3d_nodeep ./bin/wave3d || exit 1
out=gpurun_out/slab_s5.log
: > "$out"
for r in 0/2 1/8; do
  for t in 4 5; do
    for v in "--no-overlap" "--no-overlap --fake-traffic" "--fake-traffic"; do
      echo "== 512 $r slab temporal $t $v" >> "$out"
      timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r" --decomp slab --temporal "$t" $v --repeat 7 \
        --warmup 2 --quiet >> "$out" 2>&1 || exit 1
    done
  done
done
grep -E "^==|Total time" "$out"
bash scripts/gpu.sh test || exit 1
