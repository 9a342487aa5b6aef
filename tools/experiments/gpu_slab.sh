#!/bin/bash
# Slab ranks on one MI355X (fake ranks: one rank of a P-rank decomposition timed alone), pass depth 4 vs 5, with and
# without RCCL self traffic (--fake-traffic), sequential vs overlapped; then the GPU test suite.
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/slab.log
: > "$out"
for r in 0/2 1/4 1/8; do
  for t in 4 5; do
    for v in "--no-overlap" "--no-overlap --fake-traffic" "--fake-traffic"; do
      echo "== 512 $r slab temporal $t $v" >> "$out"
      timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r" --decomp slab --temporal "$t" $v --repeat 7 \
        --warmup 2 --quiet >> "$out" 2>&1 || exit 1
    done
  done
done
for v in "--no-overlap" "--no-overlap --fake-traffic" "--fake-traffic"; do
  echo "== 512 3/8 2x2x2 $v" >> "$out"
  timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank 3/8 --decomp 2x2x2 $v --repeat 7 --warmup 2 --quiet \
    >> "$out" 2>&1 || exit 1
done
grep -E "^==|Total time" "$out"
d=gpurun_out/trace_slab8
rm -rf "$d"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
  ./bin/wave3d 512 0.001 20 1 --fake-rank 1/8 --decomp slab --no-overlap --fake-traffic --repeat 5 --warmup 1 --quiet \
  > /dev/null 2>&1 || exit 1
python3 tools/trace_overlap.py "$d" > gpurun_out/trace_slab8.md
cat gpurun_out/trace_slab8.md
bash scripts/gpu.sh test || exit 1
