set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sdmastreams
for ns in 1 2 3 4; do
  for v in "--no-overlap" ""; do
    tag="blk-ns$ns${v:+-seq}"
    echo "== 2x2x2 3/8 sdma streams=$ns $v"
    W3D_SDMA_STREAMS=$ns timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank 3/8 --decomp 2x2x2 --transport sdma $v \
      --repeat 60 --warmup 2 --quiet --json gpurun_out/sdmastreams/$tag.json | grep "Total time" || exit 1
  done
done
for ns in 2 4; do
  for v in "--no-overlap" ""; do
    tag="slab-ns$ns${v:+-seq}"
    echo "== slab 1/8 sdma streams=$ns $v"
    W3D_SDMA_STREAMS=$ns timeout -k 5 120 ./bin/wave3d 512 0.001 20 1 --fake-rank 1/8 --decomp slab --transport sdma $v \
      --repeat 60 --warmup 2 --quiet --json gpurun_out/sdmastreams/$tag.json | grep "Total time" || exit 1
  done
done
