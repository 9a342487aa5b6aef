set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for N in 512; do
for fr in 1/8 1/2 ; do
for v in "" "--no-overlap" "--transport push" "--transport push --no-overlap"; do
  echo "== N=$N fake $fr $v" 
  timeout -k 5 60 ./bin/wave3d $N 0.001 20 1 --fake-rank $fr --repeat 20 --warmup 3 --quiet $v | grep "Total time" || exit 1
done; done; done
for v in "" "--no-overlap" "--transport push" "--transport push --no-overlap"; do
  echo "== N=2048 fake 3/8 $v"
  timeout -k 5 120 ./bin/wave3d 2048 0.00025 20 1 --fake-rank 3/8 --repeat 3 --warmup 1 --quiet $v | grep "Total time" || exit 1
done
