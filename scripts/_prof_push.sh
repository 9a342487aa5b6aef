set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in rccl push; do
  rm -rf gpurun_out/pp_$v
  extra=""; [ $v = push ] && extra="--transport push"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_$v -o run -- ./bin/wave3d 512 0.001 20 1 --fake-rank 1/8 --no-overlap --repeat 5 --warmup 1 --quiet $extra > gpurun_out/pp_$v.log 2>&1 || exit 1
done
