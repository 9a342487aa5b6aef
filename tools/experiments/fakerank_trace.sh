set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for spec in "1x:0/1" "s8:1/8" "s4:1/4" "s2:1/2"; do
  n=${spec%%:*}; r=${spec#*:}
  if [ "$r" = "0/1" ]; then a=""; else a="--fake-rank $r --decomp slab --no-overlap"; fi
  timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 $a --repeat 20 --warmup 2 --quiet | grep "Total time" || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fr/$n -o run -- ./bin/wave3d 512 0.001 20 1 $a --repeat 12 --warmup 2 --quiet > /dev/null 2>&1 || exit 1
done
python3 tools/experiments/trace_seq.py gpurun_out/fr/1x gpurun_out/fr/s8 gpurun_out/fr/s4 gpurun_out/fr/s2
