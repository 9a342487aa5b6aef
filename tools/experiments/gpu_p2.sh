#!/bin/bash
# Round-5 first contact for the pair-tiled pass: kernel bit-exactness tests, the 512³ golden log, the bench, and a
# kernel-trace profile. Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
out=gpurun_out/p2
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "p2 or leapfrog_tb" > $out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_kernels.log; exit 1; }
tail -3 $out/pytest_kernels.log
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --timers > $out/cli.log 2>&1 || { echo "cli failed"; cat $out/cli.log; exit 1; }
cat $out/cli.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -2 $out/bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- ./bin/wave3d 512 0.001 20 1 --bench-steps 10 > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -8 $out/kernel_stats.csv
