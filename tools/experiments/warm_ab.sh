#!/bin/bash
# bench.py's timed block: (a) one host round trip per solve (W3D_BENCH_SYNC_EACH=1) against run_batch (all K replays
# enqueued, one sync), (b) the driver's 5 warmups against 40 (clock/power settling), interleaved, fresh process each;
# plus one CLI per-solve curve (60 solves, no warmup).
mkdir -p gpurun_out/warm
timeout -k 10 120 ./bin/wave3d 512 0.001 20 1 --repeat 60 --warmup 0 --quiet --json gpurun_out/warm/curve.json \
  > gpurun_out/warm/curve.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in sync5 batch5 batch40; do
    w=${v#sync}; w=${w#batch}
    if [ "${v#sync}" != "$v" ]; then export W3D_BENCH_SYNC_EACH=1; else unset W3D_BENCH_SYNC_EACH; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup $w > gpurun_out/warm/b_${v}_r$r.log 2>&1 || exit 1
    echo "$v r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/warm/b_${v}_r$r.log)"
  done
done
