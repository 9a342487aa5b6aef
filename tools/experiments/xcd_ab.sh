#!/bin/bash
# XCD tile mapping A/B at 512³: two-row strips per XCD (default) vs square-ish blocks (W3D_TB_XCDBLOCKS=1):
# solve time interleaved, then rocprof FETCH_SIZE per 4-step pass for each (the pass is bound by its actual DRAM bytes).
mkdir -p gpurun_out/xcd
for r in 1 2 3; do
  for v in 0 1; do
    W3D_TB_XCDBLOCKS=$v timeout -k 5 60 ./bin/wave3d 512 0.001 20 1 --repeat 20 --warmup 3 --quiet | grep "Total time" | sed "s/^/xcdblocks=$v r=$r /" || exit 1
  done
done
for v in 0 1; do
  W3D_TB_XCDBLOCKS=$v timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
    -d gpurun_out/xcd/f$v -o run -- ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 --quiet > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for v in (0, 1):
    f = glob.glob(f"gpurun_out/xcd/f{v}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "leapfrog" in r["Kernel_Name"]:
            agg[r["Kernel_Name"].split("(")[0][-45:]].append(float(r["Counter_Value"]))
    for k, vals in agg.items():
        print(f"xcdblocks={v}", k, "FETCH_SIZE per dispatch (KB, rocprof units) mean", round(sum(vals) / len(vals)))
PY
