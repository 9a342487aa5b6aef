#!/bin/bash
# per-workgroup timelines of the pair-tiled passes (build/ab/wave3d_wgtime: W3D_EXTRA_DEFS_P2=-DW3D_EXPERIMENT_WGTIME)
# for one GPU and 512^3 slab ranks 1/8, 1/4 -> gpurun_out/wgtime/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/wgtime
for spec in "1x:" "s8:--fake-rank 1/8 --decomp slab --no-overlap" "s4:--fake-rank 1/4 --decomp slab --no-overlap"; do
  n=${spec%%:*}; a=${spec#*:}
  W3D_WGTIME_OUT=gpurun_out/wgtime/$n.txt timeout -k 10 120 build/ab/wave3d_wgtime 512 0.001 20 1 $a --repeat 5 \
    --warmup 2 --bench-steps 10 --quiet | grep -E "Total time|Bench" || exit 1
done
python3 tools/experiments/wgtime_report.py gpurun_out/wgtime/1x.txt gpurun_out/wgtime/s8.txt gpurun_out/wgtime/s4.txt
