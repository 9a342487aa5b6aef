#!/bin/bash
# Kernel-trace profile of the reference-config solve (CLI) -> gpurun_out/prof/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- ./bin/wave3d 512 0.001 20 1 --repeat 5 --warmup 1 ${W3D_ARGS:-} > gpurun_out/prof.log 2>&1
