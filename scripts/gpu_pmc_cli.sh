#!/bin/bash
# PMC counters of the production 512³ K=20 solve (analytic start + checked 4-step passes), one pass per group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_cli
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/pmc_cli/$name -o run -- \
    ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 0 --quiet --no-graph > gpurun_out/pmc_cli/$name.log 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE &&
run p2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_COUNT &&
run p3 FETCH_SIZE TCC_HIT_sum &&
run p4 WRITE_SIZE TCC_MISS_sum
