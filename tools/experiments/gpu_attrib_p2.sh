#!/bin/bash
# Perf attribution of the pair-tiled pass (k_leapfrog_p2) on one MI355X:
#   1. same-box A/B of the reference config (512^3, 20 steps) across the experiment builds in build/ab/
#      (noload / nostore / noload_nostore / nobarrier / nocheck — results wrong except nocheck's field) with kernel stats;
#   2. PMC passes on the production build, one counter group per run (HBM bytes, SQ waits/issue, LDS conflicts).
# Every GPU step runs under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
cd_repo=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
bins="./bin/wave3d ./build/ab/wave3d_nocheck ./build/ab/wave3d_noload ./build/ab/wave3d_nostore ./build/ab/wave3d_noload_nostore ./build/ab/wave3d_nobarrier"
bash scripts/gpu.sh abn $bins || exit 1
pmc() {  # name counters...
  local name=$1; shift
  rm -rf "gpurun_out/pmc_$name"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "gpurun_out/pmc_$name" -o run -- \
    ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 --quiet > "gpurun_out/pmc_$name.log" 2>&1 || return 1
  echo "== pmc $name done"
}
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
pmc lds SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq gpurun_out/pmc_lds \
  > gpurun_out/pmc_summary.md 2>&1
cat gpurun_out/pmc_summary.md
cd "$cd_repo"
