#!/bin/bash
# A/B of the scalar edge branch (build/ab/wave3d_edgeall: Dirichlet selects in every tile), vector-memory / LDS
# latency counters of the production pass, then the GPU test suite.
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh abn ./build/ab/wave3d_edgeall ./bin/wave3d || exit 1
pmc() {  # name counters...
  local name=$1; shift
  rm -rf "gpurun_out/pmc_$name"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "gpurun_out/pmc_$name" -o run -- \
    ./bin/wave3d 512 0.001 20 1 --repeat 2 --warmup 1 --quiet > "gpurun_out/pmc_$name.log" 2>&1 || return 1
}
pmc lat SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VMEM_WR_TA_DATA_FIFO_FULL \
  SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_DATA_FIFO_FULL || exit 1
pmc cyc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_ADDR_CONFLICT \
  SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_UNALIGNED_STALL || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_lat gpurun_out/pmc_cyc | grep -v "__amd" > gpurun_out/pmc_lat.md
grep "k_leapfrog_p2<5, 21" gpurun_out/pmc_lat.md
bash scripts/gpu.sh test || exit 1
# capture-topology probe: safe topologies first; the round-4 split (mode 2) last, it may crash the
# runtime on the host (the script ends there either way)
p=./build/probes/capture_probe3
for m in 0 1 3 4; do timeout -k 5 60 $p $m 4 > gpurun_out/capture_probe3_m$m.log 2>&1 || { cat gpurun_out/capture_probe3_m$m.log; exit 1; }; cat gpurun_out/capture_probe3_m$m.log | tail -1; done
timeout -k 5 60 $p 2 4 1 > gpurun_out/capture_probe3_m2_eager.log 2>&1 || exit 1
tail -1 gpurun_out/capture_probe3_m2_eager.log
timeout -k 5 60 $p 2 4 > gpurun_out/capture_probe3_m2.log 2>&1
echo "mode 2 captured: exit $?"; tail -3 gpurun_out/capture_probe3_m2.log
