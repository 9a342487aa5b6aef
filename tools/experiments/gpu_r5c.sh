#!/bin/bash
# Round 5 (c): cache-policy A/B of the pair-tiled pass, 3-D block ranks at S = 4 vs the 5-step pair-tiled passes
# (fake ranks, with their RCCL messages sent to themselves), 2048^3 on one GPU, then capture probe mode $PROBE_MODE
# last (it may crash on the host).
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh abn ./bin/wave3d ./build/ab/wave3d_store_aux_0 ./build/ab/wave3d_store_aux_16 \
  ./build/ab/wave3d_store_aux_18 ./build/ab/wave3d_load_aux_1 ./build/ab/wave3d_load_aux_2 || exit 1
out=gpurun_out/block_s5.log
: > "$out"
for fr in 512:0.001:3/8 2048:0.00025:3/8; do
  IFS=: read -r N tau r <<< "$fr"
  rep=24; [ "$N" = 2048 ] && rep=7
  for v in "--temporal 4 --no-overlap" "--temporal 5 --no-overlap" "--temporal 4 --no-overlap --fake-traffic" \
           "--temporal 5 --no-overlap --fake-traffic" "--temporal 4 --fake-traffic"; do
    echo "== N=$N $r 2x2x2 $v" >> "$out"
    timeout -k 5 240 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$r" --decomp 2x2x2 $v --repeat $rep --warmup 3 \
      --quiet --json gpurun_out/block_${N}_$(echo $v | tr -d ' -').json >> "$out" 2>&1 || exit 1
  done
done
grep -E "^==|Total time" "$out"
echo "== 2048^3 one GPU" >> "$out"
timeout -k 10 300 ./bin/wave3d 2048 0.00025 20 1 --repeat 3 --warmup 1 > gpurun_out/cli_2048.log 2>&1 || exit 1
tail -4 gpurun_out/cli_2048.log
if [ -n "${PROBE_MODE:-}" ]; then
  timeout -k 5 60 ./build/probes/capture_probe3 "$PROBE_MODE" 4 > gpurun_out/capture_probe3_m$PROBE_MODE.log 2>&1
  echo "probe mode $PROBE_MODE captured: exit $?"; tail -3 gpurun_out/capture_probe3_m$PROBE_MODE.log
fi
