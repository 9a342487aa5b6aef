#!/bin/bash
# Interior/halo overlap at 512^3 on one MI355X: fake slab / block ranks with their real halo traffic —
# RCCL to themselves (--fake-traffic) or the copy engines into their own ghosts (--transport sdma) — sequential vs
# overlapped; 28 solves after 8 warmups (the copy-engine runs' first replays are slow), best / mean from --json.
set -u
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out/p7
export TMPDIR=/tmp
out=gpurun_out/p7.log
: > "$out"
for rd in 0/2:slab 1/4:slab 1/8:slab 3/8:2x2x2; do
  IFS=: read -r r d <<< "$rd"
  for v in "--no-overlap" "--no-overlap --fake-traffic" "--fake-traffic" "--no-overlap --transport sdma" \
           "--transport sdma"; do
    tag=$(echo "$r-$d$v" | tr -d ' /-')
    echo "== 512 $r $d $v" >> "$out"
    timeout -k 5 150 ./bin/wave3d 512 0.001 20 1 --fake-rank "$r" --decomp "$d" $v --repeat 28 --warmup 8 --quiet \
      --json "gpurun_out/p7/$tag.json" >> "$out" 2>&1 || exit 1
  done
done
grep -E "^==|Total time" "$out"
