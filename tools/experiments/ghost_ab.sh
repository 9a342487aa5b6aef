#!/bin/bash
# Slab ranks with and without the u^{n+S-1} ghost-plane store (--no-ghost-store), interleaved: one fake rank timed
# alone with its real copy-engine transfers (sdma) or its RCCL messages sent to itself (--fake-traffic); prints the
# CLI's best-of time and the Traffic line (halo MB per solve) -> stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2 3; do
  for fr in 512:0.001:1/8 512:0.001:1/4 512:0.001:0/2; do
    IFS=: read -r N tau k <<< "$fr"
    for v in "--transport sdma" "--transport sdma --no-overlap" "--fake-traffic --no-overlap" "--fake-traffic"; do
      for g in "" "--no-ghost-store"; do
        echo "== round $r N=$N fake $k slab $v $g"
        timeout -k 5 120 ./bin/wave3d "$N" "$tau" 20 1 --fake-rank "$k" --decomp slab --repeat 10 --warmup 2 \
          $v $g | grep -E "Total time|Traffic" || exit 1
      done
    done
  done
done
