#!/bin/bash
# same-box interleaved A/B of two CLI builds on the 512^3 8-slab rank 1/8 (compute only, bench measure after
# 320 warmups) -> stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2 3; do
  for b in "$@"; do
    timeout -k 5 120 "$b" 512 0.001 20 1 --fake-rank 1/8 --decomp slab --no-overlap --repeat 5 --warmup 320 \
      --bench-steps 40 --quiet | grep -E "Bench" | sed "s|^|$r $b |" || exit 1
  done
done
