#!/bin/bash
# Round-3 A/B: exact share-gen with the sign-bit radix-2 half (default) vs the mad_i64 sign kernel
# (SDA_GEN_SIGNBIT=0), interleaved, at 1000 and at 64 vectors per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03ab}
mkdir -p $T
out=$T/ab_gen_signbit.txt; : > $out
for r in 1 2 3; do
  for V in 1000 64; do
    for sb in 1 0; do
      line=$(SDA_GEN_SIGNBIT=$sb timeout -k 10 120 python bench.py --only shamir --steps 10 --warmup 2 --no-check --shamir-vectors $V 2>&1 | grep '^\[shamir\]') || exit 1
      echo "round $r V=$V signbit=$sb $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("gen_ms","gen_canonical_ms","reveal_exact_ms","reveal_canonical_ms")))')" | tee -a $out
    done
  done
done


