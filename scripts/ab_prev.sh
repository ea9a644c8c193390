#!/bin/bash
# A/B of the packed-Shamir kernels: the previous commit's library (build/ab_prev) vs the current one,
# interleaved, 3 rounds; prints gen/reveal ms per run.  Usage: scripts/ab_prev.sh [out-name]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${1:-ab_prev}.txt; : > $out
for r in 1 2 3; do
  for v in prev cur; do
    lib=""; [ "$v" == prev ] && lib=build/ab_prev/libsda_engine.so
    line=$(SDA_ENGINE_LIB=$lib timeout -k 10 120 python bench.py --only shamir --steps 20 --no-check 2>&1 | grep '^\[shamir\]') || exit 1
    echo "round $r $v $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()[9:]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("gen_ms","gen_canonical_ms","reveal_exact_ms","reveal_canonical_ms")))')" | tee -a $out
  done
done
