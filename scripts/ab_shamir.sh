#!/bin/bash
# A/B of the packed-Shamir kernels: the round-1 library (build/ab_r01) vs the current one,
# interleaved, 3 rounds; prints gen/reveal ms per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_shamir.txt; : > $out
for r in 1 2 3; do
  for v in r01 cur; do
    lib=""; [ "$v" == r01 ] && lib=build/ab_r01/libsda_engine.so
    line=$(SDA_ENGINE_LIB=$lib timeout -k 10 120 python bench.py --only shamir --steps 20 --no-check 2>&1 | grep '^\[shamir\]') || exit 1
    echo "round $r $v $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()[9:]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("gen_ms","gen_canonical_ms","reveal_exact_ms","reveal_canonical_ms")))')" | tee -a $out
  done
done
