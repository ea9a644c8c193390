#!/bin/bash
# Round-3 A/B: exact reveal with whole-row table loads (SDA_REVEAL_ROWS=1, default) vs the split per-word
# scalar loads (build/prev/libsda_engine_prev.so, built with EXTRA=-DSDA_REVEAL_ROWS=0), interleaved, at
# 1000 and 64 vectors per launch; packed parity tests on the default first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03r}
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_device.py \
  -k "packed or Packed or reveal" > $T/pytest_packed.txt 2>&1 || { tail -30 $T/pytest_packed.txt; exit 1; }
tail -2 $T/pytest_packed.txt
out=$T/ab_reveal_rows.txt; : > $out
for r in 1 2 3; do
  for V in 1000 64; do
    for lib in new prev; do
      L=""; [ $lib = prev ] && L=build/prev/libsda_engine_prev.so
      line=$(SDA_ENGINE_LIB=$L timeout -k 10 120 python bench.py --only shamir --steps 10 --warmup 2 --no-check --shamir-vectors $V 2>&1 | grep '^\[shamir\]') || exit 1
      echo "round $r V=$V lib=$lib $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("reveal_exact_ms","reveal_canonical_ms","gen_ms")))')" | tee -a $out
    done
  done
done
