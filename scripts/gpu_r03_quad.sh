#!/bin/bash
# Round-3 A/B: canonical packed reveal with the four-product Montgomery reduction (default) vs one
# reduction per product pair (SDA_REVEAL_CANON_QUAD=0), interleaved, at 1000 and 64 vectors per launch;
# then the packed parity tests on the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03quad}
mkdir -p $T
out=$T/ab_reveal_quad.txt; : > $out
for r in 1 2 3; do
  for V in 1000 64; do
    for q in 1 0; do
      line=$(SDA_REVEAL_CANON_QUAD=$q timeout -k 10 120 python bench.py --only shamir --steps 10 --warmup 2 --no-check --shamir-vectors $V 2>&1 | grep '^\[shamir\]') || exit 1
      echo "round $r V=$V quad=$q $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("gen_ms","gen_canonical_ms","reveal_exact_ms","reveal_canonical_ms")))')" | tee -a $out
    done
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_device.py -k "packed or Packed or reveal" > $T/pytest_packed.txt 2>&1
rc=$?; tail -3 $T/pytest_packed.txt; exit $rc
