#!/bin/bash
# Interleaved A/B of engine libraries on one box: one bench.py leg per library per round.
#   bash scripts/ab_libs.sh <leg> <rounds> lib1.so lib2.so ...     (leg: shamir | chacha | codec | ...)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LEG=$1; R=$2; shift 2
out=gpurun_out/ab_$LEG.txt; : > $out
for r in $(seq 1 $R); do
  for lib in "$@"; do
    line=$(SDA_ENGINE_LIB=$lib timeout -k 10 120 python bench.py --only $LEG --steps 20 --no-check 2>&1 | grep "^\[$LEG\]") || exit 1
    echo "round $r $lib ${line:0:900}" >> $out
    echo "round $r $lib $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,v) for k,v in d.items() if k.endswith("_ms") or k=="ms"))')"
  done
done
