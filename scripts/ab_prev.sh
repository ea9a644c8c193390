#!/bin/bash
# A/B of one bench leg: the previous commit's library (build/ab_prev) vs the current one, interleaved,
# 3 rounds.   Usage: scripts/ab_prev.sh [out-name] [leg] [keys...]
#   default: shamir leg, gen/reveal ms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=${1:-ab_prev}; leg=${2:-shamir}; shift 2 2>/dev/null
keys=${@:-"gen_ms gen_canonical_ms reveal_exact_ms reveal_canonical_ms"}
out=gpurun_out/$name.txt; : > $out
for r in 1 2 3; do
  for v in prev cur; do
    lib=""; [ "$v" == prev ] && lib=build/ab_prev/libsda_engine.so
    line=$(SDA_ENGINE_LIB=$lib timeout -k 10 120 python bench.py --only $leg --steps 10 --no-check 2>&1 | grep "^\[$leg\]") || exit 1
    echo "round $r $v $(echo "$line" | KEYS="$keys" python3 -c 'import os,sys,json; s=sys.stdin.read(); d=json.loads(s[s.index("{"):]); print(" ".join("%s=%.4f"%(k,d[k]) for k in os.environ["KEYS"].split()))')" | tee -a $out
  done
done
