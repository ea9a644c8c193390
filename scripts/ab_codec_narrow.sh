#!/bin/bash
# A/B of the clerk's decode -> combine: int64 matrix (SDA_CODEC_NARROW=0) vs the int32 matrix with
# 2 or 4 columns per combine lane; interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_codec_narrow.txt; : > $out
for r in 1 2 3; do
  for v in "0 2" "1 2" "1 4"; do
    set -- $v
    line=$(SDA_CODEC_NARROW=$1 SDA_COMBINE32_VEC=$2 timeout -k 10 120 python bench.py --only codec --steps 10 2>&1 | grep '^\[codec\]') || exit 1
    echo "round $r narrow=$1 vec=$2 $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()[8:]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("decode_ms","decode_combine_ms","encode_ms")))')" | tee -a $out
  done
done
