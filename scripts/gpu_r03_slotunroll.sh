#!/bin/bash
# Round-3 A/B (knob removed after it, profiles/r03t): the clerk's slot combine with 16 blobs' slot loads in flight per lane (SDA_SLOT_UNROLL=16)
# vs 8 (the default), interleaved, on the codec leg (1000 x 1M varint payloads); codec tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03t}
mkdir -p $T
SDA_SLOT_UNROLL=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_codec_fused.py \
  > $T/pytest_codec.txt 2>&1 || { tail -30 $T/pytest_codec.txt; exit 1; }
tail -2 $T/pytest_codec.txt
out=$T/ab_slot_unroll.txt; : > $out
for r in 1 2 3; do
  for u in 16 8; do
    line=$(SDA_SLOT_UNROLL=$u timeout -k 10 150 python bench.py --only codec --steps 10 --warmup 2 --no-check 2>&1 | grep '^\[codec\]') || exit 1
    echo "round $r unroll=$u $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("decode_combine_ms","decode_ms","encode_ms")))')" | tee -a $out
  done
done
