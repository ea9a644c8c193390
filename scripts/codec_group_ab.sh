#!/bin/bash
# A/B of the clerk's decode -> combine: one pass vs grouped (SDA_CODEC_GROUP=G blobs per group), interleaved over
# <rounds>; prints each run's codec leg decode_combine_ms.  (Round 6 also timed an overlapped grouped build --
# the next group's decode on an auxiliary stream -- with this script's o<G> variants; that build was removed,
# DESIGN.md §4.5, profiles/r06f, r06g.)
#   bash scripts/codec_group_ab.sh <rounds> <G> [<G> ...]      (run from gpu_steps.sh "sh:" or directly)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=${1:-2}
GS=${*:2}
GS=${GS:-"10 20 40"}
for r in $(seq "$ROUNDS"); do
  for v in base $GS; do
    g=0
    [ "$v" != base ] && g=$v
    ms=$(env SDA_CODEC_GROUP=$g timeout -k 10 300 python3 -u bench.py --only codec --steps 5 --warmup 1 --no-cpu --no-host-path \
         2>&1 >/dev/null | grep '^\[codec\]' \
         | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(round(d["decode_combine_ms"],4))') \
      || { echo "run $v failed"; exit 1; }
    echo "round $r $v decode_combine_ms $ms"
  done
done
