#!/bin/bash
# Trace stats + SQ/HBM counter passes of the codec leg alone, then the per-kernel report.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-codec}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --only codec --steps 10 --warmup 2 > $OUT/trace.log 2>&1 || exit $?
bash scripts/pmc_shamir.sh $TAG --only codec --steps 3 --warmup 1 || exit $?
python3 scripts/kernel_report.py $OUT/trace gpurun_out/pmc_$TAG > $OUT/kernel_report.json
