#!/bin/bash
# Trace stats + SQ/HBM counter passes of the packed-Shamir leg alone, then the per-kernel report.
#   bash scripts/gpu_shamir_prof.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-shamir}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --only shamir --steps 20 --warmup 3 --no-check > $OUT/trace.log 2>&1 || exit $?
bash scripts/pmc_shamir.sh $TAG --only shamir --steps 3 --warmup 1 || exit $?
python3 scripts/kernel_report.py $OUT/trace gpurun_out/pmc_$TAG > $OUT/kernel_report.json
