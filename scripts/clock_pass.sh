#!/bin/bash
# Per-dispatch shader clock of one bench leg: one rocprofv3 run with GRBM_GUI_ACTIVE + kernel trace
# (counters and trace in the same run are allowed; no runtime/sys trace), then cycles / duration.
#   bash scripts/clock_pass.sh <tag> <bench args>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-clk}; shift
OUT=gpurun_out/clock_$TAG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace --output-format csv -d $OUT -o run -- \
    python3 bench.py "$@" > $OUT/bench.log 2>&1 || { echo "clock pass failed rc=$?"; tail -5 $OUT/bench.log; exit 1; }
find $OUT -name "*.csv" | head
