#!/bin/bash
# One rocprofv3 PMC pass (counters in $1) over `python3 bench.py $2`, then a per-kernel summary.
#   bash scripts/pmc_pass.sh "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "--only shamir --steps 5 --warmup 1" tag
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${3:-x}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d $OUT -o run -- python3 bench.py $2 > $OUT/run.log 2>&1 || exit $?
python3 scripts/summarize_pmc.py $OUT
