#!/bin/bash
# Clerk decode -> combine with its one wait at the end: the whole -m gpu suite, then the codec leg
# (3 rounds) and a kernel trace of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03nowait}
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for r in 1 2 3; do
  timeout -k 10 180 python -u bench.py --only codec --steps 10 2>&1 | grep '^\[codec\]' | cut -c1-700 | tee -a $T/codec.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --only codec --steps 5 --warmup 1 > $T/trace.log 2>&1 || { tail -5 $T/trace.log; exit 1; }
python3 scripts/stats_by_grid.py $T/trace/run_kernel_trace.csv > $T/stats_by_grid.csv
grep -E "slot|decode_kernel|scan|count|cap_kernel|sequential" $T/stats_by_grid.csv | cut -c1-160
