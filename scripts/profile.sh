#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench, and separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) over a short combine-only run.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r01}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench_traced.json 2> $OUT/bench_traced.log || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --only combine --steps 3 --warmup 1 --no-check > $OUT/pmc_$c.log 2>&1 || exit $?
done

for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_snap_$c -o run -- \
      python3 bench.py --only snapshot --steps 4 --no-check > $OUT/pmc_snap_$c.log 2>&1 || exit $?
done
find $OUT -name "*.csv" | head -30
