#!/bin/bash
# configs[3] evidence: the 100k x 10M clerk job streamed through a resident 1000-row tile on one GPU
# (bench --config 3), its rocprofv3 kernel-trace stats and its HBM traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/config3
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --no-side > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --config 3 --steps 2 --warmup 0 --no-side --no-cpu > $OUT/bench_traced.json 2> $OUT/bench_traced.log || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --config 3 --steps 1 --warmup 0 --no-side --no-cpu --no-check > $OUT/pmc_$c.log 2>&1 || exit $?
done
echo done
