#!/bin/bash
# GPU-box step runner: parity tests, then a short bench.  Stops at the first crash/timeout
# (exit >= 124 or a signal); plain test failures (exit 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.log
brc=$?
echo "bench exit $brc"
cat gpurun_out/bench.json
tail -5 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
