#!/bin/bash
# tests + integer microbenchmark + Shamir leg; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_int > gpurun_out/ubench_int.txt 2>&1 || exit $?
cat gpurun_out/ubench_int.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --only shamir --steps 10 --warmup 2 > gpurun_out/bench_shamir.log 2>&1
echo "bench exit $?"; grep shamir gpurun_out/bench_shamir.log
exit $rc
