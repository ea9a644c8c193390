#!/bin/bash
# microbench, parity tests, full bench, rocprof; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 60 ./tools/ubench_int > gpurun_out/ubench_int.txt 2>&1 || exit $?
cat gpurun_out/ubench_int.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || exit $?
cat gpurun_out/bench.json
if [ "$2" == "prof" ]; then bash scripts/profile.sh $TAG || exit $?; fi
exit $rc
