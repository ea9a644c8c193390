#!/bin/bash
# Round 2, first GPU pass: int microbench, the whole -m gpu suite, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket" >> gpurun_out/host.txt
timeout -k 10 60 ./tools/ubench_int > gpurun_out/ubench_int.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || exit $?
cat gpurun_out/bench.json
exit $rc
