#!/bin/bash
# GPU-box quick loop: parity tests (optionally filtered with -k), then one bench leg.
#   bash scripts/gpu_quick.sh "<pytest -k expr>" "<bench.py args>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
fi
rc=$?
tail -4 gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  timeout -k 10 300 python -u bench.py $2 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.log || exit $?
  cat gpurun_out/bench_quick.json; grep -v amdgpu.ids gpurun_out/bench_quick.log | tail -5
fi
