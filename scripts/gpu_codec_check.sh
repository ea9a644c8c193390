#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "codec or varint or decode or snapshot or pipeline or full_loop" > gpurun_out/pytest_q.log 2>&1 || { tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for leg in codec chacha pipelines; do timeout -k 10 200 python -u bench.py --only $leg --steps 20 > gpurun_out/b_$leg.log 2>&1 || { tail -20 gpurun_out/b_$leg.log; exit 1; }; grep "^\[$leg\]" gpurun_out/b_$leg.log | cut -c1-700; done
