cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "chacha or mask or pipeline or stream or distributed" > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for leg in chacha pipelines; do timeout -k 10 200 python -u bench.py --only $leg --steps 20 > gpurun_out/b_$leg.log 2>&1 || exit $?; grep "^\[$leg\]" gpurun_out/b_$leg.log | cut -c1-600; done
