set -o pipefail
mkdir -p gpurun_out/r04c
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "test_packed_random_schemes or test_packed_wide_random" > gpurun_out/r04c/diag.log 2>&1
rc=$?
tail -n 30 gpurun_out/r04c/diag.log
exit $rc
