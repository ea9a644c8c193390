#!/bin/bash
# Speculative ChaCha rejection check in the pipelines + device-side encode row bases: the affected GPU
# tests, then the pipelines and codec legs of the bench, and a kernel trace of the pipelines leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03spec}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_gpu_chacha_rejects.py tests/test_gpu_pipelines.py tests/test_gpu_codec.py tests/test_gpu_streams.py tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for r in 1 2 3; do
  timeout -k 10 180 python -u bench.py --only pipelines --steps 10 2>&1 | grep '^\[pipelines\]' | tee -a $T/pipelines.txt || exit 1
  timeout -k 10 180 python -u bench.py --only codec --steps 10 2>&1 | grep '^\[codec\]' | cut -c1-400 | tee -a $T/codec.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --only pipelines --steps 5 --warmup 1 > $T/trace.log 2>&1 || { tail -5 $T/trace.log; exit 1; }
echo traced
