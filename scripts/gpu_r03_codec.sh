#!/bin/bash
# Round-3 codec session: the codec GPU tests (all three decode -> combine paths), then the codec leg of
# bench.py three times (default slot path, with the matrix and fused paths timed beside it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03codec}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_codec_fused.py tests/test_gpu_pipelines.py tests/test_snapshot.py -x -q --timeout 170 --timeout-method thread > $T/pytest_codec.log 2>&1 || { tail -30 $T/pytest_codec.log; exit 1; }
tail -2 $T/pytest_codec.log
for r in 1 2 3; do
  timeout -k 10 180 python -u bench.py --only codec --steps 10 2>&1 | grep '^\[codec\]' | tee -a $T/codec_legs.txt || exit 1
done
