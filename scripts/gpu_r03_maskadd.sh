#!/bin/bash
# Round-3: the participant's one-stream ChaCha mask add as its own kernel (secrets prefetched under the
# ChaCha rounds).  Parity tests of every ChaCha / pipeline path, then the pipelines leg under the kernel
# tracer (compare with profiles/r03o/ before the change).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03p}
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chacha_rejects.py \
  tests/test_gpu_pipelines.py tests/test_gpu_streams.py tests/test_gpu_parity.py -k "chacha or mask or Chacha or pipeline or participant or recipient or stream" \
  > $T/pytest_chacha.txt 2>&1 || { tail -30 $T/pytest_chacha.txt; exit 1; }
tail -2 $T/pytest_chacha.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
  python3 bench.py --only pipelines --steps 5 --warmup 2 --no-check > $T/pipelines.log 2>&1 || { tail -5 $T/pipelines.log; exit 1; }
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --only pipelines --steps 10 --warmup 2 --no-check 2>&1 | grep '^\[pipelines\]' >> $T/pipelines_runs.txt || exit 1
done
cat $T/pipelines_runs.txt
