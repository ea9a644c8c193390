#!/bin/bash
# Round-3: ChaCha combine with round 1's uniform columns precomputed per seed and a branch-light draw loop.
# Parity tests of every ChaCha / pipeline path on the new library, then an interleaved A/B against the
# previous chacha.o (build/prev/libsda_engine_prev.so: the previous commit's chacha.hip compiled and linked
# with the other current objects, plus a two-line shim for the old chacha_work_bytes(D) signature): the
# chacha leg (256 seeds x 1M) and the recipient pipeline (256 seeds x 10M + reveal).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-r03q}
mkdir -p $T
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chacha_rejects.py \
  tests/test_gpu_pipelines.py tests/test_gpu_streams.py tests/test_gpu_parity.py tests/test_gpu_multirank.py \
  -k "chacha or mask or Chacha or pipeline or participant or recipient or stream or sharded" \
  > $T/pytest_chacha.txt 2>&1 || { tail -30 $T/pytest_chacha.txt; exit 1; }
tail -2 $T/pytest_chacha.txt
out=$T/ab_chacha_pre.txt; : > $out
for r in 1 2 3; do
  for lib in new prev; do
    L=""; [ $lib = prev ] && L=build/prev/libsda_engine_prev.so
    c=$(SDA_ENGINE_LIB=$L timeout -k 10 120 python bench.py --only chacha --steps 10 --warmup 2 --no-check 2>&1 | grep '^\[chacha\]') || exit 1
    p=$(SDA_ENGINE_LIB=$L timeout -k 10 120 python bench.py --only pipelines --steps 5 --warmup 1 --no-check 2>&1 | grep '^\[pipelines\]') || exit 1
    echo "round $r lib=$lib chacha_ms=$(echo "$c" | python3 -c 'import sys,json; print("%.4f" % json.loads(sys.stdin.read().split(" ",1)[1])["ms"])') recipient_ms=$(echo "$p" | python3 -c 'import sys,json; print("%.4f" % json.loads(sys.stdin.read().split(" ",1)[1])["recipient_ms"])')" | tee -a $out
  done
done
