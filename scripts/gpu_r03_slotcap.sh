#!/bin/bash
# Dense slot stride (4096 slots per 16 KiB region): codec GPU tests, then the codec leg 3 times and a trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03cap}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_codec_fused.py tests/test_gpu_pipelines.py -x -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for r in 1 2 3; do
  l=$(timeout -k 10 180 python -u bench.py --only codec --steps 10 2>&1 | grep '^\[codec\]') || exit 1
  echo "round $r $(echo "$l" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("decode_ms","decode_combine_ms","decode_combine_matrix_ms")))')" | tee -a $T/ab_slotcap.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --only codec --steps 5 --warmup 1 > $T/trace.log 2>&1 || { tail -5 $T/trace.log; exit 1; }
python3 scripts/stats_by_grid.py $T/trace/run_kernel_trace.csv > $T/stats_by_grid.csv
grep -E "varint|slot|combine" $T/stats_by_grid.csv | cut -c1-160
