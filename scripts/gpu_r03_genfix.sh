#!/bin/bash
# Wave-per-batch share-gen fix-up: the packed / pipeline GPU tests, then the shamir leg at 1000 and 64
# vectors per launch and the pipelines leg (3 rounds each), and a kernel trace of the shamir leg at 64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03genfix}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device.py tests/test_gpu_pipelines.py tests/test_gpu_chacha_rejects.py tests/test_gpu_configs.py tests/test_gpu_config4.py -x -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for r in 1 2 3; do
  for V in 1000 64; do
    l=$(timeout -k 10 120 python bench.py --only shamir --steps 10 --warmup 2 --no-check --shamir-vectors $V 2>&1 | grep '^\[shamir\]') || exit 1
    echo "round $r V=$V $(echo "$l" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print(" ".join("%s=%.4f"%(k,d[k]) for k in ("gen_ms","gen_canonical_ms","reveal_exact_ms","reveal_canonical_ms")))')" | tee -a $T/ab_shamir.txt
  done
  timeout -k 10 180 python -u bench.py --only pipelines --steps 10 2>&1 | grep '^\[pipelines\]' | tee -a $T/pipelines.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --only shamir --steps 5 --warmup 1 --no-check --shamir-vectors 64 > $T/trace.log 2>&1 || { tail -5 $T/trace.log; exit 1; }
python3 scripts/stats_by_grid.py $T/trace/run_kernel_trace.csv > $T/stats_by_grid.csv
grep -E "packed|fixup" $T/stats_by_grid.csv | cut -c1-160
