#!/bin/bash
# Round-3 GPU session: host model, the whole -m gpu suite, the default bench line (with the CPU
# baseline), then the same bench under rocprofv3 --kernel-trace --stats.  Stops at the first failure.
#   bash scripts/gpu_r03.sh [tag]      -> gpurun_out/<tag>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03}
mkdir -p $T
(nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS") > $T/host.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1
rc=$?
tail -5 $T/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $T/bench.json 2> $T/bench.log || { tail -20 $T/bench.log; exit 1; }
cut -c1-1200 $T/bench.json
grep -v amdgpu.ids $T/bench.log | tail -12
[ -n "$NO_TRACE" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > $T/bench_traced.json 2> $T/bench_traced.log || { tail -5 $T/bench_traced.log; exit 1; }
echo traced
