#!/bin/bash
# r02d evidence (final code of round 2): host, int-op microbench, the -m gpu suite, the default bench
# line, rocprofv3 kernel-trace stats of the bench.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02d_ev; mkdir -p $O
(nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket") > $O/host.txt
timeout -k 10 60 ./tools/ubench_int > $O/ubench_int.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_traced.json 2> $O/bench_traced.log || exit $?
echo done
