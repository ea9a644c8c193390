#!/bin/bash
# Round-3 evidence on the final code: host model, the whole -m gpu suite, smoke(), the default bench
# line (with the CPU baselines), the bench under rocprofv3 --kernel-trace --stats, the combine's HBM
# traffic passes (FETCH_SIZE, WRITE_SIZE) and the SQ passes over the packed-Shamir + ChaCha legs.
# One counter group per rocprofv3 run; stops at the first failure.
#   bash scripts/gpu_r03_final.sh [tag]      -> gpurun_out/<tag>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03e}
T=gpurun_out/$TAG
mkdir -p $T
(nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS") > $T/host.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -1 $T/smoke.log
timeout -k 10 600 python -u bench.py > $T/bench.json 2> $T/bench.log || { tail -20 $T/bench.log; exit 1; }
cut -c1-600 $T/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > $T/bench_traced.json 2> $T/bench_traced.log || { tail -5 $T/bench_traced.log; exit 1; }
python3 scripts/stats_by_grid.py $T/trace/run_kernel_trace.csv > $T/kernel_stats_by_grid.csv || exit 1
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $T/combine_p$i -o run -- python3 bench.py --only combine --steps 3 --warmup 1 > $T/combine_p$i.log 2>&1 || { echo "combine pass $i failed"; tail -5 $T/combine_p$i.log; exit 1; }
done
(python3 scripts/summarize_pmc.py $T/combine_p1; python3 scripts/summarize_pmc.py $T/combine_p2) > $T/pmc_combine.txt 2>&1
cat $T/pmc_combine.txt
bash scripts/pmc_shamir.sh ${TAG}_shamir --only shamir --steps 3 --warmup 1 > $T/pmc_shamir.txt 2>&1 || { tail -5 $T/pmc_shamir.txt; exit 1; }
bash scripts/pmc_shamir.sh ${TAG}_chacha --only chacha --steps 3 --warmup 1 > $T/pmc_chacha.txt 2>&1 || { tail -5 $T/pmc_chacha.txt; exit 1; }
echo evidence done
