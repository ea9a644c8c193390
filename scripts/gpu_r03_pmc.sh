#!/bin/bash
# Round-3 counters: the SQ / HBM passes of the packed-Shamir + ChaCha legs at the bench configuration
# (1000 vectors per launch), the combine's FETCH_SIZE / WRITE_SIZE passes, and the integer issue
# microbenchmark.  One counter group per rocprofv3 run (MI355X_MICROARCH.md); stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03pmc}
mkdir -p $T
timeout -k 10 60 ./tools/ubench_int > $T/ubench_int.txt 2>&1 || exit $?
bash scripts/pmc_shamir.sh ${1:-r03pmc}_shamir --only shamir --steps 3 --warmup 1 > $T/pmc_shamir.txt 2>&1 || { tail -5 $T/pmc_shamir.txt; exit 1; }
bash scripts/pmc_shamir.sh ${1:-r03pmc}_chacha --only chacha --steps 3 --warmup 1 > $T/pmc_chacha.txt 2>&1 || { tail -5 $T/pmc_chacha.txt; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $T/combine_p$i -o run -- python3 bench.py --only combine --steps 3 --warmup 1 > $T/combine_p$i.log 2>&1 || { echo "combine pass $i failed"; tail -5 $T/combine_p$i.log; exit 1; }
done
(python3 scripts/summarize_pmc.py $T/combine_p1; python3 scripts/summarize_pmc.py $T/combine_p2) > $T/pmc_combine.txt 2>&1
echo pmc done
