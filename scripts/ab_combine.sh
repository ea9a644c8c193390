#!/bin/bash
# Interleaved A/B of the headline combine: bench.py --only combine per library, R rounds.
#   bash scripts/ab_combine.sh <rounds> lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
out=gpurun_out/ab_combine.txt; : > $out
for r in $(seq 1 $R); do
  for lib in "$@"; do
    line=$(SDA_ENGINE_LIB=$lib timeout -k 10 120 python bench.py --only combine --steps 20 --warmup 3 --no-check 2>&1 | grep "^\[combine\]") || exit 1
    echo "round $r $lib $line" | tee -a $out
  done
done
