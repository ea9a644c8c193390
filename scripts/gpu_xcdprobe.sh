#!/bin/bash
# XCD-order variants of share-gen's memory pattern in several fresh processes (allocation luck), then the
# real kernel's shamir leg in several processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-xcdprobe}
mkdir -p $T
for i in 1 2 3 4; do
  echo "-- process $i" >> $T/ubench.txt
  timeout -k 10 120 ./tools/ubench_gen 1000 3 quick >> $T/ubench.txt 2>&1 || { tail -5 $T/ubench.txt; exit 1; }
done
cat $T/ubench.txt
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --only shamir --no-cpu --steps 10 2>&1 >/dev/null | grep "^\[shamir\]" | grep -o '"gen_ms": [0-9.]*\|"gen_canonical_ms": [0-9.]*\|"reveal_canonical_ms": [0-9.]*' | tr '\n' ' ' >> $T/shamir.txt || exit 1
  echo >> $T/shamir.txt
done
cat $T/shamir.txt
