#!/bin/bash
# bench.py with its resident buffers from sda_hbm_alloc vs torch.empty (SDA_BENCH_ALLOC=torch), alternating
# processes; hbm:<MiB> sets the chunk size (SDA_HBM_CHUNK_MB).  Output: gpurun_out/<tag>/allocab.txt.
#   bash scripts/gpu_allocab.sh <tag> "<bench args>" <rounds> [modes, default "hbm torch"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-allocab}
ARGS=${2:-"--only shamir"}
ROUNDS=${3:-3}
MODES=${4:-"hbm torch"}
mkdir -p $T
for i in $(seq $ROUNDS); do
  for a in $MODES; do
    echo "-- round $i alloc=$a" >> $T/allocab.txt
    kind=${a%%:*}
    mb=64
    [[ "$a" == *:* ]] && mb=${a#*:}
    # shellcheck disable=SC2086
    SDA_BENCH_ALLOC=$kind SDA_HBM_CHUNK_MB=$mb timeout -k 10 600 python -u bench.py $ARGS 2>&1 >/dev/null \
      | grep "^\[" | cut -c1-400 >> $T/allocab.txt || exit 1
  done
done
cat $T/allocab.txt
