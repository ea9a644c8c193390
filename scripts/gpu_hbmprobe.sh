#!/bin/bash
# sda_hbm_alloc on the GPU: hbm_check.py, then share-gen placement with torch vs hbm buffers, alternating
# processes (gen_placement.py).  Output: gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-hbmprobe}
mkdir -p $T
timeout -k 10 200 python -u scripts/hbm_check.py > $T/hbm_check.txt 2>&1 || { cat $T/hbm_check.txt; exit 1; }
cat $T/hbm_check.txt
for i in 1 2 3; do
  for mode in torch hbm; do
    echo "== process $i $mode" >> $T/placement.txt
    timeout -k 10 200 python -u scripts/gen_placement.py 4 $mode 2>&1 | grep -v amdgpu.ids >> $T/placement.txt || exit 1
  done
done
cat $T/placement.txt
