#!/bin/bash
# Round-3 refresh of the two 100k x 10M configs on the final code: configs[3] (bench --config 3, the clerk
# job through a resident 1000-row tile) and configs[4] (bench --config 4, recipient side, 100k seeds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03cfg}
mkdir -p $T
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --no-side > $T/config3.json 2> $T/config3.log || { tail -5 $T/config3.log; exit 1; }
cut -c1-400 $T/config3.json
timeout -k 10 400 python -u bench.py --config 4 --steps 3 --warmup 1 > $T/config4.json 2> $T/config4.log || { tail -5 $T/config4.log; exit 1; }
cut -c1-600 $T/config4.json
