#!/bin/bash
# kernel-trace of the codec bench leg (per-kernel times of count / decode / combine / encode passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/codec_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --only codec --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.log
