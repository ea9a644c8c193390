#!/bin/bash
# GPU box: BASELINE configs[4] (recipient side) on one MI355X, its kernel-trace stats, and the N = 2
# seed-split rehearsal (two ranks on one GPU over gloo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/config4
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config 4 --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.log || { tail -5 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --config 4 --steps 2 --warmup 1 > $OUT/bench_traced.json 2> $OUT/bench_traced.log || { tail -5 $OUT/bench_traced.log; exit 1; }
SDA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 2 --config 4 --steps 2 --warmup 1 \
    > $OUT/bench_w2.json 2> $OUT/bench_w2.log || { tail -5 $OUT/bench_w2.log; exit 1; }
grep '^{' $OUT/bench_w2.json | cut -c1-300
