#!/bin/bash
# GPU box: bench.py --gpus 2 with the shamir side leg (two ranks sharing one MI355X over gloo), to
# exercise the all-GPU shares/s measurement of the N > 1 path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SDA_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 1 --only shamir --no-check \
    > gpurun_out/bench_w2_shamir.log 2>&1 || { tail -20 gpurun_out/bench_w2_shamir.log; exit 1; }
grep "^\[shamir\]" gpurun_out/bench_w2_shamir.log | head -1 | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --rows 2000 --no-cpu \
    > gpurun_out/bench_w2_full.json 2> gpurun_out/bench_w2_full.log || { tail -20 gpurun_out/bench_w2_full.log; exit 1; }
grep '^{' gpurun_out/bench_w2_full.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["n_gpus"], d["shamir"].get("shares_per_s_all_gpus"), list(d))'
