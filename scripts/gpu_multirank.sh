#!/bin/bash
# GPU box: world-size-2 rehearsal of the multi-GPU path on one MI355X (gloo in place of RCCL):
# the multirank parity tests, then bench.py exactly as the driver launches it for N = 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_multirank.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_multirank.log
[ $rc -ne 0 ] && exit $rc
export SDA_DIST_BACKEND=gloo
for cfg in 1 3; do
  steps=5; [ $cfg = 3 ] && steps=1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps $steps --warmup 1 --no-side --config $cfg \
      > gpurun_out/bench_w2_c$cfg.json 2> gpurun_out/bench_w2_c$cfg.log || { tail -20 gpurun_out/bench_w2_c$cfg.log; exit 1; }
  cat gpurun_out/bench_w2_c$cfg.json
done
