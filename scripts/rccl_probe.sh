#!/bin/bash
# Two ranks of scripts/rccl_probe.py on one GPU over RCCL (a probe: RCCL may refuse duplicate devices).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rccl
PORT=29611
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT NCCL_DEBUG=WARN \
    timeout -k 5 90 python3 scripts/rccl_probe.py > gpurun_out/rccl/rank$r.log 2>&1 &
done
wait
tail -5 gpurun_out/rccl/rank0.log gpurun_out/rccl/rank1.log
