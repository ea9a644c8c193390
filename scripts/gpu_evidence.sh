#!/bin/bash
# One round's GPU evidence, in order, stopping at the first failure:
#   int-op microbench, the -m gpu suite, the default bench line, rocprofv3 kernel-trace stats of the
#   bench, HBM traffic passes of the combine, SQ/TCC passes over the packed-Shamir and ChaCha legs.
#   bash scripts/gpu_evidence.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
mkdir -p gpurun_out
(nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket") > gpurun_out/host.txt
timeout -k 10 60 ./tools/ubench_int > gpurun_out/ubench_int.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || exit $?
bash scripts/gpu_prof.sh $TAG || exit $?
echo done
