set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02d/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err
