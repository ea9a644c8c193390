set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "chacha or mask" > gpurun_out/pytest_chacha.log 2>&1 && tail -1 gpurun_out/pytest_chacha.log && \
bash scripts/ab_libs.sh chacha 3 build/ab/cnt1.so build/ab/cc8.so build/ab/cc7floor.so
