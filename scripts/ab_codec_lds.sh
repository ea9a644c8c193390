set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_codec_fused.py tests/test_gpu_pipelines.py tests/test_snapshot.py > gpurun_out/pytest_codec_el16.log 2>&1 && tail -1 gpurun_out/pytest_codec_el16.log && \
bash scripts/ab_libs.sh codec 3 build/ab/sub1.so build/ab/cnt1.so
