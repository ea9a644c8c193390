# fused clerk decode+combine: parity tests, codec bench leg, kernel trace of that leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fused; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_codec_fused.py tests/test_gpu_codec.py tests/test_gpu_pipelines.py tests/test_snapshot.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --only codec --steps 3 --warmup 1 > $O/bench_codec.json 2> $O/bench_codec.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o codec -- python3 bench.py --only codec --steps 3 --warmup 1 > $O/prof.log 2>&1
