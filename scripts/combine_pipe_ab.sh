# process-level A/B of SDA_COMBINE_PIPE (0 = the unpipelined kernel): bench.py --only combine, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06l
for r in 1 2 3 4; do
  for v in 0 1; do
    SDA_COMBINE_PIPE=$v timeout -k 10 200 python3 -u bench.py --only combine --steps 20 --warmup 3 --no-cpu > /dev/null 2> gpurun_out/r06l/pipe_${v}_$r.log || { echo "run $v failed"; tail -5 gpurun_out/r06l/pipe_${v}_$r.log; exit 1; }
    echo "round $r PIPE=$v $(grep '^\[combine\]' gpurun_out/r06l/pipe_${v}_$r.log | cut -c1-120) signed $(grep '^\[combine_signed\]' gpurun_out/r06l/pipe_${v}_$r.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read().split(" ",1)[1])["kernel_ms"],4))')"
  done
done
