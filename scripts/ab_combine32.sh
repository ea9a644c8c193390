# A/B record: the SDA_COMBINE32_UNROLL knob this compared was removed after the A/B (profiles/r02d/ab_combine32_unroll.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab_combine32.txt
for r in 1 2 3; do
  for u in 8 16; do
    line=$(SDA_COMBINE32_UNROLL=$u timeout -k 10 120 python bench.py --only codec --steps 20 --no-check 2>&1 | grep "^\[codec\]") || exit 1
    echo "round $r unroll $u $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().split(" ",1)[1]); print("decode_combine_ms=%.4f decode_ms=%.4f" % (d["decode_combine_ms"], d["decode_ms"]))')" | tee -a gpurun_out/ab_combine32.txt
  done
done
