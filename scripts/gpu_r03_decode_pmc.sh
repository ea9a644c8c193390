#!/bin/bash
# Counters of the two slot decodes (SDA_SLOT_DECODE=list vs the default own-word kernel) over the bench's
# codec leg: SQ issue counters, then FETCH_SIZE and WRITE_SIZE, one group per rocprofv3 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/${1:-r03decpmc}
mkdir -p $T
for k in list own; do
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    SDA_SLOT_DECODE=$k timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $T/${k}_p$i -o run -- python3 bench.py --only codec --steps 2 --warmup 1 > $T/${k}_p$i.log 2>&1 || { echo "pass $k $i failed"; tail -5 $T/${k}_p$i.log; exit 1; }
    python3 scripts/summarize_pmc.py $T/${k}_p$i > $T/${k}_p$i.txt 2>&1
    awk '/^[^ ]/{p=($0 ~ /slots_kernel|decode_kernel<int, true>/)} p' $T/${k}_p$i.txt
  done
done
