#!/bin/bash
# A/B of the ChaCha mask-combine kernel: round-1 kernel (build/ab_old) vs the current one, seed
# chunking and one/two seeds per iteration.  Interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_chacha.txt; : > $out
for r in 1 2 3; do
  for v in old "cur:0:" "cur:0:3" "cur:0:5" "cur:0:7" "cur:1:" "cur:1:3" "cur:1:5"; do
    if [ "$v" == old ]; then
      ms=$(SDA_ENGINE_LIB=build/ab_old/libsda_engine.so timeout -k 10 120 python bench.py --only chacha --steps 20 2>&1 | grep '^\[chacha\]' | sed 's/.*"ms": \([0-9.]*\).*/\1/') || exit 1
    else
      IFS=: read _ p c <<< "$v"
      ms=$(SDA_CHACHA_PAIR=$p SDA_CHACHA_CHUNKS=$c timeout -k 10 120 python bench.py --only chacha --steps 20 2>&1 | grep '^\[chacha\]' | sed 's/.*"ms": \([0-9.]*\).*/\1/') || exit 1
    fi
    echo "round $r $v $ms" | tee -a $out
  done
done
