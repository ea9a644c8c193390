#!/bin/bash
# Share-gen's time across fresh processes on one box, with each run's buffer addresses.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/${1:-genluck}
mkdir -p $T
for i in 1 2 3 4 5 6 7 8; do
  a="--only shamir --no-cpu --steps 10"
  [ $((i % 2)) = 0 ] && a="--only shamir --steps 20 --no-check"
  timeout -k 10 300 python -u bench.py $a 2>&1 >/dev/null | grep "^\[shamir\]" | python3 -c '
import sys, json
d = json.loads(sys.stdin.read().split(" ", 1)[1])
print(" ".join("%s=%.3f" % (k, d[k]) for k in ("gen_ms", "gen_canonical_ms", "reveal_canonical_ms")), d["buffers"])' >> $T/runs.txt || exit 1
done
cat $T/runs.txt
