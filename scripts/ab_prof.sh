#!/bin/bash
# A/B kernel times (rocprofv3 --kernel-trace --stats) of engine variants over one bench leg.
#   bash scripts/ab_prof.sh "<bench args>" default build/var/x/libsda_engine.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=$1; shift
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = default ]; then unset SDA_ENGINE_LIB; else export SDA_ENGINE_LIB=$lib; fi
  echo "== $lib"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp_$i -o run -- python3 bench.py $ARGS > gpurun_out/abp_$i.log 2>&1 || { tail -5 gpurun_out/abp_$i.log; exit 1; }
  grep -E '^\[' gpurun_out/abp_$i.log | cut -c1-400
  python3 - gpurun_out/abp_$i/run_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print("   %-70s %5s %12.1f us" % (x["Name"][:70], x["Calls"], float(x["AverageNs"]) / 1e3))
PY
done
