#!/bin/bash
# A/B timing of engine variants on the GPU box: bench.py side legs once per library.
#   bash scripts/ab.sh "<bench args>" default build/var/a/libsda_engine.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=$1; shift
for lib in "$@"; do
  if [ "$lib" = default ]; then unset SDA_ENGINE_LIB; else export SDA_ENGINE_LIB=$lib; fi
  echo "== $lib"
  timeout -k 10 120 python3 -u bench.py $ARGS 2>&1 | grep -E '^\[(shamir|chacha|combine)\]|Error|FAILED' || exit 1
done
