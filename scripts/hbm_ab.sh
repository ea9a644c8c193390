#!/bin/bash
# The HBM-backing A/B of DESIGN.md §2: tools/hbm_diag (ROCm's own HIP runtime, no torch) and
# scripts/hbm_diag.py (inside torch, on torch's bundled runtime), each with the trimmed virtual range retired
# (SDA_HBM_VA_FREE=0, the shipped behaviour) and returned to the runtime (=1, round 4's first allocator).
# A mismatch (exit 1) is a result, not a failure; any other non-zero exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=${1:-6}
run() {
  "$@"
  rc=$?
  echo "exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
echo "== tools/hbm_diag va_free=0"; run timeout -k 10 120 ./tools/hbm_diag 0 "$rounds"
echo "== tools/hbm_diag va_free=1"; run timeout -k 10 120 ./tools/hbm_diag 1 "$rounds"
echo "== hbm_diag.py SDA_HBM_VA_FREE=0"; export SDA_HBM_VA_FREE=0; run timeout -k 10 180 python3 -u scripts/hbm_diag.py "$rounds"
echo "== hbm_diag.py SDA_HBM_VA_FREE=1"; export SDA_HBM_VA_FREE=1; run timeout -k 10 180 python3 -u scripts/hbm_diag.py "$rounds"
exit 0
