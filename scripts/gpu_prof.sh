#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the default bench, the combine's HBM
# traffic passes, and SQ/TCC counter passes over the packed-Shamir and ChaCha legs.
#   bash scripts/gpu_prof.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
bash scripts/profile.sh $TAG || exit $?
bash scripts/pmc_shamir.sh ${TAG}_shamir --only shamir --steps 3 --warmup 1 || exit $?
bash scripts/pmc_shamir.sh ${TAG}_chacha --only chacha --steps 3 --warmup 1 || exit $?
