#!/bin/bash
# The round's evidence run on the final code (one gpurun call): host model, the whole -m gpu suite, smoke(),
# the default bench line, the bench under rocprofv3 --kernel-trace --stats, the combine's FETCH_SIZE and
# WRITE_SIZE passes, the SQ/traffic passes over the packed-Shamir and ChaCha legs, configs[3] and configs[4],
# the codec leg's FETCH_SIZE / WRITE_SIZE passes (the clerk's decode -> combine traffic).
#   bash scripts/gpu_final.sh <tag>         -> gpurun_out/<tag>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}
bash scripts/gpu_steps.sh "$TAG" host tests smoke "bench:" "trace:--steps 10 --warmup 2 --no-cpu --no-host-path" \
  "pmc:FETCH_SIZE:--only combine --steps 3 --warmup 1" "pmc:WRITE_SIZE:--only combine --steps 3 --warmup 1" \
  "sh:pmc_shamir.sh ${TAG}_shamir --only shamir --steps 3 --warmup 1" \
  "sh:pmc_shamir.sh ${TAG}_chacha --only chacha --steps 3 --warmup 1" \
  "bench:--config 3 --steps 2 --warmup 1 --no-cpu" "bench:--config 4 --steps 1 --warmup 1 --no-cpu" \
  "pmc:FETCH_SIZE:--config 3 --only combine --steps 1 --warmup 0 --no-cpu" \
  "pmc:WRITE_SIZE:--config 3 --only combine --steps 1 --warmup 0 --no-cpu" \
  "pmc:FETCH_SIZE:--only codec --steps 1 --warmup 0 --no-cpu" "pmc:WRITE_SIZE:--only codec --steps 1 --warmup 0 --no-cpu"
