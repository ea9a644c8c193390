#!/bin/bash
# Does share-gen's XCD-order gain depend on the device memory's history?  Fresh box: the share-gen
# memory ubench and the shamir leg; then the whole -m gpu suite (many allocations of every size); then
# the same two again; then the int32-stage library beside the current one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-memstate}
mkdir -p gpurun_out/$TAG
(rocm-smi --showmemorypartition --showcomputepartition; rocm-smi --showmeminfo vram) > gpurun_out/$TAG/partition.txt 2>&1 || true
bash scripts/gpu_steps.sh "$TAG" "tool:ubench_gen 1000 3" "bench:--only shamir --no-cpu" tests \
  "bench:--only shamir --no-cpu" "sh:ab_libs.sh shamir 2 sda_amd/libsda_engine.so build/dev/libsda_engine.so"
