#!/bin/bash
# Seeds whose ChaCha gen_range streams reject a draw early (tools/chacha_reject_search.hip), for the
# rejection fix-up tests: the lazy-path prime 2^32 - 2^16 + 1, a 2^-28-rate modulus on the non-lazy fast
# path, and the field prime (2^-42.5 per draw: a long search).  Build the tool first, in this container:
#   hipcc -O3 --offload-arch=gfx950 tools/chacha_reject_search.hip -o tools/chacha_reject_search
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/reject
timeout -k 10 60 ./tools/chacha_reject_search 4294901761 65536 19 0x5da 7 11 > gpurun_out/reject/m_2_32.txt || exit 1
timeout -k 10 60 ./tools/chacha_reject_search 68719676673 65536 15 0x5da 7 11 > gpurun_out/reject/m_2_36.txt || exit 1
head -3 gpurun_out/reject/m_2_32.txt gpurun_out/reject/m_2_36.txt
timeout -k 10 200 ./tools/chacha_reject_search 2147482801 1048576 23 0x5da 7 11 > gpurun_out/reject/m_field.txt || exit 1
cat gpurun_out/reject/m_field.txt
