#!/bin/bash
# Round 4's failing sequence (profiles/r04y): the GPU modules up to and including test_gpu_hbm.py, in suite
# order, once per allocator setting:
#   old  SDA_HBM_POOL_MB=0 SDA_HBM_VA_FREE=1   free unmaps, releases and returns the range (round 4's first allocator)
#   new  SDA_HBM_POOL_MB=0 SDA_HBM_VA_FREE=0   free unmaps and releases, the range is retired
# A test failure (pytest exit 1) is a result; any other non-zero exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mods="tests/test_abi_c.py tests/test_gpu_chacha_rejects.py tests/test_gpu_codec.py tests/test_gpu_codec_fused.py
      tests/test_gpu_config4.py tests/test_gpu_configs.py tests/test_gpu_device.py tests/test_gpu_hbm.py"
for va in 1 0 1 0; do
  echo "== SDA_HBM_POOL_MB=0 SDA_HBM_VA_FREE=$va"
  # shellcheck disable=SC2086
  SDA_HBM_POOL_MB=0 SDA_HBM_VA_FREE=$va timeout -k 10 600 python -u -m pytest $mods -m gpu -q -x --timeout 170 \
    --timeout-method thread 2>&1 | tail -25
  rc=${PIPESTATUS[0]}
  echo "exit $rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
done
exit 0
