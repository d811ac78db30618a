#!/bin/bash
# VAE conv tile routing (conv_ring128): kernel tests + VAE tests, then the VAE encode profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vae_gpu.py -m gpu -k "conv or vae" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r6_vae_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/vae_prof.py > gpurun_out/r6_vae_prof.txt 2>&1
rc=$?
tail -5 gpurun_out/r6_vae_tests.txt; head -3 gpurun_out/r6_vae_prof.txt
exit $rc
