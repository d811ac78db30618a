#!/bin/bash
# round 5: residual tile prefetched into the LDS by the tail DMAs (abl/libvst_rpre.so, -DVST_P8_RPRE): GEMM / LoRA
# kernel tests on that build, then A/B vs the current build, outputs md5-compared
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VST_LIB_AB=abl/libvst_rpre.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_lora_gpu.py tests/test_gemm_xattn_gpu.py tests/test_kernels_gpu.py -m gpu -k "gemm or lora or xattn or residual" \
  > gpurun_out/r5_rpre_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r5_rpre_tests.log; exit 1; }
tail -2 gpurun_out/r5_rpre_tests.log
VST_AB_SHAPES=out1280_lora,out640_lora,ff2_1280,ff2_640,ff2_320,proj320 timeout -k 10 900 python -u tools/lib_ab.py 3 cur=- rpre=abl/libvst_rpre.so > gpurun_out/r5_rpre_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_rpre_ab.txt; exit 1; }
grep shape gpurun_out/r5_rpre_ab.txt
