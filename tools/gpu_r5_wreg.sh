#!/bin/bash
# round 5: the W operand from global memory into registers (abl/libvst_wreg.so, -DVST_P8_WREG; BN 192 / 320 tiles,
# one workgroup per tile): GEMM / LoRA / xattn / conv kernel tests on that build, then A/B vs the current build with
# outputs md5-compared
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VST_LIB_AB=abl/libvst_wreg.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_lora_gpu.py tests/test_gemm_xattn_gpu.py tests/test_kernels_gpu.py -m gpu -k "gemm or conv or lora or xattn" \
  > gpurun_out/r5_wreg_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r5_wreg_tests.log; exit 1; }
tail -2 gpurun_out/r5_wreg_tests.log
timeout -k 10 900 python -u tools/lib_ab.py 2 cur=- wreg=abl/libvst_wreg.so > gpurun_out/r5_wreg_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_wreg_ab.txt; exit 1; }
grep shape gpurun_out/r5_wreg_ab.txt
