#!/bin/bash
# persistent in-GEMM LoRA kernels (128x320 tiles, VST_P8_LORA_PERSIST=1): isolated A/B with bitwise check, then the
# LoRA GEMM tests with the variant on
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1 VST_AB_SHAPES=qkv640_lora,out640_lora,qkv1280_lora
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/p8_ph_ab.py 3 2+persist 2+persist+lp 2+persist+bn320 2+persist+bn320+lp > gpurun_out/r5_lp_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_lp_ab.txt; exit 1; }
grep shape gpurun_out/r5_lp_ab.txt
VST_P8_LORA_PERSIST=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_lora_gpu.py > gpurun_out/r5_lp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_lp_tests.log; exit $rc
