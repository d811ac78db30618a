#!/bin/bash
# round 5: LoRA kernels without the fu re-read (rotated A row blocks) and without sink DMAs: tests, then A/B vs the
# round-4 build (abl/libvst_base.so) with bitwise output check
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lora_gpu.py \
  tests/test_gemm_xattn_gpu.py -m gpu > gpurun_out/r5_lora1_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r5_lora1_tests.log; exit 1; }
tail -3 gpurun_out/r5_lora1_tests.log
VST_AB_SHAPES=out1280_lora,out640_lora,qkv1280_lora,qkv640_lora,xattn1280_lora,xattn640_lora timeout -k 10 500 \
  python -u tools/lib_ab.py 3 base=abl/libvst_base.so new=- > gpurun_out/r5_lora1_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_lora1_ab.txt; exit 1; }
grep shape gpurun_out/r5_lora1_ab.txt
