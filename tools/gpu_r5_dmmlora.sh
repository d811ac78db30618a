#!/bin/bash
# round 5: DMAs inside the MFMA segments for the in-GEMM LoRA kernels only (now the default): LoRA / xattn tests,
# per-launch A/B vs the previous build (md5-compared), then the whole step alternated
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lora_gpu.py \
  tests/test_gemm_xattn_gpu.py -m gpu > gpurun_out/r5_dmmlora_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r5_dmmlora_tests.log; exit 1; }
tail -1 gpurun_out/r5_dmmlora_tests.log
VST_AB_SHAPES=out1280_lora,out640_lora,qkv1280_lora,qkv640_lora,xattn1280_lora,xattn640_lora,geglu1280 timeout -k 10 600 \
  python -u tools/lib_ab.py 3 prev=abl/libvst_prev.so cur=- > gpurun_out/r5_dmmlora_ab.txt 2>&1 || { echo "ab rc=$?"; exit 1; }
grep shape gpurun_out/r5_dmmlora_ab.txt
bash tools/gpu_r5_stepab.sh prev new prev new
