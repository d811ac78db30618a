#!/bin/bash
# attn2: the last head's text K/V issued before the u . V step and the other heads' waited for behind its attention:
# isolated A/B (bitwise), the xattn tests, a step A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
VST_AB_SHAPES=xattn1280_lora,xattn640_lora timeout -k 10 300 python -u tools/lib_ab.py 3 base=abl/libvst_xbase.so new=- > gpurun_out/r5_xkv_ab.txt 2>&1 || { tail -20 gpurun_out/r5_xkv_ab.txt; exit 1; }
grep shape gpurun_out/r5_xkv_ab.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_xattn_gpu.py > gpurun_out/r5_xkv_tests.log 2>&1 || { tail -20 gpurun_out/r5_xkv_tests.log; exit 1; }
tail -1 gpurun_out/r5_xkv_tests.log
cp abl/libvst_xbase.so abl/libvst_base.so
bash tools/gpu_r5_stepab.sh base new base new > gpurun_out/r5_xkv_step.txt 2>&1 || { tail -20 gpurun_out/r5_xkv_step.txt; exit 1; }
grep "ms/step" gpurun_out/r5_xkv_step.txt | cut -c1-120
grep "fused" gpurun_out/r5_xkv_step.txt | cut -c1-250
