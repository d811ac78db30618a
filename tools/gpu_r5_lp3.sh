#!/bin/bash
# persistent LoRA on 256-row tiles (rotation-switched epilogue staging): isolated A/B, bitwise
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1 VST_AB_SHAPES=qkv1280_lora,out640_lora,qkv640_lora,out1280_lora
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/p8_ph_ab.py 3 2+persist 2+persist+lp 2+persist+lp+no320 > gpurun_out/r5_lp3_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_lp3_ab.txt; exit 1; }
grep shape gpurun_out/r5_lp3_ab.txt
