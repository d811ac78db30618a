#!/bin/bash
# round 5: LoRA kernels, two A/Bs: the B1 placement of the plain GEMMs (abl/libvst_lorab1e.so) and 128x320 tiles
# (VST_P8_320=1) against the current build
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp VST_AB_SHAPES=out1280_lora,out640_lora,qkv1280_lora,qkv640_lora,xattn1280_lora,xattn640_lora
timeout -k 10 500 python -u tools/lib_ab.py 3 cur=- b1e=abl/libvst_lorab1e.so > gpurun_out/r5_lora2_b1e.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_lora2_b1e.txt; exit 1; }
grep shape gpurun_out/r5_lora2_b1e.txt
timeout -k 10 500 python -u tools/p8_ph_ab.py 3 2 2+320 > gpurun_out/r5_lora2_320.txt 2>&1 || { echo "ab320 rc=$?"; tail -20 gpurun_out/r5_lora2_320.txt; exit 1; }
grep shape gpurun_out/r5_lora2_320.txt
