#!/bin/bash
# round 5: LDS-DMAs inside the MFMA segments (abl/libvst_dmm.so, -DVST_P8_DMM) vs the current build and round 4's,
# every GEMM shape of the step, outputs md5-compared
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u tools/lib_ab.py 2 base=abl/libvst_base.so cur=- dmm=abl/libvst_dmm.so > gpurun_out/r5_dmm_ab.txt 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/r5_dmm_ab.txt; exit 1; }
grep shape gpurun_out/r5_dmm_ab.txt
