#!/bin/bash
# Phase timeline of the 8-phase GEMM under each diagnostics ablation (trace build, bash tools/p8_trace.sh first).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in 0 1 2 4 16 6 18; do
  VST_LIB_AB=abx/libvst_trace.so VST_GEMM_ABLATE=$a timeout -k 10 120 python -u tools/p8_trace.py "$@" 2>/dev/null || exit 1
done
