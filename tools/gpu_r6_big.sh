#!/bin/bash
# operands past 2 GiB (row / image chunking in vst_gemm_ex / vst_conv3x3_ex), then the GEMM / conv kernel tests
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -s -k "past_2gb or gemm or conv" \
  --timeout 200 --timeout-method thread > gpurun_out/r6_big.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|past_2gb" gpurun_out/r6_big.txt | tail -15; exit $rc
