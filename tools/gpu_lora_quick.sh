#!/bin/bash
# In-GEMM LoRA: kernel tests, then a same-box A/B of the denoise step against the two-pass LoRA (VST_LORA_INGEMM=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_lora_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1 || { echo "lora tests failed"; tail -40 gpurun_out/pytest_lora.log; exit 1; }
tail -2 gpurun_out/pytest_lora.log
bash tools/ab_bench.sh new nolora new2 nolora2
