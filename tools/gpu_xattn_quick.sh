#!/bin/bash
# Fused attn2 (q projection + cross-attention epilogue): kernel tests, UNet parity at F=16, then a same-box A/B of
# the denoise step against the two-launch attn2 (VST_XATTN_FUSE=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_xattn_gpu.py tests/test_gemm_lora_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_xattn.log 2>&1 || { echo "xattn tests failed"; tail -40 gpurun_out/pytest_xattn.log; exit 1; }
tail -2 gpurun_out/pytest_xattn.log
timeout -k 10 700 python -u -m pytest tests/test_parity_bf16_gpu.py -x -v -s --timeout 600 --timeout-method thread -k "configs2 or configs1" > gpurun_out/pytest_parity_xattn.log 2>&1 || { echo "parity failed"; grep -E "parity|PASS|FAIL|Error" gpurun_out/pytest_parity_xattn.log | tail -30; exit 1; }
grep -E "chained|worst|passed|failed" gpurun_out/pytest_parity_xattn.log | tail -8
bash tools/ab_bench.sh new noxattn new2 noxattn2
