#!/bin/bash
# persistent in-GEMM LoRA (128x320 tiles) as the default: LoRA / xattn tests, step A/B against VST_P8_LORA_PERSIST=0,
# then the frame-shard and parity suites
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_lora_gpu.py tests/test_gemm_xattn_gpu.py > gpurun_out/r5_lp2_tests.log 2>&1 || { tail -20 gpurun_out/r5_lp2_tests.log; exit 1; }
tail -1 gpurun_out/r5_lp2_tests.log
bash tools/gpu_r5_stepab.sh lp0 new lp0 new > gpurun_out/r5_lp_step_ab.txt 2>&1 || { tail -20 gpurun_out/r5_lp_step_ab.txt; exit 1; }
grep "ms/step" gpurun_out/r5_lp_step_ab.txt | cut -c1-150
grep "fused" gpurun_out/r5_lp_step_ab.txt | cut -c1-300
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_frame_shard.py tests/test_parity_bf16_gpu.py tests/test_parity_gpu.py tests/test_bench_rehearsal.py > gpurun_out/r5_lp2_suites.log 2>&1
rc=$?; tail -3 gpurun_out/r5_lp2_suites.log; exit $rc
