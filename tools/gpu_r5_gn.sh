#!/bin/bash
# GroupNorm statistics from the conv epilogue: kernel tests, frame-shard / parity suites, then a step A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_vae_gpu.py -k "colstat or conv or group_norm or vae" > gpurun_out/r5_gn_kernel_tests.log 2>&1 || { tail -30 gpurun_out/r5_gn_kernel_tests.log; exit 1; }
tail -1 gpurun_out/r5_gn_kernel_tests.log
bash tools/gpu_r5_stepab.sh gn0 new gn0 new > gpurun_out/r5_gn_step_ab.txt 2>&1 || { tail -20 gpurun_out/r5_gn_step_ab.txt; exit 1; }
grep "ms/step" gpurun_out/r5_gn_step_ab.txt | cut -c1-200
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_frame_shard.py tests/test_parity_bf16_gpu.py tests/test_parity_gpu.py > gpurun_out/r5_gn_suites.log 2>&1
rc=$?; tail -3 gpurun_out/r5_gn_suites.log; exit $rc
