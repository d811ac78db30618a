#!/bin/bash
# round 5: ADVICE lows -- the training GroupNorm on vst_groupnorm with the backward's statistics in the same chunking,
# and the fused vs two-launch motion attention gate at configs[2]
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_training_gpu.py tests/test_data_parallel.py \
  "tests/test_parity_bf16_gpu.py::test_configs2_motion_attention_fused_vs_two_launches" \
  > gpurun_out/r5_adv_tests.log 2>&1
rc=$?; grep -E "\[tattn\]|\[train\] (tiny|sdxl):|PASSED|FAILED|passed|failed" gpurun_out/r5_adv_tests.log | tail -40; exit $rc
