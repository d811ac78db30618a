#!/bin/bash
# Fused motion-module attention block: kernel tests, UNet parity (per layer and chained, configs[2] F=16), then a
# same-box A/B of the denoise step against the four-launch block (VST_MOTION_FUSE=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_motion_block_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_motion.log 2>&1 || { echo "motion tests failed"; tail -40 gpurun_out/pytest_motion.log; exit 1; }
tail -2 gpurun_out/pytest_motion.log
timeout -k 10 700 python -u -m pytest tests/test_parity_bf16_gpu.py -x -v -s --timeout 600 --timeout-method thread -k "configs2 or configs1 or denoise_50_steps_sdxl" > gpurun_out/pytest_parity_motion.log 2>&1 || { echo "parity failed"; grep -E "parity|PASS|FAIL|Error" gpurun_out/pytest_parity_motion.log | tail -40; exit 1; }
grep -E "motion  |chained|worst|denoise|passed|failed" gpurun_out/pytest_parity_motion.log | tail -24
bash tools/ab_bench.sh new nomotion new2 nomotion2
