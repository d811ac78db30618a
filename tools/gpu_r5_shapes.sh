#!/bin/bash
# round 5: the fused / two-launch motion attention gate, then one bench with the per-shape table (VST_BENCH_SHAPES)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu \
  "tests/test_parity_bf16_gpu.py::test_configs2_motion_attention_fused_vs_two_launches" > gpurun_out/r5_tattn_gate.log 2>&1 || { echo "tattn rc=$?"; tail -20 gpurun_out/r5_tattn_gate.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5_tattn_gate.log | tail -1
VST_BENCH_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r5_bench_shapes.json 2> gpurun_out/r5_bench_shapes.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_bench_shapes.err; exit 1; }
grep "\[shape\]" gpurun_out/r5_bench_shapes.err | head -45
