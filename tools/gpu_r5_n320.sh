#!/bin/bash
# narrow-GEMM 128x320 policy (VST_P8_320N=1): per-shape tables of both, then a step A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in 0 1; do
  VST_P8_320N=$v VST_BENCH_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vae --no-peaks > gpurun_out/r5_n320_shapes_$v.json 2> gpurun_out/r5_n320_shapes_$v.err || { tail -20 gpurun_out/r5_n320_shapes_$v.err; exit 1; }
  grep "\[shape\]" gpurun_out/r5_n320_shapes_$v.err | grep -E "x320x|x640x" > gpurun_out/r5_n320_table_$v.txt
done
paste -d'\n' gpurun_out/r5_n320_table_0.txt /dev/null | head -40
cat gpurun_out/r5_n320_table_1.txt
bash tools/gpu_r5_stepab.sh new n320 new n320 > gpurun_out/r5_n320_step_ab.txt 2>&1 || { tail -20 gpurun_out/r5_n320_step_ab.txt; exit 1; }
grep "ms/step" gpurun_out/r5_n320_step_ab.txt
