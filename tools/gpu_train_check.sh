#!/bin/bash
# GPU pass for the training path: backward-kernel tests, data-parallel TrainStep, train-step timing + rocprof stats.
# Usage (via gpurun, from the repo root): bash tools/gpu_train_check.sh [tag] [pytest -k expression]
set -o pipefail
TAG=${1:-r2}
K=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_data_parallel.py tests/test_kernels_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_train_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_train_$TAG.log | tail -40; exit 1; }
grep -E "\[train\]|\[dp\]|passed|failed" gpurun_out/pytest_train_$TAG.log | tail -60
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o run -- \
  python -u tools/train_step_bench.py 3 > gpurun_out/train_step_$TAG.json 2> gpurun_out/train_step_$TAG.err \
  || { tail -20 gpurun_out/train_step_$TAG.err; exit 1; }
cat gpurun_out/train_step_$TAG.json
S=$(find gpurun_out/tprof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" > gpurun_out/train_kernel_stats_$TAG.csv
rm -rf gpurun_out/tprof
head -25 gpurun_out/train_kernel_stats_$TAG.csv | cut -c1-160
