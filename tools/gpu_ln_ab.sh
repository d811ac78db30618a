#!/bin/bash
# LayerNorm at C = 1280 (M = 8192): rows per wave pass 1 / 2 / 4 -- isolated (graph-timed) and in the step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layer_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ln.log 2>&1 || { tail -30 gpurun_out/pytest_ln.log; exit 1; }
VST_LN_RIT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layer_norm" -x -q --timeout 120 --timeout-method thread >> gpurun_out/pytest_ln.log 2>&1 || { tail -30 gpurun_out/pytest_ln.log; exit 1; }
VST_LN_RIT=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layer_norm" -x -q --timeout 120 --timeout-method thread >> gpurun_out/pytest_ln.log 2>&1 || { tail -30 gpurun_out/pytest_ln.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_ln.log
for r in 2 1 4 2 1 4; do
  echo "RIT=$r"; VST_LN_RIT=$r timeout -k 10 120 python -u tools/norm_bench.py 2>&1 | grep '"layernorm"' | grep '"C": 1280' || exit 1
done
bash tools/ab_bench.sh new lnrita lnritb new2 lnrita2 lnritb2
