#!/bin/bash
# round 5: the training-gradient gate on the CPU bf16-autocast yardstick (deterministic), and the piecewise-capture cost
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/piecewise_cost.py > gpurun_out/r5_piecewise_cost.json 2> gpurun_out/r5_piecewise_cost.err || { echo "piecewise rc=$?"; exit 1; }
cat gpurun_out/r5_piecewise_cost.json
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 580 --timeout-method thread \
  "tests/test_training_gpu.py::test_unet_training_step_grads_vs_oracle" > gpurun_out/r5_train_grads.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|ratio|median" gpurun_out/r5_train_grads.log | tail -20; exit $rc
