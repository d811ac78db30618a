#!/bin/bash
# sa_self_kernel for inference only: the training tests, then the rest of the -m gpu suite after them
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_training_gpu.py tests/test_train_step_gpu.py tests/test_vae_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/r5_pytest_gpu_sa3.log 2>&1
rc=$?; tail -3 gpurun_out/r5_pytest_gpu_sa3.log; exit $rc
