#!/bin/bash
# sa_self_kernel as the default: step A/B against spatial_attn_kernel<0> (VST_SA_SELF=0), then the whole -m gpu suite
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_r5_stepab.sh sa0 new sa0 new > gpurun_out/r5_sa_step_ab.txt 2>&1 || { tail -20 gpurun_out/r5_sa_step_ab.txt; exit 1; }
grep "ms/step" gpurun_out/r5_sa_step_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_sa.log 2>&1
rc=$?; tail -3 gpurun_out/r5_pytest_gpu_sa.log; exit $rc
