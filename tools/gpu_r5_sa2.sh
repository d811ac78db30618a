#!/bin/bash
# sa_self_kernel (default) vs spatial_attn_kernel<0> (VST_SA_SELF=0): times, output hashes, attention + parity tests
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5_sa_ab2.txt; : > $out
for rep in 1 2; do
  for v in 0 1; do
    VST_SA_SELF=$v timeout -k 10 120 python -u tools/sa_self_ab.py >> $out 2>> gpurun_out/r5_sa_ab2.err || { echo "variant $v rc=$?"; tail -5 gpurun_out/r5_sa_ab2.err; exit 1; }
  done
done
cat $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_sa2.log 2>&1
rc=$?; tail -3 gpurun_out/r5_pytest_gpu_sa2.log; exit $rc
