#!/bin/bash
# sa_self_kernel 4 waves (VST_SA_SELF=1, default) vs 2 waves per workgroup (2) vs spatial_attn_kernel<0> (0)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/r5_sa_ab4.txt; : > $out
for rep in 1 2; do
  for v in 0 1 2; do
    VST_SA_SELF=$v timeout -k 10 120 python -u tools/sa_self_ab.py >> $out 2>> gpurun_out/r5_sa_ab4.err || { echo "variant $v rc=$?"; tail -5 gpurun_out/r5_sa_ab4.err; exit 1; }
  done
done
cat $out | cut -c1-130
