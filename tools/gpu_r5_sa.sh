#!/bin/bash
# spatial self-attention variants, alternating processes (tools/sa_self_ab.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r5_sa_ab.txt; : > $out
for rep in 1 2; do
  for v in ${SA_VARIANTS:-0 40 41 80 81}; do
    VST_SA_SELF=$v timeout -k 10 120 python -u tools/sa_self_ab.py >> $out 2>> gpurun_out/r5_sa_ab.err || { echo "variant $v rc=$?"; tail -5 gpurun_out/r5_sa_ab.err; exit 1; }
  done
done
cat $out
