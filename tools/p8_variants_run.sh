#!/bin/bash
# Timeline of each diagnostics variant (tools/p8_variants.sh) on the given shapes: bash tools/p8_variants_run.sh "base fast" shapes...
set -o pipefail
export TMPDIR=/tmp
V=$1; shift
for v in $V; do
  echo "=== variant $v"
  VST_LIB_AB=abx/libvst_$v.so timeout -k 10 150 python -u tools/p8_trace.py "$@" 2>/dev/null || exit 1
done
