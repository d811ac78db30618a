#!/bin/bash
# Run a selection of GPU tests with their prints (-s) on the box: bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "\[bf16-parity\]|\[parity\]|\[train\]|\[dp\]|\[shard\]|PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_$TAG.log | tail -150
exit $rc
