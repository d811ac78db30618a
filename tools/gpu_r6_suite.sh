#!/bin/bash
# round 6: the whole -m gpu suite with every numeric line kept (-v -s -rA), golden tests first (tests/conftest.py)
# usage: bash tools/gpu_r6_suite.sh <tag> [extra pytest args]
set -o pipefail
TAG=${1:-suite}; shift
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -v -s -rA --timeout 900 --timeout-method thread "$@" \
  > gpurun_out/r6_pytest_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r6_pytest_$TAG.log | tail -30
exit $rc
