#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_frame_shard.py tests/test_bench_rehearsal.py -m gpu -v -s -rA --timeout 600 --timeout-method thread -x > gpurun_out/r6_pytest_shard2.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|\[shard\] overlap|\[rehearsal\]" gpurun_out/r6_pytest_shard2.log | tail -20; exit $rc
