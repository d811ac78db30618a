#!/bin/bash
# round 5: frame-sharding gates (8 ranks x 4 frames of configs[3], 16x512 over 8, the 576 fusion policy), the bench
# rehearsal with the strong / configs[3] sub-records, RCCL teardown order
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_rccl_gpu.py \
  tests/test_frame_shard.py tests/test_bench_rehearsal.py -m gpu > gpurun_out/r5_shard_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|\[shard\]|\[rehearsal\]" gpurun_out/r5_shard_tests.log | tail -40; exit $rc
