#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_frame_shard.py tests/test_bench_rehearsal.py tests/test_kernels_gpu.py tests/test_gemm_lora_gpu.py tests/test_host.py tests/test_rccl_gpu.py -m gpu -v -s -rA --timeout 600 --timeout-method thread -x > gpurun_out/r6_pytest_b.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|\[shard\]|\[rehearsal\]" gpurun_out/r6_pytest_b.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6_bench_b.json 2> gpurun_out/r6_bench_b.err
rc=$?; tail -c 600 gpurun_out/r6_bench_b.json; exit $rc
