# round-4 GPU session d: the whole -m gpu suite with prints (gates, floors, shard equality, RCCL)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r4g_pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r4g_pytest_gpu.log | tail -3
exit $rc
