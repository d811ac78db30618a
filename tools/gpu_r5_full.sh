#!/bin/bash
# round 5: the shipped tree end to end -- bench (configs[2], N=1), then the whole -m gpu suite
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_bench_mid.json 2> gpurun_out/r5_bench_mid.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_bench_mid.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5_bench_mid.json').read().strip().splitlines()[-1])
print('bench', d['ms_per_step'], 'ms', d['value'], 'fps', 'frac', d['roofline']['frac'], d['roofline']['kernel'])
print(json.dumps(d['roofline']['fused_lora_gemms']))"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5_pytest_gpu_mid.log 2>&1
rc=$?; tail -3 gpurun_out/r5_pytest_gpu_mid.log; exit $rc
