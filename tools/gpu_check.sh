#!/bin/bash
# One GPU-box pass: parity tests, bench (with CPU baseline), rocprofv3 kernel stats of a short bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r1}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo done
