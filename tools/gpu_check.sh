#!/bin/bash
# One GPU-box pass: parity tests, bench (with CPU baseline), rocprofv3 kernel stats of a short bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r1}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
if [ -n "$PMC" ]; then
  md5sum video_style_transfer_amd/libvst_hip.so > gpurun_out/pmc_so.md5
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o pmc -- \
      python -u bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline \
      > gpurun_out/pmc_$C.out 2> gpurun_out/pmc_$C.err || { echo "pmc $C failed"; tail -5 gpurun_out/pmc_$C.err; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_so.md5 \
    > gpurun_out/pmc_traffic_$TAG.json || exit 1
  rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
  cp gpurun_out/pmc_traffic_$TAG.json profiles/pmc_traffic_$TAG.json  # the bench below reads the newest (same .so)
  echo pmc done
fi
VST_BENCH_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
if [ -n "$TRAIN" ]; then
  timeout -k 10 400 python -u bench.py --train --steps 5 --warmup 2 > gpurun_out/bench_train_$TAG.json 2> gpurun_out/bench_train_$TAG.err \
    || { echo "train bench failed"; tail -20 gpurun_out/bench_train_$TAG.err; exit 1; }
  cat gpurun_out/bench_train_$TAG.json
fi
# keep only the stats summary (the raw traces overflow gpurun_out's copy-back limit)
STATS=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
if [ -n "$STATS" ]; then python tools/prof_summary.py "$STATS" > gpurun_out/kernel_stats_$TAG.csv; fi
rm -rf gpurun_out/prof_$TAG

echo all done
