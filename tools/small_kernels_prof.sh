#!/bin/bash
# rocprofv3 kernel stats of a short bench for the small kernels (gemm_rows, conv_small) vs the old build:
# bash tools/small_kernels_prof.sh <tag> [VST_LIB_AB path]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
if [ -n "$2" ]; then export VST_LIB_AB=$2; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_$TAG -o run -- \
  python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/sp_$TAG.json 2> gpurun_out/sp_$TAG.err \
  || { echo "rocprof failed"; tail -20 gpurun_out/sp_$TAG.err; exit 1; }
STATS=$(find gpurun_out/sp_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$STATS" > gpurun_out/sp_stats_$TAG.csv
rm -rf gpurun_out/sp_$TAG
grep -E "gemm_rows|conv_small|RingCfg<128, 128, 2, 2, 5>, 0, 0|gemm_kernel<2|RingCfg<128, 64" gpurun_out/sp_stats_$TAG.csv | cut -c1-200
