set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o run -- python -u tools/train_step_bench.py 2 > gpurun_out/tprof.out 2> gpurun_out/tprof.err || { tail -20 gpurun_out/tprof.err; exit 1; }
cat gpurun_out/tprof.out
S=$(find gpurun_out/tprof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" > gpurun_out/train_kernel_stats_r2a.csv
rm -rf gpurun_out/tprof
head -30 gpurun_out/train_kernel_stats_r2a.csv
