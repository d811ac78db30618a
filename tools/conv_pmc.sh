# Per-shape conv timing + memory-side traffic (FETCH_SIZE / WRITE_SIZE passes) of the shipped build.  Via gpurun.
# (profiles/r2_conv_korder_ab.txt also holds a channel-block-major k-order experiment measured with this script.)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/conv_traffic.py run 2>/dev/null || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/cpmc_$C -o c -- \
    python -u tools/conv_traffic.py run > /dev/null 2> gpurun_out/cpmc_$C.err || { tail -5 gpurun_out/cpmc_$C.err; exit 1; }
done
python tools/conv_traffic.py parse gpurun_out/cpmc_FETCH_SIZE gpurun_out/cpmc_WRITE_SIZE > gpurun_out/conv_traffic.json || exit 1
rm -rf gpurun_out/cpmc_FETCH_SIZE gpurun_out/cpmc_WRITE_SIZE
cat gpurun_out/conv_traffic.json
