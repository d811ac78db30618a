# A/B of the 8-phase GEMM policy in the inference step: VST_GEMM_P8 = 0 (ring only), unset (K < 2048 rule), 1 (all).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 def 1; do
  if [ "$v" = def ]; then unset VST_GEMM_P8; else export VST_GEMM_P8=$v; fi
  VST_BENCH_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks > gpurun_out/b_p8_$v.json 2> gpurun_out/b_p8_$v.err || { tail -20 gpurun_out/b_p8_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_p8_$v.json')); print('P8=$v', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
done
