set -o pipefail
# GPU tests + short bench with the per-kernel table (no CPU baseline)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_quick.log 2>&1 \
  || { tail -30 gpurun_out/t_quick.log; exit 1; }
tail -2 gpurun_out/t_quick.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_quick.json 2> gpurun_out/b_quick.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/b_quick.json')); print(d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print(k, v['ms_per_step'], v['tflops'], v['gbs'])"
