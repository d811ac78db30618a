set -o pipefail
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lora-mode folded > gpurun_out/b_folded.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lora-rank 0 > gpurun_out/b_nolora.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --frames 32 --size 768 > gpurun_out/b_cfg4.json 2>/dev/null || exit 1
for f in b_folded b_nolora b_cfg4; do python -c "
import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"; done
