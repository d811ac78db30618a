# round-4 GPU session l320: the UnZipLoRA out-projections (single projection, N % 320 == 0) on 128x320 tiles
# (VST_P8_LORA320=1) vs the automatic 256x192 policy; LoRA tests under the knob, in-step bench A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -40 gpurun_out/$log; exit $rc; fi
  return 0
}
run 300 l320_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_gemm_lora_gpu.py -k "320"
grep -E "passed|failed" gpurun_out/l320_tests.log
for v in 0 1 0 1; do
  VST_P8_LORA320=$v run 300 l320_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/l320_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'lora' in n})"; done
