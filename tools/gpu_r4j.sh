# round-4 GPU session j: p8 conv tests + in-step A/B (VST_P8_CONV 0/1), rocprof gaps
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 600 r4j_tests.log python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "conv"
grep -E "FAILED|passed|failed" gpurun_out/r4j_tests.log | tail -5
for v in 0 1 0 1; do
  VST_P8_CONV=$v run 300 r4j_bench_conv${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4j_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'conv' in n})"; done
bash tools/gpu_r4i.sh
