# round-4 GPU session w: p8 conv k order (64-channel block, tap) = VST_P8_CONV=2 vs (tap, channel) = 1; parity + in-step A/B
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
run 300 r4w_pytest_conv.log python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "conv"
for v in 1 2 1 2; do
  VST_P8_CONV=$v run 300 r4w_bench_conv${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4w_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'conv' in n})"; done
