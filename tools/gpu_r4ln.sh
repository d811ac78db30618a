# round-4 GPU session ln: LayerNorm row statistics in one shuffle chain (VST_LN_CHAN=1, Chan combine of per-lane
# (mean, M2)) vs the two-chain two-pass statistics; LayerNorm tests under both, in-step bench A/B
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
VST_LN_CHAN=1 run 300 ln_tests_chan.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layer_norm"
run 300 ln_tests_base.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layer_norm"
grep -E "passed|failed" gpurun_out/ln_tests_*.log
for v in 0 1 0 1; do
  VST_LN_CHAN=$v run 300 ln_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/ln_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'layernorm' in n})"; done
