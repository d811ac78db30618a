# round-4 GPU session b1g: B1 fragments in J1's MFMA segment for every epilogue but GEGLU (GEGLU keeps the old placement)
# variant's tests, isolated A/B (tools/p8_ph_ab.py, old = HEAD via VST_LIB_AB), in-step bench A/B
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
run 400 b1g_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_lora_gpu.py tests/test_gemm_xattn_gpu.py -k "8phase or persistent or geglu or conv or temporal_attention or lora or xattn or gemm"
grep -E "passed|failed" gpurun_out/b1g_tests.log | tail -2
for v in old new old new; do
  if [ $v = old ]; then lib=abl/libvst_old.so; else lib=""; fi
  VST_LIB_AB=$lib run 300 b1g_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/b1g_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'gemm_p8' in n})"; done
