# round-4 GPU session z: persistent GEGLU bias brought into LDS by the k-loop (no global bias wait in the epilogue)
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
run 300 r4z_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "persistent or geglu or 8phase"
grep -E "FAILED|passed|failed" gpurun_out/r4z_tests.log | tail -3
for v in old new old new; do
  if [ $v = old ]; then lib=abl/libvst_old.so; else lib=""; fi
  VST_LIB_AB=$lib VST_PH_CHILD=1 VST_P8_PH=2 run 240 r4z_iso_${v}_$RANDOM.jsonl python -u tools/p8_ph_ab.py
done
for v in old new old new; do
  if [ $v = old ]; then lib=abl/libvst_old.so; else lib=""; fi
  VST_LIB_AB=$lib run 300 r4z_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4z_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'persist' in n})"; done
