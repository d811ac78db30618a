# round-4 GPU session r: GEGLU epilogue without LDS staging (VST_P8_GEGLU_DIRECT) — bitwise test, isolated + in-step A/B
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
VST_P8_GEGLU_DIRECT=1 run 300 r4r_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "persistent or geglu"
grep -E "FAILED|passed|failed" gpurun_out/r4r_tests.log | tail -3
run 400 r4r_ab.txt python -u tools/p8_ph_ab.py 2 2+persist 2+persist+gd
grep bitwise gpurun_out/r4r_ab.txt | grep geglu | cut -c1-260
for v in 0 1 0 1; do
  VST_P8_GEGLU_DIRECT=$v run 300 r4r_bench_gd${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4r_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'geglu' in n})"; done
