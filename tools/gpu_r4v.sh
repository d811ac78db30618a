# round-4 GPU session v: LayerNorm row passes per wave (VST_LN_RIT) now that gamma / beta come from LDS; in-step A/B
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
for v in 0 1 2 4 0 1 2 4; do
  if [ $v = 0 ]; then unset VST_LN_RIT; else export VST_LN_RIT=$v; fi
  run 300 r4v_bench_rit${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
unset VST_LN_RIT
for f in gpurun_out/r4v_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'layernorm' in n})"; done
