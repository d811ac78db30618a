# round-4 GPU session b1: B1 fragments read inside J1's MFMA segment (B1 DMA one interval earlier); every 8-phase
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
run 400 b1_tests.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_lora_gpu.py tests/test_gemm_xattn_gpu.py -k "8phase or persistent or geglu or conv or temporal_attention or lora or xattn or gemm"
grep -E "passed|failed" gpurun_out/b1_tests.log | tail -2
for v in old new old new; do
  if [ $v = old ]; then lib=abl/libvst_old.so; else lib=""; fi
  VST_LIB_AB=$lib VST_PH_CHILD=1 VST_P8_PH=2 run 240 b1_iso_${v}_$RANDOM.jsonl python -u tools/p8_ph_ab.py
done
python - <<'PY'
import json, glob
res = {}
for f in sorted(glob.glob("gpurun_out/b1_iso_*.jsonl")):
    v = f.split("_iso_")[1].split("_")[0]
    for l in open(f):
        if not l.startswith("{"): continue
        d = json.loads(l); res.setdefault((d["shape"], v), []).append((d["us"], d["md5"]))
for s in sorted({k[0] for k in res}):
    o, n = res[(s, "old")], res[(s, "new")]
    print(f"{s:14s} old {min(x[0] for x in o):8.2f} new {min(x[0] for x in n):8.2f} md5eq {o[0][1] == n[0][1]}")
PY
for v in old new old new; do
  if [ $v = old ]; then lib=abl/libvst_old.so; else lib=""; fi
  VST_LIB_AB=$lib run 300 b1_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/b1_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'gemm_p8' in n})"; done
