# round-4 GPU session abl: what the 2-interval k-loop waits on, on the diagnostics build (abl/libvst_trace.so, built
# with -DVST_P8_TRACE so VST_GEMM_ABLATE reaches the 8-phase kernel): 0 = as built, 4 = no counted vmcnt waits in the
# loop, 1 = no loop DMAs (operands of the first two k-tiles reused), 16 = no fragment reads, 2 = no MFMAs.  Results of
# the ablated runs are wrong by design; only the times are read.  tools/p8_ph_ab.py per shape, two alternations.
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
for p in 1 2; do
  for a in 0 4 1 16 2; do
    VST_LIB_AB=abl/libvst_trace.so VST_GEMM_ABLATE=$a VST_PH_CHILD=1 VST_P8_PH=2 run 240 abl_a${a}_$p.jsonl python -u tools/p8_ph_ab.py
  done
done
python - <<'PY'
import json, glob
res = {}
for f in sorted(glob.glob("gpurun_out/abl_a*.jsonl")):
    a = f.split("abl_a")[1].split("_")[0]
    for l in open(f):
        if not l.startswith("{"): continue
        d = json.loads(l)
        k = (d["shape"], a)
        res[k] = min(res.get(k, 1e9), d["us"])
for s in sorted({k[0] for k in res}):
    print(json.dumps({"shape": s, **{"abl" + a: res.get((s, a)) for a in ("0", "4", "1", "16", "2")}}))
PY
