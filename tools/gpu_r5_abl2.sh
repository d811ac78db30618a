#!/bin/bash
# round 5: operand-traffic ablations (diagnostics build): 0 as built, 64 no W-operand DMAs / fragment reads in the
# loop, 128 no A-operand ones, 16 no fragment reads at all, 1 no loop DMAs.  Times only (outputs wrong by design).
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp VST_AB_SHAPES=out1280_lora,qkv1280_lora,xattn1280_lora,geglu1280,ff2_1280
run() {
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then tail -40 gpurun_out/$log; exit $rc; fi
}
for p in 1 2; do
  for a in 0 64 128 16 1; do
    VST_LIB_AB=abl/libvst_trace.so VST_GEMM_ABLATE=$a VST_PH_CHILD=1 VST_P8_PH=2 run 240 r5abl2_a${a}_$p.jsonl python -u tools/p8_ph_ab.py
  done
done
python - <<'PY'
import json, glob
res = {}
for f in sorted(glob.glob("gpurun_out/r5abl2_*.jsonl")):
    a = f.split("r5abl2_")[1].rsplit("_", 1)[0]
    for l in open(f):
        if not l.startswith("{"): continue
        d = json.loads(l)
        res[(d["shape"], a)] = min(res.get((d["shape"], a), 1e9), d["us"])
for s in sorted({k[0] for k in res}):
    print(json.dumps({"shape": s, **{a: res.get((s, a)) for a in ("a0", "a64", "a128", "a16", "a1")}}))
PY
