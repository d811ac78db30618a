#!/bin/bash
# round 5: loop ablations of the fused base + UnZipLoRA kernels (the LoRA launchers now take
# VST_GEMM_ABLATE in the diagnostics build): 0 = as built, 4 = no counted vmcnt waits, 1 = no loop DMAs, 16 = no
# fragment reads, 2 = no MFMAs (abl/libvst_trace.so), noepi = no epilogue (abl/libvst_noepi.so), prod = the product
# library.  Outputs of ablated arms are wrong by design; only the times are read.  Two alternations, best of each.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp VST_AB_SHAPES=out1280_lora,out640_lora,qkv1280_lora,qkv640_lora,xattn1280_lora,xattn640_lora,geglu1280
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -40 gpurun_out/$log; exit $rc; fi
  return 0
}
for p in 1 2; do
  VST_PH_CHILD=1 VST_P8_PH=2 run 240 r5abl_prod_$p.jsonl python -u tools/p8_ph_ab.py
  for a in 0 4 1 16 2; do
    VST_LIB_AB=abl/libvst_trace.so VST_GEMM_ABLATE=$a VST_PH_CHILD=1 VST_P8_PH=2 run 240 r5abl_a${a}_$p.jsonl python -u tools/p8_ph_ab.py
  done
  VST_LIB_AB=abl/libvst_noepi.so VST_GEMM_ABLATE=0 VST_PH_CHILD=1 VST_P8_PH=2 run 240 r5abl_anoepi_$p.jsonl python -u tools/p8_ph_ab.py
done
python - <<'PY'
import json, glob
res = {}
for f in sorted(glob.glob("gpurun_out/r5abl_*.jsonl")):
    a = f.split("r5abl_")[1].rsplit("_", 1)[0]
    for l in open(f):
        if not l.startswith("{"): continue
        d = json.loads(l)
        k = (d["shape"], a)
        res[k] = min(res.get(k, 1e9), d["us"])
arms = ("prod", "a0", "a4", "a1", "a16", "a2", "anoepi")
for s in sorted({k[0] for k in res}):
    print(json.dumps({"shape": s, **{a: res.get((s, a)) for a in arms}}))
PY
