#!/bin/bash
# Same-box A/B of the whole denoise step over library builds (round 5): bash tools/gpu_r5_stepab.sh base new xu ...
# "new" = the in-tree .so, any other name = abl/libvst_<name>.so.  Builds alternate in the order given.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
i=0
for tag in "$@"; do
  i=$((i+1))
  unset VST_P8_320 VST_SA_SELF VST_GN_COLSTAT VST_P8_LORA_PERSIST
  base=$tag
  if [ "$tag" = new320 ]; then export VST_P8_320=1; base=new; fi  # 128x320 tiles where their rounds win (opt-in)
  if [ "$tag" = sa0 ]; then export VST_SA_SELF=0; base=new; fi  # self-attention on spatial_attn_kernel<0>
  if [ "$tag" = gn1 ]; then export VST_GN_COLSTAT=1; base=new; fi  # GroupNorm statistics from conv column statistics
  if [ "$tag" = lp0 ]; then export VST_P8_LORA_PERSIST=0; base=new; fi  # in-GEMM LoRA one workgroup per tile
  if [ "$tag" = n320 ]; then export VST_P8_320N=1; base=new; fi  # 128x320 tiles for the narrow 32x32 / 64x64 GEMMs
  if [ "$base" = new ]; then unset VST_LIB_AB; else export VST_LIB_AB=abl/libvst_$base.so; fi
  timeout -k 10 300 python -u bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-peaks --no-vae \
    > gpurun_out/stepab_${i}_$tag.json 2> gpurun_out/stepab_${i}_$tag.err || { tail -20 gpurun_out/stepab_${i}_$tag.err; exit 1; }
  python - "gpurun_out/stepab_${i}_$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "|", "  ".join(f"{n} {v['ms_per_step']:.2f}" for n, v in list(k.items())[:8]), flush=True)
print("   fused:", {s: v["us_per_launch"] for s, v in d["roofline"]["fused_lora_gemms"].items()}, flush=True)
PY
done
