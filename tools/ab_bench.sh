#!/bin/bash
# Same-box A/B of the denoise step over library builds: bash tools/ab_bench.sh new nofast old ...
# "new" = the in-tree .so, any other name = abx/libvst_<name>.so (tools/ab_lib.sh, tools/ring_variants.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in "$@"; do
  base=$(echo $tag | sed 's/[0-9]*$//')  # trailing digits: repeats of the same build
  unset VST_GEMM_P8
  unset VST_LN_GENERIC VST_P8_BN VST_CFG_STREAMS VST_LORA_INGEMM VST_XATTN_FUSE VST_LN_RIT VST_MOTION_FUSE
  if [ "$base" = motionfuse ]; then export VST_MOTION_FUSE=1; base=new; fi  # fused motion attention blocks (opt-in)
  if [ "$base" = lnritx ]; then export VST_LN_RIT=2; base=new; fi  # LayerNorm: 2 row passes per wave at every C
  if [ "$base" = lnrity ]; then export VST_LN_RIT=1; base=new; fi  # LayerNorm: 1 row pass per wave at every C
  if [ "$base" = noxattn ]; then export VST_XATTN_FUSE=0; base=new; fi  # attn2 as q GEMM + attention kernel
  if [ "$base" = nolora ]; then export VST_LORA_INGEMM=0; base=new; fi  # LoRA down-projection as its own pass
  if [ "$base" = cfgstreams ]; then export VST_CFG_STREAMS=1; base=new; fi  # CFG branches on two streams (B=1 each)
  if [ "$base" = bnall ]; then export VST_P8_BN=192; base=new; fi  # 256x192 tiles for every non-GEGLU 8-phase GEMM
  if [ "$base" = lngen ]; then export VST_LN_GENERIC=1; base=new; fi  # the generic LayerNorm kernel only
  if [ "$base" = newall ]; then export VST_GEMM_P8=1; base=new; fi  # the 8-phase kernel for every shape
  if [ "$base" = new ]; then unset VST_LIB_AB; else export VST_LIB_AB=abx/libvst_$base.so; fi
  VST_BENCH_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
  python - "$tag" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
k = d["kernels"]
print(sys.argv[1], "ms/step", d["ms_per_step"], "|", "  ".join(f"{n} {v['ms_per_step']:.2f}" for n, v in list(k.items())[:6]))
print("   fused:", {s: v["ms_per_step"] for s, v in d["roofline"]["fused_lora_gemms"].items()})
PY
done
