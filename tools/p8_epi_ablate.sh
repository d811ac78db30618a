# Diagnostics: what the 8-phase GEMM's epilogue costs.  Builds two ablated libraries next to the product one
# (abl/: -DVST_ABL_NOGELU = GEGLU without the GELU, -DVST_ABL_NOEPI = no epilogue at all, wrong outputs) on the CPU
# side:   bash tools/p8_epi_ablate.sh build
# and times the step's GEMM shapes with each (VST_LIB_AB) on the GPU:   bash tools/p8_epi_ablate.sh run
set -e
if [ "$1" = build ]; then
  mkdir -p abl
  for v in NOGELU NOEPI; do
    for f in gemm gemm_p8 gemm_big attention elementwise motion norm probe; do
      /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-function -DVST_ABL_$v \
        -c video_style_transfer_amd/csrc/$f.hip -o abl/${f}_$v.o &
    done
    wait
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abl/*_$v.o -o abl/libvst_$v.so
    rm -f abl/*_$v.o
  done
  exit 0
fi
for pass in 1 2; do
  for v in base NOGELU NOEPI; do
    if [ $v = base ]; then lib=""; else lib=abl/libvst_$v.so; fi
    VST_LIB_AB=$lib VST_PH_CHILD=1 VST_P8_PH=2 timeout -k 10 240 python -u tools/p8_ph_ab.py > gpurun_out/abl_${v}_$pass.jsonl
    echo "[abl] $v pass $pass done"
  done
done
python - <<'PY'
import json, glob
res = {}
for f in sorted(glob.glob("gpurun_out/abl_*.jsonl")):
    v = f.split("abl_")[1].rsplit("_", 1)[0]
    for l in open(f):
        d = json.loads(l)
        k = (d["shape"], v)
        res[k] = min(res.get(k, 1e9), d["us"])
for s in sorted({k[0] for k in res}):
    print(json.dumps({"shape": s, **{v: res.get((s, v)) for v in ("base", "NOGELU", "NOEPI")}}))
PY
