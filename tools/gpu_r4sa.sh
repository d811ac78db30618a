# round-4 GPU session sa: spatial self-attention K/V through a 2-slot LDS-DMA ring (PRE = -1) instead of register
# staging; ring4 = the in-tree build (4 waves/SIMD, 3 VGPR spills), ring3 = abl/libvst_ring3.so (3 waves/SIMD, no
# spills), reg = VST_SA_RING=0.  Tests, isolated timings (tools/attn_bench.py), in-step bench A/B.
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
run 300 sa_tests4.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "spatial_attention"
VST_LIB_AB=abl/libvst_ring3.so run 300 sa_tests3.log python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "spatial_attention"
grep -E "passed|failed" gpurun_out/sa_tests*.log
for p in 1 2; do
  VST_SA_RING=0 run 120 sa_iso_reg_$p.txt python -u tools/attn_bench.py self16 self32
  VST_SA_RING=16 run 120 sa_iso_ring4_$p.txt python -u tools/attn_bench.py self16 self32
  VST_SA_RING=16 VST_LIB_AB=abl/libvst_ring3.so run 120 sa_iso_ring3_$p.txt python -u tools/attn_bench.py self16 self32
done
for f in gpurun_out/sa_iso_*.txt; do echo "== $f"; cat $f; done
for v in reg ring4 ring3 reg ring4 ring3; do
  lib=""; ring=8
  if [ $v = reg ]; then ring=0; fi
  if [ $v = ring3 ]; then lib=abl/libvst_ring3.so; fi
  VST_SA_RING=$ring VST_LIB_AB=$lib run 300 sa_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/sa_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); k=d['kernels']; print('$f', d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'attn' in n})"; done
