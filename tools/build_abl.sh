#!/bin/bash
# Diagnostics builds for the loop ablations (VST_GEMM_ABLATE reaches the 8-phase kernel only with -DVST_P8_TRACE):
#   abl/libvst_trace.so  -- every source with -DVST_P8_TRACE
#   abl/libvst_noepi.so  -- the same, gemm_p8.hip also with -DVST_ABL_NOEPI (no epilogue of any kind)
set -e
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -DVST_P8_TRACE"
mkdir -p abl/o
for f in video_style_transfer_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc $F -c $f -o abl/o/$(basename ${f%.hip}).o &
done
/opt/rocm/bin/hipcc $F -DVST_ABL_NOEPI -c video_style_transfer_amd/csrc/gemm_p8.hip -o abl/o/gemm_p8_noepi.x &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abl/o/*.o -o abl/libvst_trace.so
mv abl/o/gemm_p8.o abl/o/gemm_p8.keep
cp abl/o/gemm_p8_noepi.x abl/o/gemm_p8_noepi.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abl/o/*.o -o abl/libvst_noepi.so
rm -rf abl/o
