#!/bin/bash
# Diagnostics builds of the library that differ only in gemm_p8.hip's compile-time variant macros, all with the
# per-workgroup timeline (VST_P8_TRACE): abx/libvst_<name>.so for each "name:DEFINES" argument.
# e.g. bash tools/p8_variants.sh base: fast:-DVST_P8_FASTDMA
set -e
mkdir -p abx/common
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -DVST_P8_TRACE -DVST_GEMM_DIAG"
for f in video_style_transfer_amd/csrc/*.hip; do
  b=$(basename ${f%.hip}); [ "$b" = gemm_p8 ] && continue
  /opt/rocm/bin/hipcc $F -c $f -o abx/common/$b.o &
done
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc $F $defs -c video_style_transfer_amd/csrc/gemm_p8.hip -o abx/p8_$name.o &
done
wait
for v in "$@"; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abx/common/*.o abx/p8_$name.o -o abx/libvst_$name.so
  rm -f abx/p8_$name.o
done
rm -rf abx/common
