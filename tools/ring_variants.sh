#!/bin/bash
# Product-build variants differing only in gemm_big.hip's compile-time macros: abx/libvst_<name>.so per "name:DEFINES".
set -e
mkdir -p abx/common
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950"
for f in video_style_transfer_amd/csrc/*.hip; do
  b=$(basename ${f%.hip}); [ "$b" = gemm_big ] && continue
  /opt/rocm/bin/hipcc $F -c $f -o abx/common/$b.o &
done
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc $F $defs -c video_style_transfer_amd/csrc/gemm_big.hip -o abx/r_$name.o &
done
wait
for v in "$@"; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abx/common/*.o abx/r_$name.o -o abx/libvst_$name.so
  rm -f abx/r_$name.o
done
rm -rf abx/common
