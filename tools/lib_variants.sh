#!/bin/bash
# Product-build variants of the library differing only in one source file's compile-time macros:
#   bash tools/lib_variants.sh gemm_p8 name:DEFINES ...   ->  abx/libvst_<name>.so
set -e
SRCF=$1; shift
mkdir -p abx/common
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 ${EXTRA_DEFS}"
for f in video_style_transfer_amd/csrc/*.hip; do
  b=$(basename ${f%.hip}); [ "$b" = "$SRCF" ] && continue
  /opt/rocm/bin/hipcc $F -c $f -o abx/common/$b.o &
done
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc $F $defs -c video_style_transfer_amd/csrc/$SRCF.hip -o abx/v_$name.o &
done
wait
for v in "$@"; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abx/common/*.o abx/v_$name.o -o abx/libvst_$name.so
  rm -f abx/v_$name.o
done
rm -rf abx/common
