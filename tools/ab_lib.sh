#!/bin/bash
# Build the committed (HEAD) sources into abx/libvst_old.so for same-box A/B runs (VST_LIB_AB=abx/libvst_old.so).
set -e
mkdir -p abx/src
for f in video_style_transfer_amd/csrc/*; do git show HEAD:$f > abx/src/$(basename $f) 2>/dev/null || cp $f abx/src/; done
for f in abx/src/*.hip; do /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -c $f -o ${f%.hip}.o & done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abx/src/*.o -o abx/libvst_old.so
rm -rf abx/src
