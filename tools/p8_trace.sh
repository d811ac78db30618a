#!/bin/bash
# Build the diagnostics variant of the library with per-workgroup timestamps in the 8-phase GEMM (abx/libvst_trace.so).
set -e
mkdir -p abx/trace
for f in video_style_transfer_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -DVST_P8_TRACE -c $f -o abx/trace/$(basename ${f%.hip}).o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 abx/trace/*.o -o abx/libvst_trace.so
rm -rf abx/trace
