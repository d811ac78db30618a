#!/bin/bash
# 128-row 4-wave ring tiles (2 workgroups per CU) against the 8-phase tiles on the one-round 16^2 shapes
mkdir -p gpurun_out
VST_TILE_AB_TILES="0:0,1:1,2:1,9:1,10:1" VST_TILE_AB_SHAPES="sp1280_out_lora,sp1280_ff2,sp1280_proj,sp640_out_lora,sp640_proj" \
  timeout -k 10 300 python -u tools/tile_ab.py > gpurun_out/r6_tile128_ab.txt 2>&1
rc=$?; cat gpurun_out/r6_tile128_ab.txt; exit $rc
