#!/bin/bash
# SQ counter passes over isolated 8-phase GEMM shapes (tools/p8_one.py): MFMA busy vs wave cycles, LDS
# activity and bank conflicts.  Via gpurun; one --pmc pass per counter group.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/gpmc$i -o g -- python -u tools/p8_one.py proj1280 geglu1280 qkv1280 proj320 > gpurun_out/gpmc$i.out 2> gpurun_out/gpmc$i.err || { tail -5 gpurun_out/gpmc$i.err; exit 1; }
  F=$(find gpurun_out/gpmc$i -name '*counter_collection.csv' | head -1)
  python - "$F" <<'PY' | tee -a gpurun_out/p8_pmc.txt
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_p8" not in r["Kernel_Name"]:
        continue
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    name = r["Kernel_Name"].split("(")[0].replace("void vst::", "")
    agg[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, grid), cs in agg.items():
    print(name, "grid", grid, {k: round(sum(v) / len(v)) for k, v in cs.items()})
PY
  rm -rf gpurun_out/gpmc$i
done
