#!/bin/bash
# SQ counter passes over the spatial self-attention variants (tools/sa_self_ab.py self32 self16), one pass per run
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
out=gpurun_out/r5_sapmc.txt; : > $out
for v in ${SA_VARIANTS:-0 41}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    VST_SA_SELF=$v timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/sapmc$v$i -o a -- python -u tools/sa_self_ab.py self32 self16 > gpurun_out/sapmc$v$i.out 2> gpurun_out/sapmc$v$i.err || { tail -5 gpurun_out/sapmc$v$i.err; exit 1; }
    F=$(find gpurun_out/sapmc$v$i -name '*counter_collection.csv' | head -1)
    python - "$F" "$v" >> $out <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "spatial_attn" not in r["Kernel_Name"] and "sa_self" not in r["Kernel_Name"]:
        continue
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    agg[grid][r["Counter_Name"]].append(float(r["Counter_Value"]))
for grid, cs in agg.items():
    print("variant", sys.argv[2], "grid", grid, {k: round(sum(v) / len(v)) for k, v in cs.items()})
PY
    rm -rf gpurun_out/sapmc$v$i
  done
done
cat $out
