# SQ counter passes over the spatial attention forward (self32, self16).  Via gpurun.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/apmc$i -o a -- python -u tools/attn_bench.py self32 self16 > gpurun_out/apmc$i.out 2> gpurun_out/apmc$i.err || { tail -5 gpurun_out/apmc$i.err; exit 1; }
  F=$(find gpurun_out/apmc$i -name '*counter_collection.csv' | head -1)
  python - "$F" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "spatial_attn" not in r["Kernel_Name"]:
        continue
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    agg[grid][r["Counter_Name"]].append(float(r["Counter_Value"]))
for grid, cs in agg.items():
    print("grid", grid, {k: round(sum(v) / len(v)) for k, v in cs.items()})
PY
  rm -rf gpurun_out/apmc$i
done
