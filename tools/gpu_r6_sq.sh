#!/bin/bash
# SQ counters of the 16^2 out-projection + UnZipLoRA and the 16^2 GEGLU in isolation, one pass per set
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r6_sq_gemm.txt
: > $out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/sq_$i -o sq -- python -u tools/sq_gemm.py > gpurun_out/sq_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_$i.log; exit 1; }
  python - $i >> $out <<'PY'
import csv, glob, sys, collections
i = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob(f"gpurun_out/sq_{i}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0]
        if "gemm_p8" in k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v[2:]) / max(1, len(v) - 2)) for c, v in sorted(d.items())})
PY
  rm -rf gpurun_out/sq_$i
done
cat $out
