#!/bin/bash
# round 6: XCD-local tile order A/B: the 8-phase grouped order with GROUP_M row panels per group
# (VST_GEMM_GROUP_M, read once per process; default 8), isolated launches + FETCH_SIZE per launch, then the step
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r6_group_ab.txt
: > $out
for g in 8 4 2 16 8 4; do
  echo "== GROUP_M=$g" >> $out
  VST_GEMM_GROUP_M=$g timeout -k 10 120 python -u tools/p8_one.py geglu1280 qkv1280 ff2_1280 qkv640_256 proj320 >> $out 2>&1 || exit 1
done
for g in 8 4 2; do
  VST_GEMM_GROUP_M=$g timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/grp_pmc_$g -o pmc -- python -u tools/p8_one.py geglu1280 qkv1280 > /dev/null 2>&1 || { echo "pmc $g failed"; exit 1; }
  python - "$g" >> $out <<'PY'
import csv, glob, sys, collections
g = sys.argv[1]
f = glob.glob(f"gpurun_out/grp_pmc_{g}/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for fn in f:
    for r in csv.DictReader(open(fn)):
        if r.get("Counter_Name") == "FETCH_SIZE":
            agg[r["Kernel_Name"].split("(")[0][-60:]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"PMC GROUP_M={g} {k}: {len(v)} launches, FETCH {2 * 1024 * sum(v) / len(v) / 1e6:.1f} MB per launch (x2 gfx950)")
PY
  rm -rf gpurun_out/grp_pmc_$g
done
for g in 8 4 8 4; do
  VST_GEMM_GROUP_M=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-vae --no-peaks > gpurun_out/grp_bench_$g.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/grp_bench_$g.json').read().strip().splitlines()[-1])
k=d['kernels']; print('STEP GROUP_M=$g', d['ms_per_step'], 'ms |', ' '.join(f'{n} {v[\"ms_per_step\"]:.2f}' for n, v in list(k.items())[:6]))" >> $out
done
cat $out
