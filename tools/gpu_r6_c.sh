#!/bin/bash
# round 6: the gradient gates with the split-K probe yardstick, then the idle time inside the replayed step graph
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -30 gpurun_out/$log; exit $rc; fi
  return 0
}
run 180 r6_fetch_probe.txt python -u tools/fetch_probe.py
cat gpurun_out/r6_fetch_probe.txt
run 600 r6_train_grads.log python -u -m pytest tests/test_training_gpu.py -k grads_vs_oracle -m gpu -v -s -rA --timeout 500 --timeout-method thread
grep -E "gates|probe|median" gpurun_out/r6_train_grads.log | head
run 400 r6_gaps_prof.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_gaps -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vae --no-peaks --no-roofline
python tools/graph_gaps.py gpurun_out/r6_gaps > gpurun_out/r6_graph_gaps.txt 2>&1; tail -15 gpurun_out/r6_graph_gaps.txt
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r6_gaps/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# one replayed step: between the last two pack_latents launches
idx = [i for i, r in enumerate(rows) if "pack_latents_kernel" in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
seg = rows[s:e]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
prev_end = None
for r in seg:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0][:90]
    a = agg[k]; a[0] += 1; a[1] += (en - st) / 1e3
    if prev_end is not None: a[2] += max(st - prev_end, 0) / 1e3
    prev_end = max(prev_end or 0, en)
with open("gpurun_out/r6_step_kernels.txt", "w") as o:
    tot = sum(v[1] for v in agg.values()); gap = sum(v[2] for v in agg.values())
    o.write(f"one replayed step: {len(seg)} launches, kernel time {tot/1e3:.3f} ms, gaps before launches {gap/1e3:.3f} ms\n")
    for k, (n, t, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        o.write(f"{t/1e3:8.3f} ms {n:5d}x  gap-before {g/1e3:7.3f} ms  {k}\n")
PY
head -30 gpurun_out/r6_step_kernels.txt
rm -rf gpurun_out/r6_gaps
