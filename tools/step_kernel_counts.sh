#!/bin/bash
# Kernels inside one replayed denoise step: rocprofv3 kernel stats of bench.py at 5 and at 25 timed steps; the
# per-kernel call difference / 20 is what one graph replay launches (setup, capture and the instrumented step cancel).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 5 25; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/skc$n -o run -- \
    python -u bench.py --steps $n --warmup 2 --no-cpu-baseline --no-peaks --no-vae > gpurun_out/skc$n.json 2> gpurun_out/skc$n.err || { tail -5 gpurun_out/skc$n.err; exit 1; }
  S=$(find gpurun_out/skc$n -name '*kernel_stats.csv' | head -1)
  cp "$S" gpurun_out/skc_stats_$n.csv
  rm -rf gpurun_out/skc$n
done
python - <<'PY'
import csv
def load(n):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f"gpurun_out/skc_stats_{n}.csv"))}
a, b = load(5), load(25)
rows = []
for k in b:
    dc = b[k][0] - a.get(k, (0, 0))[0]
    dt = b[k][1] - a.get(k, (0, 0.0))[1]
    if dc > 0:
        rows.append((dt / 20 / 1e3, dc / 20, k.split("(")[0][:90]))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"per replayed step: {sum(r[1] for r in rows):.0f} launches, {tot/1e3:.2f} ms of kernel time")
for us, c, k in rows[:40]:
    print(f"{us:9.1f} us/step {c:7.1f} calls  {k}")
PY
