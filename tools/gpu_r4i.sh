# rocprof kernel stats of the headline bench command (csv summaries only)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_prof -o r4i -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vae --no-peaks > gpurun_out/r4i_rocprof.log 2>&1
rc=$?; echo "rc=$rc"
mkdir -p gpurun_out/r4i_keep
for f in $(find gpurun_out/r4i_prof -name "*stats.csv"); do cp $f gpurun_out/r4i_keep/; done
python - <<'PY'
import csv, glob
tr = glob.glob("gpurun_out/r4i_prof/**/*kernel_trace.csv", recursive=True)
if tr:
    rows = list(csv.DictReader(open(tr[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the 5 timed replays are the last 5 x (launches per step) dispatches before the instrumented eager step
    t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
    gaps = [t[i + 1][0] - t[i][1] for i in range(len(t) - 1)]
    busy = sum(e - s for s, e, _ in t)
    print("dispatches", len(t), "busy_ms", busy / 1e6, "span_ms", (t[-1][1] - t[0][0]) / 1e6)
    import statistics
    small = [g for g in gaps if 0 <= g < 100000]
    print("gaps<100us: n", len(small), "sum_ms", sum(small) / 1e6, "median_us", statistics.median(small) / 1e3 if small else None)
    open("gpurun_out/r4i_keep/trace_head.txt", "w").write("\n".join(f"{s} {e} {n}" for s, e, n in t[-4000:]))
PY
rm -rf gpurun_out/r4i_prof
ls -la gpurun_out/r4i_keep
