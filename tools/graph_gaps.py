"""Idle time between kernels inside the replayed denoise-step graph, from a rocprofv3 --kernel-trace CSV:
per step (pack_latents_kernel opens a step, step_advance_kernel closes it): span, summed kernel time, the
union of kernel intervals, and the gaps between consecutive kernels.
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- python bench.py --steps 5 --warmup 2 ...
  python tools/graph_gaps.py gpurun_out/gaps"""
import csv
import glob
import os
import sys

import numpy as np


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
    en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
    starts = [i for i, n in enumerate(names) if "pack_latents_kernel" in n]
    ends = [i for i, n in enumerate(names) if "step_advance_kernel" in n]
    out = []
    for s in starts:
        e = next((j for j in ends if j > s), None)
        if e is None:
            continue
        seg = slice(s, e + 1)
        a, b = st[seg], en[seg]
        span = (b.max() - a.min()) / 1e3
        busy = 0
        cur_s, cur_e = a[0], b[0]
        for x, y in zip(a[1:], b[1:]):
            if x > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = x, y
            else:
                cur_e = max(cur_e, y)
        busy += cur_e - cur_s
        gaps = np.maximum(a[1:] - np.maximum.accumulate(b[:-1]), 0) / 1e3
        out.append((e - s + 1, span, (b - a).sum() / 1e3, busy / 1e3, np.median(gaps), np.percentile(gaps, 90)))
    for n, span, ksum, busy, g50, g90 in out:
        print(f"step: {n} kernels, span {span / 1e3:.2f} ms, kernel sum {ksum / 1e3:.2f} ms, busy {busy / 1e3:.2f} ms, "
              f"idle {(span - busy) / 1e3:.2f} ms, gap p50 {g50:.2f} us p90 {g90:.2f} us")


if __name__ == "__main__":
    main()
