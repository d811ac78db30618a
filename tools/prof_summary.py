"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite `*_results.db`, or a kernel_stats.csv) into the
per-kernel stats table committed under profiles/ (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs).  python tools/prof_summary.py gpurun_out/prof_X/run_results.db > profiles/rN_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, count(*), sum(end - start), min(end - start), max(end - start) "
                      "from kernels group by name").fetchall()
    return [(n, c, t, mn, mx) for n, c, t, mn, mx in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["MinNs"]), float(r["MaxNs"])))
    return out


def main():
    path = sys.argv[1]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    total = sum(r[2] for r in rows)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, c, t, mn, mx in sorted(rows, key=lambda r: -r[2]):
        w.writerow([n[:200], c, int(t), round(t / c, 1), round(100.0 * t / total, 3), int(mn), int(mx)])


if __name__ == "__main__":
    main()
