"""Tabulate tools/gemm_ablate.sh output: microseconds per (shape, ablation) for one tile code."""
import json
import sys

tile = sys.argv[2] if len(sys.argv) > 2 else "3"
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
shapes = []
for r in rows:
    if r["shape"] not in shapes:
        shapes.append(r["shape"])
abl = sorted({r["ablate"] for r in rows}, key=int)
print("shape".ljust(14), " ".join(("a" + a).rjust(7) for a in abl), " hipblaslt_tf  tf(a0)")
for s in shapes:
    d = {r["ablate"]: r for r in rows if r["shape"] == s}
    print(s.ljust(14), " ".join(str(d[a].get(f"t{tile}_us")).rjust(7) for a in abl), d["0"].get("hipblaslt_tf"),
          d["0"].get(f"t{tile}_tf"))
