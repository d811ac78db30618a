#!/bin/bash
# A/B of the self-attention kernel builds (the packed-f32 SLP codegen vs scalar VALU): each build
# in its own process (VST_LIB_AB), alternated 3 times; out_hash must be equal (bit-exact variants)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
out=gpurun_out/r6_sa_ab.txt
: > $out
for pass in 1 2 3; do
  for v in base noslp scalar; do
    if [ $v = base ]; then unset VST_LIB_AB; else export VST_LIB_AB=$PWD/build_ab/libvst_$v.so; fi
    SA_LABEL=$v VST_SA_SELF=1 timeout -k 10 120 python -u tools/sa_self_ab.py self32 self16 >> $out 2>/dev/null || { echo "fail $v"; exit 1; }
  done
done
unset VST_LIB_AB
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r6_sa_ab.txt") if l.startswith("{")]
best = collections.defaultdict(lambda: 1e9); hashes = collections.defaultdict(set)
for r in rows:
    k = (r["variant"], r["shape"]); best[k] = min(best[k], r["us"]); hashes[r["shape"]].add(r["out_hash"])
for k, v in sorted(best.items()): print("best", k, v)
print("bit-identical across builds:", {s: len(h) == 1 for s, h in hashes.items()})
PY
