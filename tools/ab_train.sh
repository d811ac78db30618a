#!/bin/bash
# Same-box A/B of the training step (bench.py --train): bash tools/ab_train.sh new old new2 old2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in "$@"; do
  base=$(echo $tag | sed 's/[0-9]*$//')
  if [ "$base" = new ]; then unset VST_LIB_AB; else export VST_LIB_AB=abx/libvst_$base.so; fi
  timeout -k 10 300 python -u bench.py --train --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/abt_$tag.json 2> gpurun_out/abt_$tag.err || { tail -20 gpurun_out/abt_$tag.err; exit 1; }
  python - "$tag" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/abt_{sys.argv[1]}.json"))
k = d["kernels"]
print(sys.argv[1], "ms/step", d["ms_per_step"], "|", "  ".join(f"{n} {v['ms_per_step']:.2f}" for n, v in list(k.items())[:5]))
PY
done
