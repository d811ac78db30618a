# round-4 GPU session n: persistent-grid stagger A/B (VST_P8_STAGGER), in isolation and in the step
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -40 gpurun_out/$log; exit $rc; fi
  return 0
}
run 500 r4n_ab.txt python -u tools/p8_ph_ab.py 2 2+persist 2+persist+st1 2+persist+st2
grep bitwise gpurun_out/r4n_ab.txt | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], {k[3:]: v for k, v in d.items() if k.startswith('us_')})"
for v in 0 1 0 1; do
  VST_P8_STAGGER=$v run 300 r4n_bench_st${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
for f in gpurun_out/r4n_bench_*.json; do python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', d['ms_per_step'])"; done
