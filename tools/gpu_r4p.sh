# round-4 GPU session p: full -m gpu suite + bench on the current build (fused temporal attention, packed GEGLU)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -60 gpurun_out/$log; exit $rc; fi
  return 0
}
run 900 r4p_pytest_gpu.log python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu
grep -E "FAILED|passed|failed" gpurun_out/r4p_pytest_gpu.log | tail -5
run 300 r4p_bench.json python -u bench.py --steps 10 --warmup 3 --no-peaks --no-vae
tail -c 400 gpurun_out/r4p_bench.json
