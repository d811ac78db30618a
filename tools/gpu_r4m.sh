# round-4 GPU session m: full -m gpu suite on the current build (persistent grid default), epilogue ablation, bench
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
run 300 r4m_abl.log bash tools/p8_epi_ablate.sh run
tail -14 gpurun_out/r4m_abl.log
run 900 r4m_pytest_gpu.log python -u -m pytest -v -x --timeout 300 --timeout-method thread tests -m gpu
grep -E "FAILED|passed|failed" gpurun_out/r4m_pytest_gpu.log | tail -3
run 300 r4m_bench.json python -u bench.py --steps 10 --warmup 3 --no-peaks --no-vae
tail -c 600 gpurun_out/r4m_bench.json
