# round-4 GPU session b: new tests + p8 schedule / tile A/B.  Each step under its own limit; a timeout / abort / fault
# ends the script (test failures, exit 1, do not).
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 900 r4b_tests.log python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_lora_gpu.py "tests/test_training_gpu.py::test_colsum" tests/test_frame_shard.py tests/test_bench_rehearsal.py
run 500 r4b_ph_ab.log python -u tools/p8_ph_ab.py 2 3 2 3+320 2+320
for v in 3 2 3+320 2+320 3 2 3+320 2+320; do
  VST_P8_PH=${v%%+*} VST_P8_320=$([ "$v" != "${v%+320}" ] && echo 1 || echo 0) run 300 r4b_bench_${v}_$RANDOM.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae
done
run 300 r4b_rccl.log python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_rccl_gpu.py
for f in gpurun_out/r4b_bench_*.json; do python -c "import sys,json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['kernel_time_ms_per_step'])"; done
