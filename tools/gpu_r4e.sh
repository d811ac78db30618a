# round-4 GPU session e: re-run of the tests that failed in d, shard diag of the rehearsal config
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 400 r4e_shard_diag.log python -u tools/shard_diag.py --frames 16 --size 256 --clips 2 --world 2
run 700 r4e_tests.log python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gemm_xattn_gpu.py "tests/test_parity_bf16_gpu.py::test_legacy_init_sdxl_f2_per_layer" "tests/test_training_gpu.py::test_unet_training_step_grads_vs_oracle" tests/test_rccl_gpu.py
