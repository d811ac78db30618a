# round-4: the parity gates of the final build with their printed floors / yardsticks (-s), and the training bench
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # run <limit> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[step] $log rc=$rc"
  if [ $rc -ne 0 ]; then echo "[step] stopping after rc=$rc"; tail -20 gpurun_out/$log; exit $rc; fi
  return 0
}
run 900 r4_parity_gpu.log python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_parity_bf16_gpu.py tests/test_parity_gpu.py tests/test_training_gpu.py tests/test_text_encoder_gpu.py tests/test_frame_shard.py -m gpu
grep -E "FAILED|passed|failed" gpurun_out/r4_parity_gpu.log | tail -3
run 600 r4_bench_train.json python -u bench.py --train
tail -c 300 gpurun_out/r4_bench_train.json
