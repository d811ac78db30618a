# round-4 GPU session f: SDXL training-gradient accuracy with / without the in-GEMM LoRA (shape-only policy)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in 1 0; do
  VST_LORA_INGEMM=$v timeout -k 10 400 python -u -m pytest -v -s --timeout 380 --timeout-method thread "tests/test_training_gpu.py::test_unet_training_step_grads_vs_oracle[sdxl]" > gpurun_out/r4f_train_ingemm$v.log 2>&1
  rc=$?; echo "[step] ingemm=$v rc=$rc"; grep "\[train\] sdxl:" gpurun_out/r4f_train_ingemm$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 400 python -u tools/shard_diag.py --frames 16 --size 256 --clips 2 --world 2 > gpurun_out/r4f_shard_diag.log 2>&1
rc=$?; echo "[step] shard_diag rc=$rc"; grep -v "Gloo\|amdgpu.ids\|socket.cpp" gpurun_out/r4f_shard_diag.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_bench_rehearsal.py tests/test_frame_shard.py > gpurun_out/r4f_shard_tests.log 2>&1
rc=$?; echo "[step] shard tests rc=$rc"; grep -E "PASSED|FAILED|\[shard\]|\[rehearsal\]" gpurun_out/r4f_shard_tests.log | tail -12
