# round-4 GPU session c: shard mismatch diagnosis, RCCL capture diagnosis, eager-vs-graph step, GEMM A/B in isolation
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
run 400 r4c_shard_diag.log python -u tools/shard_diag.py --frames 16 --size 256 --clips 2 --world 2
run 400 r4c_piecewise.log python -u -m pytest -v --timeout 300 --timeout-method thread "tests/test_frame_shard.py::test_frame_shard_piecewise_graph_two_ranks_one_gpu" tests/test_bench_rehearsal.py
run 500 r4c_ph_ab.log python -u tools/p8_ph_ab.py 2 3 2 3+320 2+320
run 300 r4c_bench_eager.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae --no-graph --no-roofline
run 300 r4c_bench_graph.json python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks --no-vae --no-roofline
run 300 r4c_rccl_diag.log python -u tools/rccl_diag.py ar ag a2a
