set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_gpu.py tests/test_kernels_gpu.py "tests/test_training_gpu.py::test_colsum" tests/test_frame_shard.py tests/test_bench_rehearsal.py > gpurun_out/r4a_tests.log 2>&1
