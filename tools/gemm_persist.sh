set -o pipefail
timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/ps0.txt 2>&1 || exit 1
VST_GEMM_PERSIST=1 timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/ps1.txt 2>&1 || exit 1
VST_GEMM_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k gemm > gpurun_out/ps_t.log 2>&1; tail -1 gpurun_out/ps_t.log
