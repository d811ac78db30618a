set -o pipefail
VST_GEMM_PERSIST=0 timeout -k 10 400 python -u tools/gemm_sweep.py > gpurun_out/sweep_p0.txt 2>&1 || exit 1
VST_GEMM_PERSIST=1 NO_BLAS=1 timeout -k 10 400 python -u tools/gemm_sweep.py > gpurun_out/sweep_p1.txt 2>&1 || exit 1
