set -o pipefail
# A/B: current libvst_hip.so vs ab/libvst_old.so (same box, same process order)
timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/ab_new.txt 2>&1 || exit 1
VST_LIB_AB=ab/libvst_old.so timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/ab_old.txt 2>&1 || exit 1
timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/ab_new2.txt 2>&1 || exit 1
