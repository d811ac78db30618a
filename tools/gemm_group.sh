set -o pipefail
for g in 8 4 16 32 2; do VST_GEMM_GROUP_M=$g timeout -k 10 150 python -u tools/gemm_ablate.py > gpurun_out/grp_$g.txt 2>&1 || exit 1; done
