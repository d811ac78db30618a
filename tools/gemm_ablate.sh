set -o pipefail
# VST_GEMM_ABLATE bits: 1 no loop DMA, 2 no MFMA, 8 no epilogue, 16 no fragment ds_reads
for a in ${ABL:-0 1 2 3 8 11 19 27}; do VST_GEMM_ABLATE=$a timeout -k 10 120 python -u tools/gemm_ablate.py || exit 1; done
