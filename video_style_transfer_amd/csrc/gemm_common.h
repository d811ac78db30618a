// Shared GEMM argument block and LDS swizzle (gemm.hip, gemm_big.hip).
#pragma once
#include "vst_common.h"

namespace vst {

struct GemmArgs {
  const bf16_t* A1; const bf16_t* A2;
  int lda1, lda2, K1;
  // conv geometry (AMODE 1/2): input NHWC [nimg, H, W, C1 (+C2)] -> output [nimg, OH, OW, N]
  int H, W, C1, C2, OH, OW, stride, up;
  int pad0;  // 1: no top/left padding (F.pad (0,1,0,1) + stride-2 conv of diffusers Downsample2D(padding=0))
  const bf16_t* Wt; int ldw;
  int M, N, K;
  const float* bias;
  const float* rbias; int rbias_div, ldrb;
  const bf16_t* R; int ldr;
  bf16_t* C; int ldc;
  float* ws;  // split-K slabs [splits][M][N] fp32
  int splits;
  int act;     // EPI 0 only: 1 = GELU(erf) after the bias (TemporalTransformerBlock ffn, no residual / row bias)
  int persist;  // > 0: persistent launch over `persist` CUs (VST_GEMM_PERSIST; 0 = one workgroup per tile)
  int group_m;  // grouped tile order: row panels per group (0 = default 8; VST_GEMM_GROUP_M for tuning)
  int p8_bn;   // 8-phase kernel tile width: 0 / 256 or 192 (gemm_p8.hip)
  int ablate;  // diagnostics only (VST_GEMM_ABLATE): bit0 skip loop DMA, bit1 skip MFMA
  uint32_t a1_bytes, a2_bytes, w_bytes, r_bytes;
  // in-GEMM LoRA down-projection (gemm_p8.hip LORA, vst_gemm_lora): Acat [la_p][K] bf16 (row stride lda_la); the
  // output columns of group g = n / la_gn use u columns [g la_gr, (g + 1) la_gr), whose up-projection sits in W's
  // columns K + that range (ldw >= K + la_p); wtail_bytes covers those columns
  const bf16_t* la;
  int lda_la, la_p, la_gn, la_gr;
  uint32_t la_bytes, wtail_bytes;
  // cross-attention epilogue (gemm_p8.hip EPI 4, vst_gemm_cross_attention): the GEMM output is the q of a
  // BasicTransformerBlock's attn2; instead of storing it, each tile writes softmax(q K^T scale) V of its heads over
  // the xa_nk text keys of text batch (m / xa_nq) / xa_kvdiv (K/V rows [batch * xa_nk + key], row stride xa_ldkv)
  const bf16_t* xa_k;
  const bf16_t* xa_v;
  int xa_ldkv, xa_nk, xa_nq, xa_kvdiv;
  float xa_scale_log2;
  uint32_t xa_kv_bytes;
  // temporal attention epilogue (gemm_p8.hip EPI 5, vst_gemm_temporal_attention): frames per clip 16, head dim ta_d
  // (40: two heads per 256-column tile, 80: one); ta_hw pixels per frame; the output O [M, ta_heads * ta_d]
  // (p.C / p.ldc) is written in (clip, frame, pixel) rows
  int ta_hw, ta_heads, ta_d;
  float ta_scale_log2;
  // GroupNorm column statistics of the stored output (tile_epilogue EPI 0 on 128x320 tiles, vst_conv3x3_colstat):
  // colstat[m_tile][N] = (sum, sum of squares) over the tile's rows of the bf16 values written to C, fp32
  float* colstat;
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

}  // namespace vst
