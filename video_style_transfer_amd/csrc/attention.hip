// Attention cores of the AnimateDiff-XL denoise path.
//
// 1) vst_spatial_attention: softmax(Q K^T / sqrt(64)) V per (frame, head), head_dim 64.
//    Replaces F.scaled_dot_product_attention in AnimateDiffAttnProcessor2_0.__call__
//    (animatediff/attention_processor.py:78-80).  Self-attention (Nk = Nq = H*W) and
//    cross-attention over the text tokens.  The processor's repeat_interleave of the
//    text states to B*F (:63-66) is replaced by indexing: K/V row batch = frame / kv_div,
//    so the text K/V projection runs once per clip instead of once per frame.
//    Flash-style: 4 waves x 32 queries; 64-key K/V tiles double-buffered in LDS;
//    S^T = K.Q^T on v_mfma_f32_16x16x32_bf16 so each lane owns one query column and the
//    softmax row state is lane-local (2 cross-lane shuffles per reduction);
//    O^T = V^T.P^T with V^T fragments from ds_read_b64_tr_b16 transposed LDS reads and
//    P^T fed straight from the S^T accumulators (no LDS round trip for P).
//
// 2) vst_temporal_attention: self-attention across the frame axis for every spatial
//    position (the motion-module attention core: diffusers AnimateDiffTransformer3D /
//    the reference's TemporalTransformerBlock, animatediff/temporal_transformer.py:66-68).
//    Tokens stay in the spatial layout [(b*F + f)*HW + p, C]; the kernel reads the frame
//    axis with stride HW rows, so no permute/contiguous copies are made on either side.
//    One wave per (b, p, head); F <= 32; head_dim = C/8 (40/80/160 for SDXL).
#include "attn_common.h"

namespace vst {

constexpr int SA_KT = 64;                         // keys per tile
constexpr int SA_TILE = SA_KT * 64 * 2;           // 8 KiB
constexpr int SA_LDS = 4 * SA_TILE;               // K,V double-buffered

typedef __attribute__((address_space(3))) void sa_lds_void;

// One 1-KiB LDS-DMA piece: 64 lanes x 16 B, lane-linear in LDS at `lds_piece` (wave-uniform).
__device__ __forceinline__ void sa_dma16(__amdgpu_buffer_rsrc_t r, char* lds_piece, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (sa_lds_void*)((__attribute__((address_space(3))) char*)(uintptr_t)lds_piece), 16, off, 0, 0, 0);
}

// PRE = 0: K/V tiles of 64 keys double-buffered through registers (long key ranges: the 32x32 / 64x64 levels).
// PRE = n (1..4, Nk <= 64 n): the whole K/V of the (batch, head) is brought into LDS up front by LDS-DMA -- every
// load of the workgroup in flight at once, no per-tile barrier -- for the 77 text tokens of cross-attention, where
// the short key loop left one HBM latency exposed per tile (dispatch: up to two tiles, see vst_spatial_attention).  The DMA writes each
// 8-row piece lane-linearly, so each lane fetches the global chunk that the tile's swizzle (k_off / v_off) puts at
// its LDS slot.
template <int PRE>
__global__ __launch_bounds__(256, 2) void spatial_attn_kernel(
    const bf16_t* __restrict__ Q, int ldq, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldkv,
    bf16_t* __restrict__ O, int ldo, int nbatch, int heads, int Nq, int Nk, int kv_div, float scale_log2,
    uint32_t q_bytes, uint32_t kv_bytes, float* __restrict__ lse, int causal = 0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nqb = (Nq + 127) / 128;
  const int wg = xcd_remap(blockIdx.x, nqb * heads * nbatch);
  const int qblk = wg % nqb;
  const int bh = wg / nqb;
  const int h = bh % heads, b = bh / heads;
  const int bkv = b / kv_div;
  const int fr = lane & 15, g = lane >> 4;

  const auto rq = make_rsrc(Q, q_bytes);
  const auto rk = make_rsrc(K, kv_bytes);
  const auto rv = make_rsrc(V, kv_bytes);

  // Q^T fragments (B operand of S^T = K.Q^T): lane (col q, group g) holds Q[q][32kk + 8g .. +7]
  bf16x8 qf[2][2];
  const int qbase = qblk * 128 + wid * 32;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qbase + qb * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int off = q < Nq ? ((b * Nq + q) * ldq + h * 64 + kk * 32 + g * 8) * 2 : kOOB;
      qf[qb][kk] = __builtin_bit_cast(bf16x8, buf_load16(rq, off));
    }
  }

  // K/V staging: 64 rows x 8 chunks = 512 chunks per tile; 2 per thread per operand
  const int sc = tid & 7, sr = tid >> 3;  // rows sr, sr+32
  u32x4 kreg[2], vreg[2];
  auto load_kv = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = t * SA_KT + sr + 32 * i;
      const int off = key < Nk ? ((bkv * Nk + key) * ldkv + h * 64 + sc * 8) * 2 : kOOB;
      kreg[i] = buf_load16(rk, off);
      vreg[i] = buf_load16(rv, off);
    }
  };
  auto store_kv = [&](int buf) {
    char* Ks = smem + buf * 2 * SA_TILE;
    char* Vs = Ks + SA_TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = sr + 32 * i;
      *reinterpret_cast<u32x4*>(Ks + k_off(row, sc)) = kreg[i];
      *reinterpret_cast<u32x4*>(Vs + v_off(row, sc)) = vreg[i];
    }
  };

  f32x4 o[4][2];  // O^T accumulators [d-block][q-block]: lane col q, rows d = 16db + 4g + i
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) o[d][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {-INFINITY, -INFINITY};
  float lrun[2] = {0.f, 0.f};

  const int nt = (Nk + SA_KT - 1) / SA_KT;
  // V^T fragment reads: lane 4q'+p' of group g reads row 4g + q' (+16, +32, +48), cols 16db + 4p'
  int voff[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    const int li = lane & 15, r0 = g * 4 + (li >> 2), col = db * 16 + (li & 3) * 4;
    voff[db] = v_off(r0, col >> 3) + (col & 7) * 2;
  }
  if constexpr (PRE == 0) {
    load_kv(0);
    store_kv(0);
  } else {
    // pieces: tile t, operand (K, V), 8-row piece p; wave w issues p = w and p = w + 4 of every tile and operand
    const int prow = lane >> 3, pslot = lane & 7;
#pragma unroll
    for (int t = 0; t < PRE; ++t)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int row = (wid + 4 * pp) * 8 + prow;
        const int key = t * SA_KT + row;
        const int ck = pslot ^ ((row >> 1) & 7), cv = pslot ^ (((row >> 1) & 3) << 1);
        const int base = (bkv * Nk + key) * ldkv + h * 64;
        char* dst = smem + t * 2 * SA_TILE + (wid + 4 * pp) * 1024;
        sa_dma16(rk, dst, key < Nk ? (base + ck * 8) * 2 : kOOB);
        sa_dma16(rv, dst + SA_TILE, key < Nk ? (base + cv * 8) * 2 : kOOB);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int cur = PRE ? t : (t & 1);
    if (PRE == 0 && t + 1 < nt) load_kv(t + 1);
    const char* Ks = smem + cur * 2 * SA_TILE;
    const char* Vs = Ks + SA_TILE;

    // ---- S^T = K Q^T : s[kt][qb], lane col q, rows key = 16kt + 4g + i ----
    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      bf16x8 kf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        kf[kk] = *reinterpret_cast<const bf16x8*>(Ks + k_off(kt * 16 + fr, kk * 4 + g));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 a{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qb][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qb][1], a, 0, 0, 0);
        s[kt][qb] = a;
      }
    }
    // ---- mask keys beyond Nk (last tile); causal: keys after the query (CLIP text self-attention) ----
    if ((t + 1) * SA_KT > Nk || causal) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = t * SA_KT + kt * 16 + g * 4 + i;
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            if (key >= Nk || (causal && key > qbase + qb * 16 + fr)) s[kt][qb][i] = -INFINITY;
        }
    }
    // ---- online softmax (lane-local rows; reduce over the 4 g-lanes) ----
    float alpha[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[kt][qb][i]);
      mx = group_max(mx);
      const float mnew = fmaxf(mrun[qb], mx);
      alpha[qb] = fast_exp2((mrun[qb] - mnew) * scale_log2);
      mrun[qb] = mnew;
      const float mb = mnew * scale_log2;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = fast_exp2(s[kt][qb][i] * scale_log2 - mb);
          s[kt][qb][i] = pv;
          ls += pv;
        }
      lrun[qb] = lrun[qb] * alpha[qb] + ls;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) o[d][qb] *= alpha[qb];

    // ---- O^T += V^T P^T: two 32-key k-steps st (P tiles 2st -> elements 0-3, 2st+1 -> 4-7) ----
    bf16x8 pf[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        pf[st][qb] = pack_p8(s[2 * st][qb][0], s[2 * st][qb][1], s[2 * st][qb][2], s[2 * st][qb][3],
                             s[2 * st + 1][qb][0], s[2 * st + 1][qb][1], s[2 * st + 1][qb][2], s[2 * st + 1][qb][3]);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const char* vp = Vs + voff[db];  // rows +16 / +32 keep the swizzle: immediate offsets 2048 / 4096
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 vf = cat_tr(ds_read_tr(vp + st * 4096), ds_read_tr(vp + st * 4096 + 2048));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[st][qb], o[db][qb], 0, 0, 0);
      }
    }
    if constexpr (PRE == 0) {
      if (t + 1 < nt) store_kv(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- finalize: O[q][d] = O^T[d][q] / l ----
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float l = lrun[qb];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = 1.0f / l;
    const int q = qbase + qb * 16 + fr;
    if (q >= Nq) continue;
    if (lse && g == 0) lse[(size_t)bh * Nq + q] = mrun[qb] * scale_log2 + __log2f(l);  // training: P = exp2(s sl2 - lse)
    bf16_t* orow = O + (size_t)(b * Nq + q) * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4 v = o[db][qb] * inv;
      u32x2 w{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      *reinterpret_cast<u32x2*>(orow + db * 16 + g * 4) = w;
    }
  }
}

// ---------------------------------------------------------------------------------
// Self-attention over long key ranges (the 16x16 and 32x32 levels: 256 / 1024 keys), the default for
// vst_spatial_attention's self-attention: spatial_attn_kernel<0>'s arithmetic (S^T = K.Q^T with the query on the lane,
// online softmax against the running max, P rounded to bf16 unnormalised, O^T = V^T.P^T from transposed V reads, K/V
// tiles double-buffered through registers, 4 waves x 32 queries) without its causal mask, whose code spilled 31 SGPRs
// into VGPR lanes (~29 v_readlane / v_writelane per 64-key tile).  32x32: 148-156 -> 145-147 us, 16x16: 26.2-26.6 ->
// 25.4 us (profiles/r5_ab_sa_self.txt).  At head_dim 64 the softmax VALU, not the MFMA, bounds the loop (per tile and
// wave 32 MFMAs = 512 cycles against ~700-1,100 cycles of vector issue).  Not kept (same file):
//  - a deferred rescale (the running max moves only when a tile's max exceeds it by 2^8; the alpha exp2s and the 32 O
//    multiplies skipped): 32x32 135-142 us, but a row's largest P is then exp2(d), 0 < d <= 8, rounded to bf16
//    instead of an exact 1.0, and peaked rows lose accuracy (a configs[2] block rel_max 1.13e-2 -> 1.70e-2 against the
//    1.6e-2 gate, rel_l2 2.43e-3 -> 2.99e-3);
//  - 8 waves x 32 queries (one K/V fill per 256 queries): 128 VGPRs with spills, or one workgroup per CU; 16x16 31 us;
//  - S_{t+1} issued before tile t's softmax (software pipelining inside the wave): 208 VGPRs, 2 waves per SIMD, 32x32
//    169 us.
template <int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(3))) void sa_self_kernel(
    const bf16_t* __restrict__ Q, int ldq, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldkv,
    bf16_t* __restrict__ O, int ldo, int nbatch, int heads, int Nq, int Nk, float scale_log2, uint32_t q_bytes,
    uint32_t kv_bytes, float* __restrict__ lse) {
  constexpr int NCH = 512 / (NW * 64);  // 16-B chunks per thread and operand per tile (64 rows x 8 chunks)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nqb = (Nq + NW * 32 - 1) / (NW * 32);
  const int wg = xcd_remap(blockIdx.x, nqb * heads * nbatch);
  const int qblk = wg % nqb;
  const int bh = wg / nqb;
  const int h = bh % heads, b = bh / heads;
  const int fr = lane & 15, g = lane >> 4;

  const auto rq = make_rsrc(Q, q_bytes);
  const auto rk = make_rsrc(K, kv_bytes);
  const auto rv = make_rsrc(V, kv_bytes);

  bf16x8 qf[2][2];
  const int qbase = qblk * (NW * 32) + wid * 32;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qbase + qb * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int off = q < Nq ? ((b * Nq + q) * ldq + h * 64 + kk * 32 + g * 8) * 2 : kOOB;
      qf[qb][kk] = __builtin_bit_cast(bf16x8, buf_load16(rq, off));
    }
  }

  const int sc = tid & 7, sr = tid >> 3;  // rows sr + NW * 8 * i
  u32x4 kreg[NCH], vreg[NCH];
  const int kvrow0 = b * Nk;
  auto load_kv = [&](int t) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int key = t * SA_KT + sr + NW * 8 * i;
      const int off = key < Nk ? ((kvrow0 + key) * ldkv + h * 64 + sc * 8) * 2 : kOOB;
      kreg[i] = buf_load16(rk, off);
      vreg[i] = buf_load16(rv, off);
    }
  };
  auto store_kv = [&](int buf) {
    char* Ks = smem + buf * 2 * SA_TILE;
    char* Vs = Ks + SA_TILE;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = sr + NW * 8 * i;
      *reinterpret_cast<u32x4*>(Ks + k_off(row, sc)) = kreg[i];
      *reinterpret_cast<u32x4*>(Vs + v_off(row, sc)) = vreg[i];
    }
  };

  f32x4 o[4][2];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) o[d][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {-INFINITY, -INFINITY};
  float mb[2] = {0.f, 0.f};  // mrun * scale_log2
  float lrun[2] = {0.f, 0.f};

  const int nt = (Nk + SA_KT - 1) / SA_KT;
  int voff[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    const int li = lane & 15, r0 = g * 4 + (li >> 2), col = db * 16 + (li & 3) * 4;
    voff[db] = v_off(r0, col >> 3) + (col & 7) * 2;
  }
  load_kv(0);
  store_kv(0);
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) load_kv(t + 1);
    const char* Ks = smem + cur * 2 * SA_TILE;
    const char* Vs = Ks + SA_TILE;

    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      bf16x8 kf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        kf[kk] = *reinterpret_cast<const bf16x8*>(Ks + k_off(kt * 16 + fr, kk * 4 + g));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 a{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qb][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qb][1], a, 0, 0, 0);
        s[kt][qb] = a;
      }
    }
    if ((t + 1) * SA_KT > Nk) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool dead = t * SA_KT + kt * 16 + g * 4 + i >= Nk;
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            if (dead) s[kt][qb][i] = -INFINITY;
        }
    }
    // The softmax is written expression for expression as spatial_attn_kernel's (max from -inf, P = exp2(s sl2 - mb),
    // l = l alpha + sum P), so both kernels round alike and their outputs are bit-identical
    // (test_kernels_gpu.py::test_sa_self_bitwise_equals_spatial_attn): one forward arithmetic for inference and
    // training.  (Round 5 wrote P with an explicit fmaf and l as two roundings; that moved outputs by ulps.)
    float mx[2], alpha[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) m = fmaxf(m, s[kt][qb][i]);
      mx[qb] = group_max(m);
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const float mnew = fmaxf(mrun[qb], mx[qb]);
      alpha[qb] = fast_exp2((mrun[qb] - mnew) * scale_log2);
      mrun[qb] = mnew;
      mb[qb] = mnew * scale_log2;
#ifdef VST_SA_SCALAR
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[d][qb][e] = o[d][qb][e] * alpha[qb];
#else
#pragma unroll
      for (int d = 0; d < 4; ++d) o[d][qb] *= alpha[qb];
#endif
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = fast_exp2(s[kt][qb][i] * scale_log2 - mb[qb]);
          s[kt][qb][i] = pv;
          ls += pv;
        }
      lrun[qb] = lrun[qb] * alpha[qb] + ls;
    }
    bf16x8 pf[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        pf[st][qb] = pack_p8(s[2 * st][qb][0], s[2 * st][qb][1], s[2 * st][qb][2], s[2 * st][qb][3],
                             s[2 * st + 1][qb][0], s[2 * st + 1][qb][1], s[2 * st + 1][qb][2], s[2 * st + 1][qb][3]);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const char* vp = Vs + voff[db];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 vf = cat_tr(ds_read_tr(vp + st * 4096), ds_read_tr(vp + st * 4096 + 2048));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[st][qb], o[db][qb], 0, 0, 0);
      }
    }
    if (t + 1 < nt) store_kv(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float l = lrun[qb];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = 1.0f / l;
    const int q = qbase + qb * 16 + fr;
    if (q >= Nq) continue;
    if (lse && g == 0) lse[(size_t)bh * Nq + q] = mrun[qb] * scale_log2 + __log2f(l);  // training: P = exp2(s sl2 - lse)
    bf16_t* orow = O + (size_t)(b * Nq + q) * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4 v = o[db][qb] * inv;
      u32x2 w{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      *reinterpret_cast<u32x2*>(orow + db * 16 + g * 4) = w;
    }
  }
}

// ---------------------------------------------------------------------------------
// Temporal attention.  NT = number of 16-frame tiles (1: F<=16, 2: F<=32); D = head dim.
// A workgroup holds `blockDim.x / 64` consecutive units, i.e. all heads of one (clip, pixel) when they fit: the
// heads' 16-B q/k/v/o segments of a token row then meet in one CU's L1 instead of splitting cache lines
// between workgroups on two XCDs.
template <int NT, int D>
__global__ __launch_bounds__(512) void temporal_attn_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldqkv,
    bf16_t* __restrict__ O, int ldo, int nclip, int F, int HW, int heads, float scale_log2, uint32_t qkv_bytes) {
  constexpr int KS = (D + 31) / 32;  // 32-deep k-steps for S
  constexpr int DB = (D + 15) / 16;  // 16-wide d blocks for O
  constexpr int NF = 16 * NT;
  constexpr int VROW = DB * 32;      // bytes per V row in LDS
  extern __shared__ __attribute__((aligned(16))) char vsm[];  // [waves][NV KiB]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int unit = blockIdx.x * (blockDim.x >> 6) + wid;
  const int nunits = nclip * HW * heads;
  if (unit >= nunits) return;  // whole wave exits (unit is wave-uniform)
  const int h = unit % heads;
  const int bp = unit / heads;
  const int b = bp / HW, p = bp - b * HW;
  const int fr = lane & 15, g = lane >> 4;

  const auto rq = make_rsrc(Q, qkv_bytes);
  const auto rk = make_rsrc(K, qkv_bytes);
  const auto rv = make_rsrc(V, qkv_bytes);
  auto row_of = [&](int f) { return (b * F + f) * HW + p; };

  // ---- V rows into registers (zero rows >= F and columns >= D); they go to LDS after the S MFMAs, so the V, K and
  // Q loads are in flight together (one memory round trip per wave instead of two) ----
  constexpr int CPR = VROW / 16;  // 16-B chunks per LDS row
  constexpr int NV = (NF * CPR + 63) / 64;
  char* vs = vsm + wid * (NV * 1024);  // one wave's tile, padded to whole 1-KiB pieces (every lane stores)
  u32x4 vreg[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = lane + 64 * j;
    const int f = idx / CPR, c = idx - f * CPR;
    const int off = (idx < NF * CPR && f < F && c * 8 < D) ? (row_of(f) * ldqkv + h * D + c * 8) * 2 : kOOB;
    vreg[j] = buf_load16(rv, off);
  }
  __builtin_amdgcn_sched_barrier(0);  // every V load issues before the K / Q loads (the compiler sinks them otherwise)

  // ---- S^T = K Q^T ----
  f32x4 s[NT][NT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int c = 0; c < NT; ++c) s[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int d0 = kk * 32 + g * 8;
    bf16x8 kf[NT], qf[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const int f = tt * 16 + fr;
      const int off = (f < F && d0 < D) ? (row_of(f) * ldqkv + h * D + d0) * 2 : kOOB;
      kf[tt] = __builtin_bit_cast(bf16x8, buf_load16(rk, off));
      qf[tt] = __builtin_bit_cast(bf16x8, buf_load16(rq, off));
    }
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int c = 0; c < NT; ++c) s[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[a], qf[c], s[a][c], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < NV; ++j)  // chunk idx = f * CPR + c sits at byte idx * 16; the pad chunks get zeros
    *reinterpret_cast<u32x4*>(vs + (lane + 64 * j) * 16) = vreg[j];
  // mask keys >= F
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (a * 16 + g * 4 + i >= F) {
#pragma unroll
        for (int c = 0; c < NT; ++c) s[a][c][i] = -INFINITY;
      }
  // softmax per query column
  float inv[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[a][c][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mb = mx * scale_log2;
    float ls = 0.f;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = fast_exp2(s[a][c][i] * scale_log2 - mb);
        s[a][c][i] = pv;
        ls += pv;
      }
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    inv[c] = 1.0f / ls;
  }
  // V staging stores (this wave only) complete before the transposed reads
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // ---- O^T = V^T P^T (one 32-key k-step; for NT=1 the upper 16 keys are zero) ----
  bf16x8 pf[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    if (NT == 2)
      pf[c] = pack_p8(s[0][c][0], s[0][c][1], s[0][c][2], s[0][c][3], s[NT - 1][c][0], s[NT - 1][c][1],
                      s[NT - 1][c][2], s[NT - 1][c][3]);
    else
      pf[c] = pack_p8(s[0][c][0], s[0][c][1], s[0][c][2], s[0][c][3], 0.f, 0.f, 0.f, 0.f);
  }
  const int li = lane & 15;
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int r0 = g * 4 + (li >> 2);
    const int colb = (db * 16 + (li & 3) * 4) * 2;
    const s16x4 lo = ds_read_tr(vs + r0 * VROW + colb);
    s16x4 hi = s16x4{0, 0, 0, 0};
    if (NT == 2) hi = ds_read_tr(vs + (r0 + 16) * VROW + colb);
    const bf16x8 vf = cat_tr(lo, hi);
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[c], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const int f = c * 16 + fr;
      const int d = db * 16 + g * 4;
      if (f < F && d < D) {
        acc *= inv[c];
        u32x2 w{pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3])};
        *reinterpret_cast<u32x2*>(O + (size_t)row_of(f) * ldo + h * D + d) = w;
      }
    }
  }
}


// Temporal attention backward (training path): one wave per (clip, pixel, head), F <= 32, on the
// forward's v_mfma_f32_16x16x32_bf16 tiles.  P = softmax(scale Q K^T) is recomputed; with dP = dO V^T,
// D_i = sum_j P_ij dP_ij and dS = P * (dP - D):  dQ = scale dS K,  dK = scale dS^T Q,  dV = P^T dO.
// The three products need the score tiles with the query as the accumulator column (dQ^T = K^T dS^T) and with the key
// as the column (dK^T = Q^T dS, dV^T = dO^T P), so S and dP are formed both ways from the same row fragments
// (swapping the MFMA operands); the softmax statistics live in the transposed (query-column) tiles and reach the
// key-column tiles by one ds_bpermute per row.  The d-major A operands (K^T, Q^T, dO^T) come from ds_read_b64_tr_b16
// reads of the wave's own LDS copy of those rows, exactly like the forward's V^T.
template <int NT, int D>
__global__ __launch_bounds__(512) void temporal_attn_bwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldqkv,
    const bf16_t* __restrict__ dO, int lddo, bf16_t* __restrict__ dQ, bf16_t* __restrict__ dK,
    bf16_t* __restrict__ dV, int lddqkv, int nclip, int F, int HW, int heads, float scale, float scale_log2,
    uint32_t qkv_bytes, uint32_t do_bytes) {
  constexpr int KS = (D + 31) / 32;  // 32-deep k-steps over d
  constexpr int DB = (D + 15) / 16;  // 16-wide d blocks of the outputs
  constexpr int NF = 16 * NT;
  constexpr int VROW = DB * 32;      // bytes per staged row
  constexpr int CPR = VROW / 16;
  constexpr int ARR = NF * VROW;     // one staged operand
  extern __shared__ __attribute__((aligned(16))) char tbm[];  // [waves][K, Q, dO][NF * VROW]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int unit = blockIdx.x * (blockDim.x >> 6) + wid;
  if (unit >= nclip * HW * heads) return;  // whole wave exits (unit is wave-uniform); no workgroup barriers below
  const int h = unit % heads;
  const int bp = unit / heads;
  const int b = bp / HW, p = bp - b * HW;
  const int fr = lane & 15, g = lane >> 4;
  const auto rq = make_rsrc(Q, qkv_bytes);
  const auto rk = make_rsrc(K, qkv_bytes);
  const auto rv = make_rsrc(V, qkv_bytes);
  const auto ro = make_rsrc(dO, do_bytes);
  auto row_of = [&](int f) { return (b * F + f) * HW + p; };

  // ---- stage K, Q, dO rows (zero rows >= F, columns >= D) for the transposed reads ----
  char* ks = tbm + wid * 3 * ARR;
  char* qs = ks + ARR;
  char* os = qs + ARR;
  for (int idx = lane; idx < NF * CPR; idx += 64) {
    const int f = idx / CPR, c = idx - f * CPR;
    const bool in = f < F && c * 8 < D;
    const int off = in ? (row_of(f) * ldqkv + h * D + c * 8) * 2 : kOOB;
    const int ooff = in ? (row_of(f) * lddo + h * D + c * 8) * 2 : kOOB;
    *reinterpret_cast<u32x4*>(ks + f * VROW + c * 16) = buf_load16(rk, off);
    *reinterpret_cast<u32x4*>(qs + f * VROW + c * 16) = buf_load16(rq, off);
    *reinterpret_cast<u32x4*>(os + f * VROW + c * 16) = buf_load16(ro, ooff);
  }

  // ---- scores both ways: st = S^T [key][query], sn = S [query][key]; dpt = dP^T, dpn = dP ----
  f32x4 st[NT][NT], sn[NT][NT], dpt[NT][NT], dpn[NT][NT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      st[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
      sn[a][c] = st[a][c];
      dpt[a][c] = st[a][c];
      dpn[a][c] = st[a][c];
    }
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int d0 = kk * 32 + g * 8;
    bf16x8 kf[NT], qf[NT], vf[NT], of[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const int f = tt * 16 + fr;
      const bool in = f < F && d0 < D;
      const int off = in ? (row_of(f) * ldqkv + h * D + d0) * 2 : kOOB;
      const int ooff = in ? (row_of(f) * lddo + h * D + d0) * 2 : kOOB;
      kf[tt] = __builtin_bit_cast(bf16x8, buf_load16(rk, off));
      qf[tt] = __builtin_bit_cast(bf16x8, buf_load16(rq, off));
      vf[tt] = __builtin_bit_cast(bf16x8, buf_load16(rv, off));
      of[tt] = __builtin_bit_cast(bf16x8, buf_load16(ro, ooff));
    }
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        st[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[a], qf[c], st[a][c], 0, 0, 0);
        sn[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[a], kf[c], sn[a][c], 0, 0, 0);
        dpt[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[a], of[c], dpt[a][c], 0, 0, 0);
        dpn[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(of[a], vf[c], dpn[a][c], 0, 0, 0);
      }
  }
  // mask keys >= F: rows of st, columns (whole lanes) of sn
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (a * 16 + g * 4 + i >= F) {
#pragma unroll
        for (int c = 0; c < NT; ++c) st[a][c][i] = -INFINITY;
      }
#pragma unroll
  for (int c = 0; c < NT; ++c)
    if (c * 16 + fr >= F) {
#pragma unroll
      for (int a = 0; a < NT; ++a) sn[a][c] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    }

  // ---- softmax statistics per query column; P^T and dS^T = P^T (dP^T - D) in place ----
  float mb[NT], inv[NT], dd[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = fmaxf(mx, st[a][c][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    mb[c] = mx * scale_log2;
    float ls = 0.f;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = fast_exp2(st[a][c][i] * scale_log2 - mb[c]);
        st[a][c][i] = e;
        ls += e;
      }
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    inv[c] = 1.0f / ls;
    float di = 0.f;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[a][c][i] *= inv[c];
        di += st[a][c][i] * dpt[a][c][i];
      }
    di += __shfl_xor(di, 16);
    di += __shfl_xor(di, 32);
    dd[c] = di;
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) dpt[a][c][i] = st[a][c][i] * (dpt[a][c][i] - di);
  }
  // ---- key-column tiles: row (query) 16a + 4g + i takes its statistics from lane 4g + i ----
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int src = g * 4 + i;
      const float m = __shfl(mb[a], src), iv = __shfl(inv[a], src), di = __shfl(dd[a], src);
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const float pv = fast_exp2(sn[a][c][i] * scale_log2 - m) * iv;
        sn[a][c][i] = pv;
        dpn[a][c][i] = pv * (dpn[a][c][i] - di);
      }
    }

  // ---- B operands (32-deep k = the 16 or 32 frames; upper half zero for NT = 1) ----
  bf16x8 bq[NT], bk[NT], bv[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int a1 = NT - 1;
    const float z = NT == 2 ? 1.f : 0.f;
    bq[c] = pack_p8(dpt[0][c][0], dpt[0][c][1], dpt[0][c][2], dpt[0][c][3], z * dpt[a1][c][0], z * dpt[a1][c][1],
                    z * dpt[a1][c][2], z * dpt[a1][c][3]);
    bk[c] = pack_p8(dpn[0][c][0], dpn[0][c][1], dpn[0][c][2], dpn[0][c][3], z * dpn[a1][c][0], z * dpn[a1][c][1],
                    z * dpn[a1][c][2], z * dpn[a1][c][3]);
    bv[c] = pack_p8(sn[0][c][0], sn[0][c][1], sn[0][c][2], sn[0][c][3], z * sn[a1][c][0], z * sn[a1][c][1],
                    z * sn[a1][c][2], z * sn[a1][c][3]);
  }
  // the staging stores (this wave only) complete before the transposed reads
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // ---- dQ^T = K^T dS^T, dK^T = Q^T dS, dV^T = dO^T P, per 16-wide d block ----
  const int li = lane & 15;
  const int r0 = g * 4 + (li >> 2);
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int colb = (db * 16 + (li & 3) * 4) * 2;
    const s16x4 z4{0, 0, 0, 0};
    const bf16x8 kT = cat_tr(ds_read_tr(ks + r0 * VROW + colb), NT == 2 ? ds_read_tr(ks + (r0 + 16) * VROW + colb) : z4);
    const bf16x8 qT = cat_tr(ds_read_tr(qs + r0 * VROW + colb), NT == 2 ? ds_read_tr(qs + (r0 + 16) * VROW + colb) : z4);
    const bf16x8 oT = cat_tr(ds_read_tr(os + r0 * VROW + colb), NT == 2 ? ds_read_tr(os + (r0 + 16) * VROW + colb) : z4);
    const int d = db * 16 + g * 4;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const f32x4 z{0.f, 0.f, 0.f, 0.f};
      const f32x4 gq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kT, bq[c], z, 0, 0, 0) * scale;
      const f32x4 gk = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qT, bk[c], z, 0, 0, 0) * scale;
      const f32x4 gv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oT, bv[c], z, 0, 0, 0);
      const int f = c * 16 + fr;
      if (f < F && d < D) {
        const size_t o = (size_t)row_of(f) * lddqkv + h * D + d;
        *reinterpret_cast<u32x2*>(dQ + o) = u32x2{pack2bf(gq[0], gq[1]), pack2bf(gq[2], gq[3])};
        *reinterpret_cast<u32x2*>(dK + o) = u32x2{pack2bf(gk[0], gk[1]), pack2bf(gk[2], gk[3])};
        *reinterpret_cast<u32x2*>(dV + o) = u32x2{pack2bf(gv[0], gv[1]), pack2bf(gv[2], gv[3])};
      }
    }
  }
}


// ---------------------------------------------------------------------------------
// Spatial attention backward (training path), head_dim 64, flash-attention style on the same
// v_mfma_f32_16x16x32_bf16 tiles as the forward, deterministic (no atomics), P recomputed from the forward's
// log2-domain logsumexp (lse2 = max * scale*log2(e) + log2(l), written by spatial_attn_kernel):
//   P = exp2(S * sl2 - lse2),  dP = dO V^T,  D_i = dO_i . O_i,  dS = P * (dP - D),
//   dQ = scale dS K,  dK = scale dS^T Q,  dV = P^T dO.
// sa_bwd_dq_kernel: 4 waves x 32 queries per workgroup, loop over 64-key tiles (K row + K transposed + V row copies
//   double-buffered in LDS); per tile and wave 48 MFMAs (S^T, dP^T, dQ^T); also writes D for the dK/dV kernel.
// sa_bwd_dkv_kernel: 4 waves x 32 keys per workgroup, loop over 64-query tiles of every query batch that reads these
//   K/V (kv_div > 1: all frames of a clip share the text K/V, so their contributions sum in registers); per tile and
//   wave 64 MFMAs (S, dP, dV^T, dK^T).  Skipped when the caller needs no dK/dV (frozen cross-attention K/V).
// Fragment conventions follow the forward: accumulators hold transposed tiles (lane column = the row token), P / dS
// feed the B operand straight from the accumulators, and the A operands of the d-major products (K^T, dO^T, Q^T)
// come from ds_read_b64_tr_b16 reads of a v_off-swizzled LDS copy.
constexpr int SB_TILE = 64 * 64 * 2;  // one 64-row x 64-d bf16 tile, 8 KiB

// one transposed A fragment: T^T[d = 16 db + li][rows 32 st + 4 g + {0..3}, 32 st + 16 + 4 g + {0..3}]
__device__ __forceinline__ bf16x8 tr_frag(const char* T, int st, int db, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const int r0 = st * 32 + g * 4 + (li >> 2);
  const int col = db * 16 + (li & 3) * 4;
  const int ch = col >> 3, within = (col & 7) * 2;
  return cat_tr(ds_read_tr(T + v_off(r0, ch) + within), ds_read_tr(T + v_off(r0 + 16, ch) + within));
}

__global__ __launch_bounds__(256, 2) void sa_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, int ldq, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldkv,
    const bf16_t* __restrict__ O, int ldo, const bf16_t* __restrict__ dO, int lddo, const float* __restrict__ lse,
    bf16_t* __restrict__ dQ, int lddq, float* __restrict__ dvec, int nbatch, int heads, int Nq, int Nk, int kv_div,
    float scale, float sl2, uint32_t q_bytes, uint32_t o_bytes, uint32_t do_bytes, uint32_t kv_bytes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nqb = (Nq + 127) / 128;
  const int wg = xcd_remap(blockIdx.x, nqb * heads * nbatch);
  const int qblk = wg % nqb, bh = wg / nqb;
  const int h = bh % heads, b = bh / heads, bkv = b / kv_div;
  const int fr = lane & 15, g = lane >> 4;
  const auto rq = make_rsrc(Q, q_bytes);
  const auto ro = make_rsrc(O, o_bytes);
  const auto rdo = make_rsrc(dO, do_bytes);
  const auto rk = make_rsrc(K, kv_bytes);
  const auto rv = make_rsrc(V, kv_bytes);

  // Q^T / dO^T B fragments (lane column = query), D = dO . O, lse per query
  bf16x8 qf[2][2], dof[2][2];
  float Dq[2], l2[2];
  const int qbase = qblk * 128 + wid * 32;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qbase + qb * 16 + fr;
    float dsum = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int col = h * 64 + kk * 32 + g * 8;
      qf[qb][kk] = __builtin_bit_cast(bf16x8, buf_load16(rq, q < Nq ? ((b * Nq + q) * ldq + col) * 2 : kOOB));
      const u32x4 dov = buf_load16(rdo, q < Nq ? ((b * Nq + q) * lddo + col) * 2 : kOOB);
      const u32x4 ov = buf_load16(ro, q < Nq ? ((b * Nq + q) * ldo + col) * 2 : kOOB);
      dof[qb][kk] = __builtin_bit_cast(bf16x8, dov);
      float a[8], c[8];
      unpack8(dov, a);
      unpack8(ov, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += a[e] * c[e];
    }
    dsum += __shfl_xor(dsum, 16);
    dsum += __shfl_xor(dsum, 32);
    Dq[qb] = dsum;
    const size_t qi = (size_t)bh * Nq + q;
    l2[qb] = q < Nq ? lse[qi] : 0.f;
    if (g == 0 && q < Nq) dvec[qi] = dsum;
  }

  const int sc = tid & 7, sr = tid >> 3;  // staging: rows sr, sr + 32, 16-B chunk sc
  u32x4 kreg[2], vreg[2];
  auto load_kv = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = t * 64 + sr + 32 * i;
      const int off = key < Nk ? ((bkv * Nk + key) * ldkv + h * 64 + sc * 8) * 2 : kOOB;
      kreg[i] = buf_load16(rk, off);
      vreg[i] = buf_load16(rv, off);
    }
  };
  auto store_kv = [&](int buf) {
    char* Kr = smem + buf * 3 * SB_TILE;
    char* Kt = Kr + SB_TILE;
    char* Vr = Kt + SB_TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = sr + 32 * i;
      *reinterpret_cast<u32x4*>(Kr + k_off(row, sc)) = kreg[i];
      *reinterpret_cast<u32x4*>(Kt + v_off(row, sc)) = kreg[i];
      *reinterpret_cast<u32x4*>(Vr + k_off(row, sc)) = vreg[i];
    }
  };

  f32x4 acc[4][2];  // dQ^T [d-block][q-block]
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) acc[d][qb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (Nk + 63) / 64;
  load_kv(0);
  store_kv(0);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) load_kv(t + 1);
    const char* Kr = smem + cur * 3 * SB_TILE;
    const char* Kt = Kr + SB_TILE;
    const char* Vr = Kt + SB_TILE;
    f32x4 s[4][2], dp[4][2];  // S^T, dP^T: lane column q, rows key = 16 kt + 4 g + i
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      bf16x8 kf[2], vf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        kf[kk] = *reinterpret_cast<const bf16x8*>(Kr + k_off(kt * 16 + fr, kk * 4 + g));
        vf[kk] = *reinterpret_cast<const bf16x8*>(Vr + k_off(kt * 16 + fr, kk * 4 + g));
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 a{0.f, 0.f, 0.f, 0.f}, c{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qb][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qb][1], a, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[0], dof[qb][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[1], dof[qb][1], c, 0, 0, 0);
        s[kt][qb] = a;
        dp[kt][qb] = c;
      }
    }
    // dS^T = P^T * (dP^T - D), keys >= Nk masked
    const bool tail = (t + 1) * 64 > Nk;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool dead = tail && (t * 64 + kt * 16 + g * 4 + i >= Nk);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const float pv = dead ? 0.f : fast_exp2(s[kt][qb][i] * sl2 - l2[qb]);
          s[kt][qb][i] = pv * (dp[kt][qb][i] - Dq[qb]);
        }
      }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        pf[qb] = pack_p8(s[2 * st][qb][0], s[2 * st][qb][1], s[2 * st][qb][2], s[2 * st][qb][3],
                         s[2 * st + 1][qb][0], s[2 * st + 1][qb][1], s[2 * st + 1][qb][2], s[2 * st + 1][qb][3]);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8 kt_f = tr_frag(Kt, st, db, lane);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          acc[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt_f, pf[qb], acc[db][qb], 0, 0, 0);
      }
    }
    if (t + 1 < nt) store_kv(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qbase + qb * 16 + fr;
    if (q >= Nq) continue;
    bf16_t* row = dQ + (size_t)(b * Nq + q) * lddq + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4 v = acc[db][qb] * scale;
      *reinterpret_cast<u32x2*>(row + db * 16 + g * 4) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
    }
  }
}

__global__ __launch_bounds__(256, 2) void sa_bwd_dkv_kernel(
    const bf16_t* __restrict__ Q, int ldq, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V, int ldkv,
    const bf16_t* __restrict__ dO, int lddo, const float* __restrict__ lse, const float* __restrict__ dvec,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int lddkv, int nkv, int heads, int Nq, int Nk, int kv_div,
    float scale, float sl2, uint32_t q_bytes, uint32_t do_bytes, uint32_t kv_bytes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = 4 * SB_TILE + 2 * 64 * 4;  // Q row, Q^T, dO row, dO^T, lse2[64], D[64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nkb = (Nk + 127) / 128;
  const int wg = xcd_remap(blockIdx.x, nkb * heads * nkv);
  const int kblk = wg % nkb, bh = wg / nkb;
  const int h = bh % heads, bkv = bh / heads;
  const int fr = lane & 15, g = lane >> 4;
  const auto rq = make_rsrc(Q, q_bytes);
  const auto rdo = make_rsrc(dO, do_bytes);
  const auto rk = make_rsrc(K, kv_bytes);
  const auto rv = make_rsrc(V, kv_bytes);

  // K / V B fragments (lane column = key)
  bf16x8 kf[2][2], vf[2][2];
  const int kbase = kblk * 128 + wid * 32;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = kbase + kb * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int off = key < Nk ? ((bkv * Nk + key) * ldkv + h * 64 + kk * 32 + g * 8) * 2 : kOOB;
      kf[kb][kk] = __builtin_bit_cast(bf16x8, buf_load16(rk, off));
      vf[kb][kk] = __builtin_bit_cast(bf16x8, buf_load16(rv, off));
    }
  }

  const int sc = tid & 7, sr = tid >> 3;
  const int nqt = (Nq + 63) / 64;
  const int ntiles = kv_div * nqt;  // (query batch bkv * kv_div + j, query tile)
  u32x4 qreg[2], oreg[2];
  float lreg = 0.f, dreg = 0.f;
  auto load_q = [&](int it) {
    const int b = bkv * kv_div + it / nqt, q0 = (it % nqt) * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = q0 + sr + 32 * i;
      qreg[i] = buf_load16(rq, q < Nq ? ((b * Nq + q) * ldq + h * 64 + sc * 8) * 2 : kOOB);
      oreg[i] = buf_load16(rdo, q < Nq ? ((b * Nq + q) * lddo + h * 64 + sc * 8) * 2 : kOOB);
    }
    if (tid < 64) {
      const int q = q0 + tid;
      const size_t qi = (size_t)(b * heads + h) * Nq + q;
      lreg = q < Nq ? lse[qi] : INFINITY;  // padded queries: P = 0
      dreg = q < Nq ? dvec[qi] : 0.f;
    }
  };
  auto store_q = [&](int buf) {
    char* Qr = smem + buf * BUF;
    char* Qt = Qr + SB_TILE;
    char* Or = Qt + SB_TILE;
    char* Ot = Or + SB_TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = sr + 32 * i;
      *reinterpret_cast<u32x4*>(Qr + k_off(row, sc)) = qreg[i];
      *reinterpret_cast<u32x4*>(Qt + v_off(row, sc)) = qreg[i];
      *reinterpret_cast<u32x4*>(Or + k_off(row, sc)) = oreg[i];
      *reinterpret_cast<u32x4*>(Ot + v_off(row, sc)) = oreg[i];
    }
    if (tid < 64) {
      float* ls = reinterpret_cast<float*>(Ot + SB_TILE);
      ls[tid] = lreg;
      ls[64 + tid] = dreg;
    }
  };

  f32x4 dk[4][2], dv[4][2];  // dK^T, dV^T [d-block][key-block]
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      dk[d][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[d][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  load_q(0);
  store_q(0);
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int cur = it & 1;
    if (it + 1 < ntiles) load_q(it + 1);
    const char* Qr = smem + cur * BUF;
    const char* Qt = Qr + SB_TILE;
    const char* Or = Qt + SB_TILE;
    const char* Ot = Or + SB_TILE;
    const float* ls = reinterpret_cast<const float*>(Ot + SB_TILE);
    f32x4 s[4][2], dp[4][2];  // S, dP: lane column key, rows q = 16 qt + 4 g + i
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      bf16x8 qa[2], oa[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        qa[kk] = *reinterpret_cast<const bf16x8*>(Qr + k_off(qt * 16 + fr, kk * 4 + g));
        oa[kk] = *reinterpret_cast<const bf16x8*>(Or + k_off(qt * 16 + fr, kk * 4 + g));
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        f32x4 a{0.f, 0.f, 0.f, 0.f}, c{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[0], kf[kb][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[1], kf[kb][1], a, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa[0], vf[kb][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa[1], vf[kb][1], c, 0, 0, 0);
        s[qt][kb] = a;
        dp[qt][kb] = c;
      }
    }
    // P into s, dS into dp
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const f32x4 lq = *reinterpret_cast<const f32x4*>(ls + qt * 16 + g * 4);
      const f32x4 dq = *reinterpret_cast<const f32x4*>(ls + 64 + qt * 16 + g * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const float pv = fast_exp2(s[qt][kb][i] * sl2 - lq[i]);
          s[qt][kb][i] = pv;
          dp[qt][kb][i] = pv * (dp[qt][kb][i] - dq[i]);
        }
    }
    // dV^T += dO^T P,  dK^T += Q^T dS
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        pf[kb] = pack_p8(s[2 * st][kb][0], s[2 * st][kb][1], s[2 * st][kb][2], s[2 * st][kb][3],
                         s[2 * st + 1][kb][0], s[2 * st + 1][kb][1], s[2 * st + 1][kb][2], s[2 * st + 1][kb][3]);
        sf[kb] = pack_p8(dp[2 * st][kb][0], dp[2 * st][kb][1], dp[2 * st][kb][2], dp[2 * st][kb][3],
                         dp[2 * st + 1][kb][0], dp[2 * st + 1][kb][1], dp[2 * st + 1][kb][2], dp[2 * st + 1][kb][3]);
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8 ot = tr_frag(Ot, st, db, lane);
        const bf16x8 qtf = tr_frag(Qt, st, db, lane);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          dv[db][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ot, pf[kb], dv[db][kb], 0, 0, 0);
          dk[db][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qtf, sf[kb], dk[db][kb], 0, 0, 0);
        }
      }
    }
    if (it + 1 < ntiles) store_q(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = kbase + kb * 16 + fr;
    if (key >= Nk) continue;
    bf16_t* krow = dK + (size_t)(bkv * Nk + key) * lddkv + h * 64;
    bf16_t* vrow = dV + (size_t)(bkv * Nk + key) * lddkv + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const f32x4 a = dk[db][kb] * scale;
      const f32x4 c = dv[db][kb];
      *reinterpret_cast<u32x2*>(krow + db * 16 + g * 4) = u32x2{pack2bf(a[0], a[1]), pack2bf(a[2], a[3])};
      *reinterpret_cast<u32x2*>(vrow + db * 16 + g * 4) = u32x2{pack2bf(c[0], c[1]), pack2bf(c[2], c[3])};
    }
  }
}


template <int NT, int D>
static int launch_temporal(const bf16_t* Q, const bf16_t* K, const bf16_t* V, int ld, bf16_t* O, int ldo,
                           int nclip, int F, int HW, int heads, float sl2, uint32_t bytes, hipStream_t s) {
  const int units = nclip * HW * heads;
  constexpr int VBYTES = (16 * NT * ((D + 15) / 16) * 32 + 1023) / 1024 * 1024;  // one wave's V tile, 1-KiB pieces
  // all heads of a (clip, pixel) in one workgroup when they fit (<= 8 waves, <= 64 KiB of V tiles), else 4 units
  const int wpg = (heads <= 8 && heads * VBYTES <= 64 * 1024) ? heads : 4;
  hipLaunchKernelGGL((temporal_attn_kernel<NT, D>), dim3((units + wpg - 1) / wpg), dim3(64 * wpg), wpg * VBYTES, s,
                     Q, K, V, ld, O, ldo, nclip, F, HW, heads, sl2, bytes);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

}  // namespace vst

using namespace vst;

static int g_sa_self = -1;  // VST_SA_SELF, or vst_sa_self (tests, A/B)
static int sa_self_on() {
  if (g_sa_self < 0) {
    const char* e = getenv("VST_SA_SELF");
    g_sa_self = e ? (atoi(e) != 0) : 1;
  }
  return g_sa_self;
}

extern "C" int vst_sa_self(int on) {
  const int prev = sa_self_on();
  g_sa_self = on != 0;
  return prev;
}

extern "C" int vst_spatial_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, void* o,
                                     int ldo, int nbatch, int heads, int Nq, int Nk, int kv_div, int head_dim,
                                     float scale, float* lse, void* stream) {
  Fit31 fit;
  if (head_dim != 64 || !q || !k || !v || !o || nbatch <= 0 || heads <= 0 || Nq <= 0 || Nk <= 0 || kv_div <= 0)
    return VST_ERR_ARG;
  if ((ldq & 7) || (ldkv & 7) || (ldo & 7) || nbatch % kv_div) return VST_ERR_ARG;
  const int nqb = (Nq + 127) / 128;
  const int nkv = nbatch / kv_div;
  const uint32_t qb = fit(((size_t)(nbatch * Nq - 1) * ldq + heads * 64) * 2);
  // K and V may be column views of one fused buffer; each rsrc is sized from its own base
  const uint32_t kvb_v = fit(((size_t)(nkv * Nk - 1) * ldkv + heads * 64) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse, never read zeros
  const int nt = (Nk + SA_KT - 1) / SA_KT;
  static int pre_env = -1;  // VST_SA_PRELOAD=0 disables the whole-K/V preload (A/B diagnostics)
  if (pre_env < 0) {
    const char* e = getenv("VST_SA_PRELOAD");
    pre_env = e ? atoi(e) : 1;
  }
  // measured (tools/attn_bench.py, one process, alternating): cross-attention over 77 text keys 33 -> 28.5 us at 32x32
  // and 18 -> 17.3 us at 16x16; the 16x16 self-attention (4 tiles) 29.2 -> 31.2 us (64 KiB of LDS per workgroup
  // drops occupancy from 3 to 2 workgroups per CU), so only up to two tiles are preloaded
  const int pre = pre_env && nt <= 2 ? nt : 0;
  const dim3 grid(nqb * heads * nbatch);
  const size_t lds = pre ? (size_t)pre * 2 * SA_TILE : SA_LDS;
  hipStream_t st = (hipStream_t)stream;
  const float sl2 = scale * 1.4426950408889634f;
#define VST_SA_LAUNCH(P)                                                                                         \
  hipLaunchKernelGGL(spatial_attn_kernel<P>, grid, dim3(256), lds, st, (const bf16_t*)q, ldq, (const bf16_t*)k, \
                     (const bf16_t*)v, ldkv, (bf16_t*)o, ldo, nbatch, heads, Nq, Nk, kv_div, sl2, qb, kvb_v, lse)
  // the long self-attention (inference AND the training forward, which also asks for the logsumexp) on
  // sa_self_kernel, bit-identical to spatial_attn_kernel<0>; vst_sa_self(0) / VST_SA_SELF=0 restores the latter
  if (pre == 0 && kv_div == 1 && sa_self_on()) {
    const dim3 g2(((Nq + 127) / 128) * heads * nbatch);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sa_self_kernel<4>), g2, dim3(256), SA_LDS, st, (const bf16_t*)q, ldq,
                       (const bf16_t*)k, (const bf16_t*)v, ldkv, (bf16_t*)o, ldo, nbatch, heads, Nq, Nk, sl2, qb,
                       kvb_v, lse);
    return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
  }
  switch (pre) {
    case 1: VST_SA_LAUNCH(1); break;
    case 2: VST_SA_LAUNCH(2); break;
    case 3: VST_SA_LAUNCH(3); break;
    case 4: VST_SA_LAUNCH(4); break;
    default: VST_SA_LAUNCH(0); break;
  }
#undef VST_SA_LAUNCH
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// Causal self-attention over N tokens, head_dim 64 (the CLIP text encoders' CLIPAttention with the causal mask of
// transformers' CLIPTextTransformer): query i attends to keys 0..i.  Same kernel as vst_spatial_attention.
extern "C" int vst_causal_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, void* o, int ldo,
                                    int nbatch, int heads, int N, int head_dim, float scale, void* stream) {
  Fit31 fit;
  if (head_dim != 64 || !q || !k || !v || !o || nbatch <= 0 || heads <= 0 || N <= 0) return VST_ERR_ARG;
  if ((ldq & 7) || (ldkv & 7) || (ldo & 7)) return VST_ERR_ARG;
  const int nqb = (N + 127) / 128;
  const uint32_t qb = fit(((size_t)(nbatch * N - 1) * ldq + heads * 64) * 2);
  const uint32_t kvb = fit(((size_t)(nbatch * N - 1) * ldkv + heads * 64) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse, never read zeros
  const dim3 grid(nqb * heads * nbatch);
  hipLaunchKernelGGL(spatial_attn_kernel<0>, grid, dim3(256), SA_LDS, (hipStream_t)stream, (const bf16_t*)q, ldq,
                     (const bf16_t*)k, (const bf16_t*)v, ldkv, (bf16_t*)o, ldo, nbatch, heads, N, N, 1,
                     scale * 1.4426950408889634f, qb, kvb, (float*)nullptr, 1);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

extern "C" int vst_temporal_attention(const void* q, const void* k, const void* v, int ldqkv, void* o, int ldo,
                                      int nclip, int F, int HW, int heads, int head_dim, float scale, void* stream) {
  Fit31 fit;
  if (!q || !k || !v || !o || nclip <= 0 || F <= 0 || F > 32 || HW <= 0 || heads <= 0) return VST_ERR_ARG;
  if ((ldqkv & 7) || (ldo & 7) || (head_dim & 7)) return VST_ERR_ARG;
  const uint32_t bytes = fit(((size_t)(nclip * F * HW - 1) * ldqkv + heads * head_dim) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse, never read zeros
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t *Q = (const bf16_t*)q, *K = (const bf16_t*)k, *V = (const bf16_t*)v;
  bf16_t* O = (bf16_t*)o;
#define VST_TA(D)                                                                                    \
  case D:                                                                                          \
    return F <= 16 ? launch_temporal<1, D>(Q, K, V, ldqkv, O, ldo, nclip, F, HW, heads, sl2, bytes, s) \
                   : launch_temporal<2, D>(Q, K, V, ldqkv, O, ldo, nclip, F, HW, heads, sl2, bytes, s);
  switch (head_dim) {
    VST_TA(8)
    VST_TA(16)
    VST_TA(32)
    VST_TA(40)
    VST_TA(64)
    VST_TA(80)
    VST_TA(160)
    default:
      return VST_ERR_ARG;
  }
#undef VST_TA
}

extern "C" int vst_temporal_attention_bwd(const void* q, const void* k, const void* v, int ldqkv, const void* dout,
                                          int lddo, void* dq, void* dk, void* dv, int lddqkv, int nclip, int F, int HW,
                                          int heads, int head_dim, float scale, void* stream) {
  Fit31 fit;
  if (!q || !k || !v || !dout || !dq || !dk || !dv || nclip <= 0 || F <= 0 || F > 32 || HW <= 0 || heads <= 0)
    return VST_ERR_ARG;
  if ((ldqkv & 7) || (lddo & 7) || (lddqkv & 3) || (head_dim & 7)) return VST_ERR_ARG;
  const size_t units = (size_t)nclip * HW * heads;
  if (units > 0x7fffffffULL) return VST_ERR_ARG;
  const uint32_t qkvb = fit(((size_t)(nclip * F * HW - 1) * ldqkv + heads * head_dim) * 2);
  const uint32_t dob = fit(((size_t)(nclip * F * HW - 1) * lddo + heads * head_dim) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse, never read zeros
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t *Q = (const bf16_t*)q, *K = (const bf16_t*)k, *V = (const bf16_t*)v, *G = (const bf16_t*)dout;
  bf16_t *GQ = (bf16_t*)dq, *GK = (bf16_t*)dk, *GV = (bf16_t*)dv;
  auto launch = [&](auto kern, int nf, int D) {
    const int wave_bytes = 3 * nf * ((D + 15) / 16) * 32;  // K, Q, dO rows
    // all heads of a (clip, pixel) in one workgroup when they fit in 64 KiB, else as many units as do
    const int wpg = heads * wave_bytes <= 64 * 1024 ? std::min(heads, 8) : std::max(1, 64 * 1024 / wave_bytes);
    hipLaunchKernelGGL(kern, dim3((unsigned)((units + wpg - 1) / wpg)), dim3(64 * wpg), wpg * wave_bytes, s, Q, K, V,
                       ldqkv, G, lddo, GQ, GK, GV, lddqkv, nclip, F, HW, heads, scale, sl2, qkvb, dob);
    return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
  };
#define VST_TAB(D)                                                                              \
  case D:                                                                                       \
    return F <= 16 ? launch(temporal_attn_bwd_kernel<1, D>, 16, D) : launch(temporal_attn_bwd_kernel<2, D>, 32, D);
  switch (head_dim) {
    VST_TAB(8)
    VST_TAB(16)
    VST_TAB(32)
    VST_TAB(40)
    VST_TAB(64)
    VST_TAB(80)
    VST_TAB(160)
    default:
      return VST_ERR_ARG;
  }
#undef VST_TAB
}

// D = dO . O per query (written by the dQ kernel, read by the dK/dV kernel)
extern "C" size_t vst_spatial_attention_bwd_workspace_bytes(int nbatch, int heads, int Nq, int Nk) {
  (void)Nk;
  return (size_t)nbatch * heads * Nq * sizeof(float);
}

extern "C" int vst_spatial_attention_bwd(const void* q, int ldq, const void* k, const void* v, int ldkv, const void* o,
                                         int ldo, const void* dout, int lddo, const float* lse, void* dq, int lddq,
                                         void* dk, void* dv, int lddkv, int nbatch, int heads, int Nq, int Nk,
                                         int kv_div, int head_dim, float scale, void* workspace, void* stream) {
  Fit31 fit;
  if (head_dim != 64 || !q || !k || !v || !o || !dout || !lse || !dq || !workspace || nbatch <= 0 || heads <= 0 ||
      Nq <= 0 || Nk <= 0 || kv_div <= 0 || nbatch % kv_div || (!dk) != (!dv))
    return VST_ERR_ARG;
  if ((ldq & 7) || (ldkv & 7) || (ldo & 7) || (lddo & 7) || (lddq & 3) || (dk && (lddkv & 3))) return VST_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  float* dvec = (float*)workspace;
  const int nkv = nbatch / kv_div;
  const float sl2 = scale * 1.4426950408889634f;
  const uint32_t qb = fit(((size_t)(nbatch * Nq - 1) * ldq + heads * 64) * 2);
  const uint32_t ob = fit(((size_t)(nbatch * Nq - 1) * ldo + heads * 64) * 2);
  const uint32_t dob = fit(((size_t)(nbatch * Nq - 1) * lddo + heads * 64) * 2);
  const uint32_t kvb = fit(((size_t)(nkv * Nk - 1) * ldkv + heads * 64) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse, never read zeros
  const int nqb = (Nq + 127) / 128, nkb = (Nk + 127) / 128;
  hipLaunchKernelGGL(sa_bwd_dq_kernel, dim3(nqb * heads * nbatch), dim3(256), 6 * SB_TILE, s, (const bf16_t*)q, ldq,
                     (const bf16_t*)k, (const bf16_t*)v, ldkv, (const bf16_t*)o, ldo, (const bf16_t*)dout, lddo, lse,
                     (bf16_t*)dq, lddq, dvec, nbatch, heads, Nq, Nk, kv_div, scale, sl2, qb, ob, dob, kvb);
  if (dk) {
    hipLaunchKernelGGL(sa_bwd_dkv_kernel, dim3(nkb * heads * nkv), dim3(256), 2 * (4 * SB_TILE + 512), s,
                       (const bf16_t*)q, ldq, (const bf16_t*)k, (const bf16_t*)v, ldkv, (const bf16_t*)dout, lddo, lse,
                       dvec, (bf16_t*)dk, (bf16_t*)dv, lddkv, nkv, heads, Nq, Nk, kv_div, scale, sl2, qb, dob, kvb);
  }
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}
