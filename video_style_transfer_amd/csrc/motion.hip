// Fused motion-module attention block (one launch per BasicTransformerBlock attention of a motion module):
//   y = x + to_out( attention_over_frames( to_qkv( LayerNorm(x) * gamma + beta + pe[frame] ) ) )
// = diffusers BasicTransformerBlock's  norm1 -> (+ sinusoidal PE) -> attn1 -> + residual  (and the same for norm2 /
// attn2, double_self_attention) inside AnimateDiff's motion module (the reference's own copy of the
// block: unziplora_unet/unzip_attention.py:150-151, 196-197; PE: animatediff/temporal_transformer.py:11-27; the
// attention core: TemporalTransformerBlock, temporal_transformer.py:66-68).
//
// Why: at the 64x64 level (C = 320, 131072 tokens per CFG-batched step) the unfused block is four launches that each
// stream the activation through HBM -- LayerNorm (read + write), the q/k/v GEMM (K = 320: fill / epilogue bound),
// the frame-axis attention (read q/k/v, write o) and the out-projection (read o and the residual, write y): ~13
// passes over 84 MB.  Here a workgroup owns 8 pixels x 16 frames = 128 tokens: x is read once, normalised into LDS,
// and everything after that stays on chip until y is written.
// Status: correct, OPT-IN (VST_MOTION_FUSE=1).  It measured 380-415 us per block against 337-345 us for
// the four launches (tools/motion_bench.py): without the weight stream it still takes ~330 us, i.e. the per-workgroup
// compute (both waves of a SIMD in the same phase, every wave re-reading each 32-KiB weight slice from LDS) is the
// bound, not HBM.
//
// Layout: tokens are rows (b * F + f) * HW + p (token-major NHWC); the workgroup's row r = pp * 16 + f (pixel-major),
// so wave w owns pixel p0 + w: its 16 rows are exactly the 16 frames attended over, one 16-row MFMA block.
// Per head h (D = 40, padded to 48 = three 16-wide blocks, the pad rows of every weight slice zero):
//   q, k = N . W^T  as mfma(W rows, N rows)  -> lane (token, g) holds 4 consecutive d      (16x16x32, K = C)
//   v^T  = W . N^T  as mfma(N rows, W rows)  -> lane (d, g) holds 4 consecutive tokens
//   S^T = K . Q^T, O^T = V^T . P^T, y += Wo_h . O^T on 16x16x16 MFMAs whose operand layouts ARE those accumulator
//   layouts (lane (i, g) holds elements 4g..4g+3 of row i), so nothing moves between registers and LDS.
// Weight slices (q / k / v rows of head h: [48][C]; Wo columns of head h: [C][48]) stream through two LDS buffers by
// LDS-DMA, one slice ahead.  Roundings are the unfused path's: LayerNorm output, q / k / v, P (unnormalised), O, and
// the projection output before the residual add are bf16.
#include "attn_common.h"

namespace vst {

namespace {

constexpr int MB_C = 320, MB_D = 40, MB_H = 8, MB_F = 16, MB_PB = 8;  // channels, head dim, heads, frames, pixels
constexpr int MB_TOK = MB_PB * MB_F;                                  // 128 tokens per workgroup
constexpr int MB_NSTRIDE = MB_C * 2 + 16;                             // 656 B: conflict-free 16-B row reads
constexpr int MB_NS_BYTES = MB_TOK * MB_NSTRIDE;                      // 83968
constexpr int MB_QCH = MB_C / 8 + 1;                                  // 41 16-B slots per q/k/v slice row (1 pad)
constexpr int MB_QK_SLOTS = 48 * MB_QCH;                              // 1968 (rows 40-47 zero)
constexpr int MB_OCH = 7;                                             // Wo slice row: 5 data slots + 2 pad (112 B)
constexpr int MB_O_SLOTS = MB_C * MB_OCH;                             // 2240
constexpr int MB_SLICE = 35840;                                       // >= 1968 * 16 and 2240 * 16
constexpr int MB_LDS = MB_NS_BYTES + 2 * MB_SLICE;                    // 155648
static_assert(MB_QK_SLOTS * 16 <= MB_SLICE && MB_O_SLOTS * 16 <= MB_SLICE && MB_LDS <= 160 * 1024, "LDS");

typedef __attribute__((address_space(3))) void mb_lds_void;

__device__ __forceinline__ void mb_dma16(__amdgpu_buffer_rsrc_t r, char* lds_piece, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (mb_lds_void*)((__attribute__((address_space(3))) char*)(uintptr_t)lds_piece), 16, off, 0, 0, 0);
}

// wait until at most n of this wave's vector-memory operations are outstanding (n = the pieces of the NEXT slice)
__device__ __forceinline__ void mb_vmwait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
  }
}

// raw workgroup barrier: __syncthreads() would also drain vmcnt and so wait for the slice prefetched one step ahead
__device__ __forceinline__ void mb_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ s16x4 mb_pack4(f32x4 a) {
  const u32x2 w{pack2bf(a[0], a[1]), pack2bf(a[2], a[3])};
  return __builtin_bit_cast(s16x4, w);
}

struct MbArgs {
  const bf16_t* x;
  int ldx;
  const float* gamma;
  const float* beta;
  float eps;
  const float* pe;  // [F][C] fp32 (row f added to frame f's normalised row) or null
  const bf16_t* wqkv;  // [3C][C]: q rows, k rows, v rows (head h = rows h*D .. h*D+D-1 of each)
  int ldw;
  const float* bqkv;  // [3C] or null
  const bf16_t* wo;   // [C][C]
  int ldwo;
  const float* bo;    // [C] or null
  bf16_t* y;
  int ldy;
  int HW;
  float scale_log2;
  uint32_t x_bytes, w_bytes, wo_bytes;
};

}  // namespace

__global__ __launch_bounds__(512, 1) void motion_attn_block_kernel(MbArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* NS = smem;                          // normalised tokens [128][C] bf16, 656-B rows
  char* SL = smem + MB_NS_BYTES;            // two weight-slice buffers
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int pix_blocks = a.HW / MB_PB;
  const int b = blockIdx.x / pix_blocks, p0 = (blockIdx.x - b * pix_blocks) * MB_PB;
  auto grow = [&](int f) { return (b * MB_F + f) * a.HW + p0 + w; };  // global row of this wave's frame f

  const auto rx = make_rsrc(a.x, a.x_bytes);
  const auto rw = make_rsrc(a.wqkv, a.w_bytes);
  const auto rwo = make_rsrc(a.wo, a.wo_bytes);

  // ---- weight slice s (0..31): head s / 4, kind s % 4 (q, k, v rows of head h: [48][C]; Wo columns: [C][48]) ----
  auto slice_pieces = [&](int s) {  // DMA instructions this wave issues for slice s
    const int n = (s & 3) == 3 ? (MB_O_SLOTS + 63) / 64 : (MB_QK_SLOTS + 63) / 64;
    return (n - w + 7) / 8;
  };
  auto issue_slice = [&](int s) {
    const int h = s >> 2, kind = s & 3;
    char* base = SL + (s & 1) * MB_SLICE;
    if (kind < 3) {
      const int n = (MB_QK_SLOTS + 63) / 64;
      for (int i = w; i < n; i += 8) {
        const int slot = i * 64 + lane, row = slot / MB_QCH, ch = slot - row * MB_QCH;
        const bool ok = slot < MB_QK_SLOTS && row < MB_D && ch < MB_C / 8;
        const int off = ok ? (((kind * MB_C + h * MB_D + row) * a.ldw + ch * 8) * 2) : kOOB;
        mb_dma16(rw, base + i * 1024, off);
      }
    } else {
      const int n = (MB_O_SLOTS + 63) / 64;
      for (int i = w; i < n; i += 8) {
        const int slot = i * 64 + lane, row = slot / MB_OCH, ch = slot - row * MB_OCH;
        const bool ok = slot < MB_O_SLOTS && ch < MB_D / 8;
        const int off = ok ? ((row * a.ldwo + h * MB_D + ch * 8) * 2) : kOOB;
        mb_dma16(rwo, base + i * 1024, off);
      }
    }
  };

  issue_slice(0);  // first weight slice in flight while the tokens are normalised

  // ---- LayerNorm (+ PE) of this wave's 16 rows into NS: lane (frame fr, g) holds chunks g + 4i, i < 10 ----
  {
    constexpr int CPL = MB_C / 8 / 4;  // 10
    float v[CPL][8];
    const int row = grow(fr);
#pragma unroll
    for (int i = 0; i < CPL; ++i) unpack8(buf_load16(rx, (row * a.ldx + (g + 4 * i) * 8) * 2), v[i]);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float mean = s * (1.0f / MB_C);
    float q2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q2 += d * d; }
    q2 += __shfl_xor(q2, 16);
    q2 += __shfl_xor(q2, 32);
    const float rstd = rsqrtf(q2 * (1.0f / MB_C) + a.eps);
    char* nrow = NS + (w * MB_F + fr) * MB_NSTRIDE;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c0 = (g + 4 * i) * 8;
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(a.gamma + c0), g1 = *reinterpret_cast<const f32x4*>(a.gamma + c0 + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.beta + c0), b1 = *reinterpret_cast<const f32x4*>(a.beta + c0 + 4);
      f32x4 p0 = f32x4{0.f, 0.f, 0.f, 0.f}, p1 = p0;
      if (a.pe) {
        p0 = *reinterpret_cast<const f32x4*>(a.pe + fr * MB_C + c0);
        p1 = *reinterpret_cast<const f32x4*>(a.pe + fr * MB_C + c0 + 4);
      }
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = (v[i][e] - mean) * (rstd * g0[e]) + b0[e] + p0[e];
        o[e + 4] = (v[i][e + 4] - mean) * (rstd * g1[e]) + b1[e] + p1[e];
      }
      *reinterpret_cast<u32x4*>(nrow + c0 * 2) = pack8(o);
    }
  }
  // this wave's A fragments of N (rows = its 16 tokens), k-chunk kk: columns 32 kk + 8 g .. +7 (constant all kernel)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // (re-read per slice from NS: keeping all ten in registers left the compiler no room to run the slice reads ahead)
  const char* nrow_a = NS + (w * MB_F + fr) * MB_NSTRIDE + g * 16;

  f32x4 yacc[MB_C / 16];  // out-projection accumulators: lane (token fr, g) holds y[token][16 i + 4 g + e]
#pragma unroll
  for (int i = 0; i < MB_C / 16; ++i) yacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 qa[3], ka[3], va[3];
  s16x4 ob[3];
  const s16x4 zero4 = {0, 0, 0, 0};

  for (int s = 0; s < 4 * MB_H; ++s) {
    const int h = s >> 2, kind = s & 3;
    if (s + 1 < 4 * MB_H) {
      issue_slice(s + 1);
      mb_vmwait(slice_pieces(s + 1));  // slice s landed (its DMAs are older than slice s + 1's)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mb_barrier();  // every wave's pieces of slice s landed -> visible to all (slice s + 1 stays in flight)
    const char* S = SL + (s & 1) * MB_SLICE;
    if (kind < 3) {
      // q / k: acc = mfma(W rows d, N rows token); v^T: acc = mfma(N rows token, W rows d)
      f32x4 acc[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // software-pipelined over the ten k-steps: the N and W fragments of k-step kk + 1 are read before the MFMAs
      // of k-step kk are issued (the two waves of a SIMD run the same phase, so only in-wave overlap hides LDS latency)
      bf16x8 nf[2], wf[2][3];
      auto load_k = [&](int kk, int u) {
        nf[u] = *reinterpret_cast<const bf16x8*>(nrow_a + kk * 64);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          wf[u][j] = *reinterpret_cast<const bf16x8*>(S + (j * 16 + fr) * (MB_QCH * 16) + (kk * 32 + g * 8) * 2);
      };
      load_k(0, 0);
#pragma unroll
      for (int kk = 0; kk < MB_C / 32; ++kk) {
        const int u = kk & 1;
        if (kk + 1 < MB_C / 32) load_k(kk + 1, u ^ 1);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[j] = kind < 2 ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u][j], nf[u], acc[j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(nf[u], wf[u][j], acc[j], 0, 0, 0);
      }
      // + bias (fp32), rounding to bf16 happens at the packing below
      if (a.bqkv) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (kind < 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int d = j * 16 + 4 * g + e;
              acc[j][e] += d < MB_D ? a.bqkv[kind * MB_C + h * MB_D + d] : 0.f;
            }
          } else {
            const int d = j * 16 + fr;
            const float bv = d < MB_D ? a.bqkv[2 * MB_C + h * MB_D + d] : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][e] += bv;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (kind == 0) qa[j] = acc[j];
        else if (kind == 1) ka[j] = acc[j];
        else va[j] = acc[j];
      }
      if (kind == 2) {
        // ---- attention over the 16 frames of this wave's pixel, head h ----
        // S^T[key][q] = sum_j K_j . Q_j^T  (lane (q, g) holds keys 4g + e)
        f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 3; ++j) st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(mb_pack4(ka[j]), mb_pack4(qa[j]), st, 0, 0, 0);
        float mx = fmaxf(fmaxf(st[0], st[1]), fmaxf(st[2], st[3]));
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mb = mx * a.scale_log2;
        f32x4 pv;
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pv[e] = fast_exp2(st[e] * a.scale_log2 - mb);
          ls += pv[e];
        }
        ls += __shfl_xor(ls, 16);
        ls += __shfl_xor(ls, 32);
        const float inv = 1.0f / ls;
        const s16x4 pb = mb_pack4(pv);  // P (unnormalised, bf16): lane (q, g) holds P[q][keys 4g + e]
        // O^T[d][q] = V^T . P^T per 16-wide d block; O = O^T / l, rounded to bf16 -> out-projection operand
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(mb_pack4(va[j]), pb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          ob[j] = j * 16 + 4 * g < MB_D ? mb_pack4(o * inv) : zero4;
        }
      }
    } else {
      // ---- y += Wo[:, h D .. h D + 48) . O^T  (Wo slice [C][48], 112-B rows; columns 40-47 zero) ----
      s16x4 wo_f[2][3];
      auto load_o = [&](int i, int u) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          wo_f[u][j] = *reinterpret_cast<const s16x4*>(S + (i * 16 + fr) * (MB_OCH * 16) + (j * 16 + 4 * g) * 2);
      };
      load_o(0, 0);
#pragma unroll
      for (int i = 0; i < MB_C / 16; ++i) {
        const int u = i & 1;
        if (i + 1 < MB_C / 16) load_o(i + 1, u ^ 1);
#pragma unroll
        for (int j = 0; j < 3; ++j) yacc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wo_f[u][j], ob[j], yacc[i], 0, 0, 0);
      }
    }
    mb_barrier();  // every wave done with buffer s & 1 before slice s + 2 is issued into it
  }

  // ---- y = bf16(bf16(acc + bo) + x): lane (frame fr, g) holds columns 16 i + 4 g .. +3 of its token ----
  const int row = grow(fr);
#pragma unroll
  for (int i = 0; i < MB_C / 16; ++i) {
    const int n = i * 16 + 4 * g;
    const u32x2 r2 = buf_load8(rx, (row * a.ldx + n) * 2);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t = round_bf(yacc[i][e] + (a.bo ? a.bo[n + e] : 0.f));
      const float res = __uint_as_float(e & 1 ? (r2[e >> 1] & 0xffff0000u) : (r2[e >> 1] << 16));
      o[e] = t + res;
    }
    const u32x2 v{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
    *reinterpret_cast<u32x2*>(a.y + (size_t)row * a.ldy + n) = v;
  }
}

}  // namespace vst

using namespace vst;

extern "C" int vst_motion_attention_block_supported(int C, int F, int HW, int heads) {
  return (C == MB_C && F == MB_F && heads == MB_H && HW > 0 && HW % MB_PB == 0) ? 1 : 0;
}

extern "C" int vst_motion_attention_block(const void* x, int ldx, int nclip, int F, int HW, int C, int heads,
                                          const float* gamma, const float* beta, float eps, const float* pe,
                                          const void* wqkv, int ldw, const float* bqkv, const void* wo, int ldwo,
                                          const float* bo, float scale, void* y, int ldy, void* stream) {
  if (!x || !gamma || !beta || !wqkv || !wo || !y || nclip <= 0) return VST_ERR_ARG;
  if (!vst_motion_attention_block_supported(C, F, HW, heads)) return VST_ERR_UNSUPPORTED;
  if ((ldx & 7) || (ldw & 7) || (ldwo & 7) || (ldy & 7) || ldx < C || ldy < C || ldw < C || ldwo < C) return VST_ERR_ARG;
  if (x == y) return VST_ERR_ARG;  // the residual is re-read at the end: out of place only
  if (((uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)pe) & 15) return VST_ERR_ARG;  // 16-B vector loads
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)motion_attn_block_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MB_LDS);
    attr = true;
  }
  MbArgs a{};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.gamma = gamma; a.beta = beta; a.eps = eps; a.pe = pe;
  a.wqkv = (const bf16_t*)wqkv; a.ldw = ldw; a.bqkv = bqkv; a.wo = (const bf16_t*)wo; a.ldwo = ldwo; a.bo = bo;
  a.y = (bf16_t*)y; a.ldy = ldy; a.HW = HW; a.scale_log2 = scale * 1.4426950408889634f;
  const size_t rows = (size_t)nclip * F * HW;
  auto clampb = [](size_t v) { return v > 0x7fffffffULL ? 0x7fffffffu : (uint32_t)v; };
  a.x_bytes = clampb(((rows - 1) * ldx + C) * 2);
  a.w_bytes = clampb(((size_t)(3 * C - 1) * ldw + C) * 2);
  a.wo_bytes = clampb(((size_t)(C - 1) * ldwo + C) * 2);
  if (rows * ldx * 2 > 0x7fffffffULL || rows * ldy * 2 > 0x7fffffffULL) return VST_ERR_ARG;
  hipLaunchKernelGGL(motion_attn_block_kernel, dim3(nclip * (HW / MB_PB)), dim3(512), MB_LDS, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}
