// bf16 MFMA GEMM for every dense contraction on the AnimateDiff-XL denoise path:
//   C[M,N] = epilogue( A[M,K] . W[N,K]^T )
// W is nn.Linear layout ([out, in], K contiguous) so both operands are K-contiguous
// and every MFMA fragment is one 16-byte LDS read.
//
// A operand loaders (template AMODE):
//   0  dense rows, optionally split along K into two sources (A1 for k < K1, A2
//      after).  The split carries (a) channel concatenation without a copy and
//      (b) the UnZipLoRA low-rank delta as extra K columns: [x | x.Acat^T] .
//      [W | s.(B (.) m)]^T  = x W^T + s.Delta(x)  (unziplora_linear_layer.py:298-346).
//   1  implicit-GEMM 3x3 conv over NHWC activations (per-frame SDXL conv, diffusers
//      ResnetBlock2D / Downsample2D / Upsample2D): K = (ky,kx,ci), zero padding via
//      out-of-range buffer loads, stride 1/2, fused nearest-2x upsample, two-source
//      channel concat (up-block skip connections).
//   2  same conv with a scalar gather (tiny Cin, e.g. conv_in with 4 channels).
// Epilogues (template EPI): 0 = +bias[n] +row_bias[m/div][n] +residual[m,n];
//   1 = GEGLU (tile columns [0,64) hidden, [64,128) gate of the same 64 outputs;
//   the host interleaves the weight rows accordingly).
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 via 4x4
// v_mfma_f32_16x16x32_bf16.  Register-staged double-buffered LDS with the
// load-early / write-late split; XOR-swizzled 128-byte LDS rows (conflict-free
// ds_read_b128 fragment reads); XCD-aware tile order; fp32 LDS-staged epilogue
// with 16-byte coalesced stores.
#include "vst_common.h"

namespace vst {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile
constexpr int GEMM_LDS = 4 * TILE_BYTES;  // 2 buffers x (A,B) = 64 KiB (= fp32 C tile)

struct GemmArgs {
  const bf16_t* A1; const bf16_t* A2;
  int lda1, lda2, K1;
  // conv geometry (AMODE 1/2): input NHWC [nimg, H, W, C1 (+C2)] -> output [nimg, OH, OW, N]
  int H, W, C1, C2, OH, OW, stride, up;
  const bf16_t* Wt; int ldw;
  int M, N, K;
  const float* bias;
  const float* rbias; int rbias_div, ldrb;
  const bf16_t* R; int ldr;
  bf16_t* C; int ldc;
  uint32_t a1_bytes, a2_bytes, w_bytes, r_bytes;
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int AMODE, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int nbn = (p.N + BN - 1) / BN, nbm = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nbn * nbm);
  const int bm = wg / nbn, bn = wg - bm * nbn;
  const int m0 = bm * BM, n0 = bn * BN;

  const auto ra1 = make_rsrc(p.A1, p.a1_bytes);
  const auto ra2 = make_rsrc(p.A2 ? p.A2 : p.A1, p.A2 ? p.a2_bytes : 0u);
  const auto rw = make_rsrc(p.Wt, p.w_bytes);

  const int sc = tid & 7, sr = tid >> 3;  // staging chunk / base row
  // per-staged-row A geometry (fixed over the K loop)
  int rowA[4], oyv[4], oxv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + sr + 32 * i;
    if (AMODE == 0) {
      rowA[i] = m < p.M ? m : -1;
      oyv[i] = oxv[i] = 0;
    } else {
      if (m < p.M) {
        const int hw = p.OH * p.OW;
        const int img = m / hw, rem = m - img * hw;
        rowA[i] = img;
        oyv[i] = rem / p.OW;
        oxv[i] = rem - oyv[i] * p.OW;
      } else {
        rowA[i] = -1; oyv[i] = oxv[i] = 0;
      }
    }
  }
  int rowB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + sr + 32 * i;
    rowB[i] = n < p.N ? n : -1;
  }

  u32x4 va[4], vb[4];
  const int nk = (p.K + BK - 1) / BK;
  const int Ctot = p.C1 + p.C2;

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    const int k = k0 + sc * 8;
    // ---- B (weights) ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (rowB[i] >= 0 && k < p.K) ? (rowB[i] * p.ldw + k) * 2 : kOOB;
      vb[i] = buf_load16(rw, off);
    }
    // ---- A ----
    if (AMODE == 0) {
      if (k0 < p.K1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int off = (rowA[i] >= 0 && k < p.K1) ? (rowA[i] * p.lda1 + k) * 2 : kOOB;
          va[i] = buf_load16(ra1, off);
        }
      } else {
        const int kk = k - p.K1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int off = (rowA[i] >= 0 && k < p.K) ? (rowA[i] * p.lda2 + kk) * 2 : kOOB;
          va[i] = buf_load16(ra2, off);
        }
      }
    } else if (AMODE == 1) {
      const int tap = k0 / Ctot;
      const int ci0 = k0 - tap * Ctot;
      const int ky = tap / 3, kx = tap - ky * 3;
      const bool first = ci0 < p.C1;
      const int cs = first ? p.C1 : p.C2;
      const int ci = (first ? ci0 : ci0 - p.C1) + sc * 8;
      const auto rs = first ? ra1 : ra2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int iy, ix;
        bool ok = rowA[i] >= 0 && tap < 9;
        if (p.up) {
          const int uy = oyv[i] + ky - 1, ux = oxv[i] + kx - 1;
          ok = ok && uy >= 0 && uy < 2 * p.H && ux >= 0 && ux < 2 * p.W;
          iy = uy >> 1; ix = ux >> 1;
        } else {
          iy = oyv[i] * p.stride + ky - 1; ix = oxv[i] * p.stride + kx - 1;
          ok = ok && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        }
        const int off = ok ? (((rowA[i] * p.H + iy) * p.W + ix) * cs + ci) * 2 : kOOB;
        va[i] = buf_load16(rs, off);
      }
    } else {  // scalar gather conv (single source)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kj = k + j;
          const int tap = kj / p.C1, ci = kj - tap * p.C1;
          const int ky = tap / 3, kx = tap - ky * 3;
          int iy, ix;
          bool ok = rowA[i] >= 0 && kj < p.K1;
          if (p.up) {
            const int uy = oyv[i] + ky - 1, ux = oxv[i] + kx - 1;
            ok = ok && uy >= 0 && uy < 2 * p.H && ux >= 0 && ux < 2 * p.W;
            iy = uy >> 1; ix = ux >> 1;
          } else {
            iy = oyv[i] * p.stride + ky - 1; ix = oxv[i] * p.stride + kx - 1;
            ok = ok && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
          }
          const int off = ok ? (((rowA[i] * p.H + iy) * p.W + ix) * p.C1 + ci) * 2 : kOOB;
          e[j] = buf_load2(ra1, off);
        }
        va[i] = u32x4{(uint32_t)e[0] | ((uint32_t)e[1] << 16), (uint32_t)e[2] | ((uint32_t)e[3] << 16),
                      (uint32_t)e[4] | ((uint32_t)e[5] << 16), (uint32_t)e[6] | ((uint32_t)e[7] << 16)};
      }
    }
  };

  auto store_tile = [&](int buf) {
    char* As = smem + buf * 2 * TILE_BYTES;
    char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = sr + 32 * i;
      *reinterpret_cast<u32x4*>(As + swz(row, sc)) = va[i];
      *reinterpret_cast<u32x4*>(Bs + swz(row, sc)) = vb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
    const char* As = smem + cur * 2 * TILE_BYTES;
    const char* Bs = As + TILE_BYTES;
    // skip the second 32-deep half when it lies wholly beyond K (LoRA tail tile)
    const int nkk = (kt * BK + 32 < p.K) ? 2 : 1;
    for (int kk = 0; kk < nkk; ++kk) {
      bf16x8 af[4], bfr[4];
      const int chunk = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + swz(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wc * 64 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + swz(row, chunk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue: fp32 tile through LDS ----------------
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + i * 16 + fq * 4 + r;
        const int col = wc * 64 + j * 16 + fr;
        Cs[row * BN + col] = acc[i][j][r];
      }
  __syncthreads();

  const auto rr = make_rsrc(p.R ? p.R : p.Wt, p.R ? p.r_bytes : 0u);
  if (EPI == 0) {
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int idx = tid + 256 * it;
      const int row = idx >> 4, cc = idx & 15;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      float v[8];
      const f32x4 c0 = *reinterpret_cast<const f32x4*>(Cs + row * BN + cc * 8);
      const f32x4 c1 = *reinterpret_cast<const f32x4*>(Cs + row * BN + cc * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = c0[e]; v[e + 4] = c1[e]; }
      const int nv = min(8, p.N - n);
      if (p.bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) if (e < nv) v[e] += p.bias[n + e];
      }
      if (p.rbias) {
        const float* rb = p.rbias + (size_t)(m / p.rbias_div) * p.ldrb + n;
#pragma unroll
        for (int e = 0; e < 8; ++e) if (e < nv) v[e] += rb[e];
      }
      if (nv == 8) {
        if (p.R) {
          float r8[8];
          unpack8(buf_load16(rr, (m * p.ldr + n) * 2), r8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += r8[e];
        }
        *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + n) = pack8(v);
      } else {
        for (int e = 0; e < nv; ++e) {
          float x = v[e];
          if (p.R) x += bf2f(p.R[(size_t)m * p.ldr + n + e]);
          p.C[(size_t)m * p.ldc + n + e] = f2bf(x);
        }
      }
    }
  } else {  // GEGLU: out[m, n0/2 + c] = (h + bh) * gelu(g + bg)
#pragma unroll 2
    for (int it = 0; it < 4; ++it) {
      const int idx = tid + 256 * it;
      const int row = idx >> 3, cc = idx & 7;
      const int m = m0 + row;
      if (m >= p.M || n0 >= p.N) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float h = Cs[row * BN + cc * 8 + e];
        float g = Cs[row * BN + 64 + cc * 8 + e];
        if (p.bias) { h += p.bias[n0 + cc * 8 + e]; g += p.bias[n0 + 64 + cc * 8 + e]; }
        v[e] = h * gelu_erf(g);
      }
      *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + (n0 >> 1) + cc * 8) = pack8(v);
    }
  }
}

template <int AMODE, int EPI>
static int launch(const GemmArgs& a, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<AMODE, EPI>), dim3(nwg), dim3(256), GEMM_LDS, s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

static inline uint32_t clamp_bytes(size_t b) { return b > 0x7fffffffULL ? 0x7fffffffu : (uint32_t)b; }

}  // namespace vst

using namespace vst;

extern "C" int vst_gemm(const void* A, int lda, const void* A2, int lda2, int K1,
                        const void* W, int ldw, int M, int N, int K,
                        const float* bias, const float* row_bias, int row_bias_div, int ld_row_bias,
                        const void* R, int ldr, void* C, int ldc, int epilogue, void* stream) {
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0) return VST_ERR_ARG;
  if ((K & 7) || (lda & 7) || (ldw & 7) || (ldc & 7)) return VST_ERR_ARG;
  if (A2) {
    if (K1 <= 0 || K1 % BK || K1 >= K || (lda2 & 7)) return VST_ERR_ARG;
  } else {
    K1 = K;
  }
  if (epilogue == 1 && (N % BN)) return VST_ERR_ARG;
  if (R && (ldr & 7)) return VST_ERR_ARG;
  if (row_bias && row_bias_div <= 0) return VST_ERR_ARG;
  GemmArgs a{};
  a.A1 = (const bf16_t*)A; a.A2 = (const bf16_t*)A2; a.lda1 = lda; a.lda2 = lda2; a.K1 = K1;
  a.Wt = (const bf16_t*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.bias = bias; a.rbias = row_bias; a.rbias_div = row_bias_div; a.ldrb = ld_row_bias;
  a.R = (const bf16_t*)R; a.ldr = ldr; a.C = (bf16_t*)C; a.ldc = ldc;
  a.a1_bytes = clamp_bytes(((size_t)(M - 1) * lda + K1) * 2);
  a.a2_bytes = A2 ? clamp_bytes(((size_t)(M - 1) * lda2 + (K - K1)) * 2) : 0;
  a.w_bytes = clamp_bytes(((size_t)(N - 1) * ldw + K) * 2);
  a.r_bytes = R ? clamp_bytes(((size_t)(M - 1) * ldr + N) * 2) : 0;
  a.C1 = 0; a.C2 = 0; a.stride = 1; a.up = 0;
  hipStream_t s = (hipStream_t)stream;
  return epilogue == 1 ? launch<0, 1>(a, s) : launch<0, 0>(a, s);
}

// 3x3 conv, padding 1, NHWC.  x1: [nimg,H,W,C1], optional x2: [nimg,H,W,C2] concatenated
// on channels.  Wt: [Cout][3][3][C1+C2].  stride 1 or 2; upsample=1 applies nearest 2x to
// the input first (output 2H x 2W).  Output [nimg, OH, OW, Cout] with row stride ldc.
extern "C" int vst_conv3x3(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W,
                           int stride, int upsample, const void* Wt, int Cout,
                           const float* bias, const float* row_bias, int row_bias_div,
                           const void* R, int ldr, void* out, int ldc, void* stream) {
  if (!x1 || !Wt || !out || nimg <= 0 || H <= 0 || W <= 0 || Cout <= 0) return VST_ERR_ARG;
  if (stride != 1 && stride != 2) return VST_ERR_ARG;
  if (upsample && stride != 1) return VST_ERR_ARG;
  const int Ct = C1 + (x2 ? C2 : 0);
  const bool vec = (Ct % BK == 0) && (C1 % 8 == 0);
  if (x2 && !vec) return VST_ERR_ARG;
  GemmArgs a{};
  a.OH = upsample ? 2 * H : (stride == 2 ? (H + 1) / 2 : H);
  a.OW = upsample ? 2 * W : (stride == 2 ? (W + 1) / 2 : W);
  a.A1 = (const bf16_t*)x1; a.A2 = (const bf16_t*)x2; a.C1 = C1; a.C2 = x2 ? C2 : 0;
  a.H = H; a.W = W; a.stride = stride; a.up = upsample;
  a.K = 9 * Ct; a.K1 = a.K;
  a.M = nimg * a.OH * a.OW; a.N = Cout;
  if (!vec) a.K = (a.K + 7) & ~7;  // scalar gather: pad K to a chunk; weight rows padded too
  a.Wt = (const bf16_t*)Wt; a.ldw = a.K;
  a.bias = bias; a.rbias = row_bias; a.rbias_div = row_bias_div; a.ldrb = Cout;
  a.R = (const bf16_t*)R; a.ldr = ldr; a.C = (bf16_t*)out; a.ldc = ldc;
  a.a1_bytes = clamp_bytes((size_t)nimg * H * W * C1 * 2);
  a.a2_bytes = x2 ? clamp_bytes((size_t)nimg * H * W * C2 * 2) : 0;
  a.w_bytes = clamp_bytes((size_t)Cout * a.K * 2);
  a.r_bytes = R ? clamp_bytes(((size_t)(a.M - 1) * ldr + Cout) * 2) : 0;
  if ((ldc & 7) && Cout >= 8) return VST_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  return vec ? launch<1, 0>(a, s) : launch<2, 0>(a, s);
}
