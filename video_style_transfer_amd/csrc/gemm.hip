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
// Epilogues (template EPI): 0 = +bias[n] +row_bias[m/div][n] +residual[m,n] -> bf16;
//   1 = GEGLU (per 64 columns: [0,32) hidden, [32,64) gate of the same 32 outputs;
//   the host interleaves the weight rows accordingly); 2 = fp32 split-K partial slab
//   (the epilogue then runs in gemm_splitk_reduce_kernel).
//
// Tile BM=128 x BN (128 or 64) x BK=64, 256 threads = 4 waves (2x2), each wave 64 x BN/2 via
// v_mfma_f32_16x16x32_bf16.  Register-staged double-buffered LDS with the load-early /
// write-late split; XOR-swizzled 128-byte LDS rows (conflict-free ds_read_b128 fragment
// reads); XCD-aware tile order; fp32 LDS-staged epilogue with 16-byte coalesced stores.
// Host-side heuristic (vst_gemm): BN=64 when the 128x128 grid would run in few waves on
// 256 CUs (tail effect), split-K (blockIdx.z) when even that grid cannot fill the chip.
#include <cstdlib>

#include "gemm_common.h"

namespace vst {

constexpr int BM = 128, BK = 64;
constexpr int A_TILE = BM * BK * 2;  // 16 KiB

template <int BN>
constexpr int gemm_lds_bytes() {
  return (2 * (A_TILE + BN * BK * 2)) > (BM * BN * 4) ? 2 * (A_TILE + BN * BK * 2) : BM * BN * 4;
}

template <int AMODE, int EPI, int BN>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs p) {
  constexpr int B_TILE = BN * BK * 2;
  constexpr int STAGE = A_TILE + B_TILE;
  constexpr int NT = BN / 32;      // 16-wide n tiles per wave
  constexpr int BCH = BN / 32;     // B staging chunks per thread
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
  int rowB[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int n = n0 + sr + 32 * i;
    rowB[i] = n < p.N ? n : -1;
  }

  u32x4 va[4], vb[BCH];
  const int nk_all = (p.K + BK - 1) / BK;
  int kt_beg = 0, kt_end = nk_all;
  if (EPI == 2) {
    const int z = blockIdx.z;
    kt_beg = (int)((long long)nk_all * z / p.splits);
    kt_end = (int)((long long)nk_all * (z + 1) / p.splits);
  }
  const int Ctot = p.C1 + p.C2;

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    const int k = k0 + sc * 8;
    // ---- B (weights) ----
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
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
          iy = oyv[i] * p.stride + ky - 1 + p.pad0; ix = oxv[i] * p.stride + kx - 1 + p.pad0;
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
            iy = oyv[i] * p.stride + ky - 1 + p.pad0; ix = oxv[i] * p.stride + kx - 1 + p.pad0;
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
    char* As = smem + buf * STAGE;
    char* Bs = As + A_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(As + swz(sr + 32 * i, sc)) = va[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i) *reinterpret_cast<u32x4*>(Bs + swz(sr + 32 * i, sc)) = vb[i];
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  if (kt_beg < kt_end) {
    load_tile(kt_beg);
    store_tile(0);
  }
  __syncthreads();

  for (int kt = kt_beg; kt < kt_end; ++kt) {
    const int cur = (kt - kt_beg) & 1;
    if (kt + 1 < kt_end) load_tile(kt + 1);
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_TILE;
    // skip the second 32-deep half when it lies wholly beyond K (LoRA tail tile)
    const int nkk = (kt * BK + 32 < p.K) ? 2 : 1;
    for (int kk = 0; kk < nkk; ++kk) {
      bf16x8 af[4], bfr[NT];
      const int chunk = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(As + swz(wr * 64 + i * 16 + fr, chunk));
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + swz(wc * (BN / 2) + j * 16 + fr, chunk));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kt_end) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue: fp32 tile through LDS ----------------
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + i * 16 + fq * 4 + r;
        const int col = wc * (BN / 2) + j * 16 + fr;
        Cs[row * BN + col] = acc[i][j][r];
      }
  __syncthreads();

  constexpr int CPR = BN / 8;  // 8-column chunks per tile row
  if (EPI == 2) {
    float* slab = p.ws + (size_t)blockIdx.z * p.M * p.N;
#pragma unroll 2
    for (int it = 0; it < BM * CPR / 256; ++it) {
      const int idx = tid + 256 * it;
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      const f32x4 c0 = *reinterpret_cast<const f32x4*>(Cs + row * BN + cc * 8);
      const f32x4 c1 = *reinterpret_cast<const f32x4*>(Cs + row * BN + cc * 8 + 4);
      float* dst = slab + (size_t)m * p.N + n;
      if (n + 8 <= p.N) {
        *reinterpret_cast<f32x4*>(dst) = c0;
        *reinterpret_cast<f32x4*>(dst + 4) = c1;
      } else {
        for (int e = 0; e < p.N - n; ++e) dst[e] = e < 4 ? c0[e] : c1[e - 4];
      }
    }
    return;
  }
  const auto rr = make_rsrc(p.R ? p.R : p.Wt, p.R ? p.r_bytes : 0u);
  if (EPI == 0) {
#pragma unroll 2
    for (int it = 0; it < BM * CPR / 256; ++it) {
      const int idx = tid + 256 * it;
      const int row = idx / CPR, cc = idx - row * CPR;
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
      if (p.rbias || p.R) {  // same rounding points as the ring kernel: bf16 linear output, then the adds
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = round_bf(v[e]);
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
  } else {  // GEGLU (BN == 128): out[m, n0/2 + c] = (h + bh) * gelu(g + bg)
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
        v[e] = round_bf(h) * gelu_erf(round_bf(g));  // bf16 projection output, as the ring kernel stages it
      }
      *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + (n0 >> 1) + cc * 8) = pack8(v);
    }
  }
}

// sum the split-K slabs and apply the epilogue.  geglu: slab columns are the interleaved
// [h(32) | g(32)] blocks; each thread produces 8 output columns.
// Skinny GEMM for the UnZipLoRA down-projection u = x . Acat^T (N = padded 2r per projection <= 64,
// no epilogue): HBM/MALL-bound on reading x once.  A workgroup = 8 waves owns 32 rows (two 16-row
// MFMA fragments) and all N columns; wave w takes the k32-steps w, w+8, ..., issuing a whole group
// of fragment-shaped loads before its MFMAs (lane l reads 16 B of row l&15 at k-chunk l>>4, which IS
// the 16x16x32 operand layout: no LDS staging).  Each W fragment feeds two row fragments, so the W
// bytes read per x byte are N/32 (the L2 traffic that bounded the 16-row version).  The 8 partial
// accumulators are summed through LDS (64 KiB at N = 64).  ceil(M/32) workgroups (256 at M = 8192), 2 per CU.
template <int NJ>
#ifndef VST_SKINNY_MI
#define VST_SKINNY_MI 2
#endif
__global__ __launch_bounds__(512, 2) void gemm_skinny_kernel(GemmArgs p) {
  constexpr int MI = VST_SKINNY_MI, NW = 8;
  constexpr int SK = NJ <= 2 ? 6 : 3;  // k32-steps per wave per load group (all in flight at once)
  __shared__ f32x4 red[NW][MI][NJ][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16 * MI;
  const auto ra = make_rsrc(p.A1, p.a1_bytes);
  const auto rw = make_rsrc(p.Wt, p.w_bytes);
  const int r = lane & 15, kc = (lane >> 4) * 8;
  uint32_t abase[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int arow = m0 + 16 * i + r;
    abase[i] = arow < p.M ? (uint32_t)(arow * p.lda1 + kc) * 2u : (uint32_t)kOOB;
  }
  uint32_t wbase[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    wbase[j] = (16 * j + r) < p.N ? (uint32_t)((16 * j + r) * p.ldw + kc) * 2u : (uint32_t)kOOB;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.K + 31) / 32;
  for (int g = w; g < nk; g += NW * SK) {
    u32x4 a[SK][MI], b[SK][NJ];
#pragma unroll
    for (int t = 0; t < SK; ++t) {
      const int ks = g + NW * t;
      const bool kin = ks < nk && ks * 32 + kc < p.K;
#pragma unroll
      for (int i = 0; i < MI; ++i) a[t][i] = buf_load16(ra, kin ? (int)(abase[i] + ks * 64u) : kOOB);
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[t][j] = buf_load16(rw, kin ? (int)(wbase[j] + ks * 64u) : kOOB);
    }
    // keep the whole group's loads in flight: one memory round trip per group, not one per k-step
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < SK; ++t)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&b[t][j]),
                                                              *reinterpret_cast<bf16x8*>(&a[t][i]), acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) red[w][i][j][lane] = acc[i][j];
  __syncthreads();
  if (w >= MI) return;
  // wave i (< MI) sums row fragment i over the 8 waves and stores it
  const int i = w;
  f32x4 sum[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    sum[j] = red[0][i][j][lane];
#pragma unroll
    for (int q = 1; q < NW; ++q) sum[j] += red[q][i][j][lane];
  }
  // sum[j][e] = C[m0 + 16i + (lane&15)][16j + 4(lane>>4) + e]
  const int m = m0 + 16 * i + r;
  if (m >= p.M) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = 16 * j + 4 * (lane >> 4);
    if (n >= p.N) continue;
    bf16_t* dst = p.C + (size_t)m * p.ldc + n;
    if (n + 4 <= p.N) {
      u32x2 v;
      v[0] = pack2bf(sum[j][0], sum[j][1]);
      v[1] = pack2bf(sum[j][2], sum[j][3]);
      *reinterpret_cast<u32x2*>(dst) = v;
    } else {
      for (int e = 0; e < p.N - n; ++e) dst[e] = f2bf(sum[j][e]);
    }
  }
}

static int launch_skinny(const GemmArgs& a, hipStream_t s) {
  const dim3 grid((a.M + 16 * VST_SKINNY_MI - 1) / (16 * VST_SKINNY_MI));
  switch ((a.N + 15) / 16) {
    case 1: hipLaunchKernelGGL(gemm_skinny_kernel<1>, grid, dim3(512), 0, s, a); break;
    case 2: hipLaunchKernelGGL(gemm_skinny_kernel<2>, grid, dim3(512), 0, s, a); break;
    case 3: hipLaunchKernelGGL(gemm_skinny_kernel<3>, grid, dim3(512), 0, s, a); break;
    case 4: hipLaunchKernelGGL(gemm_skinny_kernel<4>, grid, dim3(512), 0, s, a); break;
    default: return VST_ERR_ARG;
  }
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// Row-vector GEMM for M <= 8 (the time-embedding MLPs and the batched time_emb_proj of every ResnetBlock2D: M = the
// CFG pair, unet_motion.UNetMotionModel.embed / batched_temb; diffusers TimestepEmbedding, ResnetBlock2D).  These
// read N x K weights once to make 2 x N outputs: HBM-bound on W, nothing for MFMA to do.  The 128x128 split-K tiles
// they used to run on spent 46 us per launch on 2 live rows of 128 (0.4 TF/s, profiles/r3s9_kernel_stats.csv).
// A wave owns CPW output columns: lane l reads 16-B k-chunks l, l + 64, ... of each weight row (NT chunks per row in
// flight at once) and the same chunks of the M activation rows (L1/L2 hits: every wave reads the same x), sums in
// fp32, reduces across the wave, then the ring epilogue's rounding points: bias (+GELU) -> bf16 -> + row bias
// + residual -> bf16.  Each output's k order is fixed by (K, lane), so a column's value does not depend on N:
// the batched time_emb_proj equals the per-resnet Linear bit for bit.
template <int MR>
__global__ __launch_bounds__(256) void gemm_rows_kernel(GemmArgs p) {
  constexpr int CPW = 2, NT = MR <= 2 ? 4 : 2;
  const int lane = threadIdx.x & 63;
  const int nb = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CPW;
  if (nb >= p.N) return;  // no barriers below
  const auto ra = make_rsrc(p.A1, p.a1_bytes);
  const auto rw = make_rsrc(p.Wt, p.w_bytes);
  float acc[MR][CPW];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int c = 0; c < CPW; ++c) acc[m][c] = 0.f;
  const int nch = p.K >> 3;
  for (int q0 = 0; q0 < nch; q0 += 64 * NT) {
    u32x4 wv[NT][CPW], xv[NT][MR];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int q = q0 + t * 64 + lane;
      const bool in = q < nch;
#pragma unroll
      for (int c = 0; c < CPW; ++c)
        wv[t][c] = buf_load16(rw, in && nb + c < p.N ? ((nb + c) * p.ldw + q * 8) * 2 : kOOB);
#pragma unroll
      for (int m = 0; m < MR; ++m) xv[t][m] = buf_load16(ra, in && m < p.M ? (m * p.lda1 + q * 8) * 2 : kOOB);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        float w8[8];
        unpack8(wv[t][c], w8);
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          float x8[8];
          unpack8(xv[t][m], x8);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[m][c] = fmaf(x8[e], w8[e], acc[m][c]);
        }
      }
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const float s = wave_sum(acc[m][c]);
      if (lane == m * CPW + c) v = s;
    }
  const int m = lane / CPW, n = nb + lane % CPW;
  if (lane >= MR * CPW || m >= p.M || n >= p.N) return;
  if (p.bias) v += p.bias[n];
  if (p.act) v = gelu_erf(v);
  if (p.rbias || p.R) {
    v = round_bf(v);
    if (p.rbias) v += p.rbias[(size_t)(m / p.rbias_div) * p.ldrb + n];
    if (p.R) v += bf2f(p.R[(size_t)m * p.ldr + n]);
  }
  p.C[(size_t)m * p.ldc + n] = f2bf(v);
}

static bool rows_applies(int M, int N, int K) { return M >= 1 && M <= 8 && N >= 1 && K >= 8 && !(K & 7); }

static int launch_rows(const GemmArgs& a, hipStream_t s) {
  const dim3 grid((a.N + 7) / 8);
  if (a.M <= 2) hipLaunchKernelGGL(gemm_rows_kernel<2>, grid, dim3(256), 0, s, a);
  else if (a.M <= 4) hipLaunchKernelGGL(gemm_rows_kernel<4>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(gemm_rows_kernel<8>, grid, dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(GemmArgs p, int geglu) {
  const int Nout = geglu ? p.N / 2 : p.N;
  const int CPR = (Nout + 7) / 8;
  const size_t total = (size_t)p.M * CPR;
  const size_t slab = (size_t)p.M * p.N;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
    const int m = (int)(idx / CPR);
    const int n = (int)(idx - (size_t)m * CPR) * 8;
    const int nv = min(8, Nout - n);
    float v[8];
    if (!geglu) {
      const float* src = p.ws + (size_t)m * p.N + n;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      for (int z = 0; z < p.splits; ++z) {
        const float* s = src + z * slab;
        if (nv == 8) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(s), b = *reinterpret_cast<const f32x4*>(s + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] += a[e]; v[e + 4] += b[e]; }
        } else {
          for (int e = 0; e < nv; ++e) v[e] += s[e];
        }
      }
      for (int e = 0; e < nv; ++e) {
        if (p.bias) v[e] += p.bias[n + e];
        if (p.rbias || p.R) v[e] = round_bf(v[e]);  // rounding points of the ring kernel's epilogue
        if (p.rbias) v[e] += p.rbias[(size_t)(m / p.rbias_div) * p.ldrb + n + e];
        if (p.R) v[e] += bf2f(p.R[(size_t)m * p.ldr + n + e]);
        if (p.act) v[e] = gelu_erf(v[e]);
      }
    } else {
      const int blk = n / 32, c = n - blk * 32;
      const int hc = blk * 64 + c, gc = hc + 32;
      float h[8], g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { h[e] = 0.f; g[e] = 0.f; }
      for (int z = 0; z < p.splits; ++z) {
        const float* s = p.ws + z * slab + (size_t)m * p.N;
#pragma unroll
        for (int e = 0; e < 8; ++e) { h[e] += s[hc + e]; g[e] += s[gc + e]; }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (p.bias) { h[e] += p.bias[hc + e]; g[e] += p.bias[gc + e]; }
        v[e] = round_bf(h[e]) * gelu_erf(round_bf(g[e]));
      }
    }
    bf16_t* dst = p.C + (size_t)m * p.ldc + n;
    if (nv == 8 && !((uintptr_t)dst & 15)) {
      *reinterpret_cast<u32x4*>(dst) = pack8(v);
    } else {
      for (int e = 0; e < nv; ++e) dst[e] = f2bf(v[e]);
    }
  }
}

template <int AMODE, int EPI, int BN>
static int launch_one(const GemmArgs& a, hipStream_t s, int splits) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<AMODE, EPI, BN>), dim3(nwg, 1, splits), dim3(256), gemm_lds_bytes<BN>(), s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}


constexpr int kCUs = 256;

// tile / split choice.  tile: 0 auto, 1 = 128x128, 2 = 128x64.  splits: 0 auto, >=1 forced.
// tile codes: 1 = 128x128, 2 = 128x64 (gemm_kernel, 4 waves, up to 2 WG/CU);
//             3 = 256x256, 4 = 256x128 (gemm_big_kernel, 8 waves, LDS-DMA staging, 1 WG/CU)

// 256x160 ring tiles for Cout = 320 / 640 convs on full grids: Cout splits into 160-column tiles without the
// 256-wide tiles' padding (Cout = 320: 37.5 % of the MFMA work wasted, 640: 17 %).  Measured in the denoise step
// (tools/ab_bench.sh, profiles/r2_ab_t160.txt): convs 13.1 -> 12.4 ms per step.  The same tiles for N = 640 / 1280
// projections win in isolation (tools/tile_ab.py: 32768x640x672 50.1 -> 43.8 us) but lose in the step
// (74.0 -> 74.7 ms: operands arrive cold), so projections stay on the 8-phase kernel; Cout = 1280 convs gain
// nothing; GEGLU needs 64-column [h | g] blocks.
static bool t160_auto(int M, int N, bool geglu, bool conv) {
  if (geglu || N % 160) return false;
  const bool n_ok = conv && (N == 320 || N == 640);
  const int mb = (M + 255) / 256;
  return n_ok && mb * ((N + 255) / 256) >= kCUs / 2;
}

static void choose(int M, int N, int K, int geglu, int conv, size_t ws_bytes, int& tile, int& splits) {
  const int mt = (M + BM - 1) / BM;
  const int t128 = mt * ((N + 127) / 128);
  const int t64 = mt * ((N + 63) / 64);
  const int nk = (K + BK - 1) / BK;
  const int mb = (M + 255) / 256;
  const int t256 = mb * ((N + 255) / 256), t256n = mb * ((N + 127) / 128);
  const int nk32 = (K + 31) / 32;  // ring kernel k-tiles
  // Tile policy (MI355X, measured in one process per comparison: tools/gemm_ablate.py TILES=..., bench.py):
  // the 256x256 ping-pong ring wins every projection / FF / GEGLU / conv shape of the path with at least a
  // quarter-wave of tiles, including the under-filled M = 8192, N = 1280 grids (160 tiles on 256 CUs:
  // 38 us vs 56 us for 192x256 at K = 1312, 116 vs 190 us at K = 5120; whole step 88.6 vs 92.9 ms);
  // tiny-M GEMMs (text states, temb) use 128x128 with split-K; conv_out (Cout = 4) 128x64.
  // Below half a wave of 256x256 tiles (the training step's 16x16 level: M = 4096, N = 1280 -> 80 tiles) the
  // 128x128 tile's 4x larger grid wins (tools/tile_ab.py: 4096x1280x1312 44.6 -> 30.7 us, x5120 112 -> 82 us).
  if (tile == 0) {
    if (conv && N <= 64) tile = 2;
    else if (t160_auto(M, N, geglu, conv)) tile = 6;
    // under-filled conv grids (the 16x16 level's Cout = 1280 convs: 160 tiles of 256x256): 192x256 tiles, 215 of
    // them, 4.12 -> 3.85 ms per step (profiles/r2_ab_conv_192x256.txt)
    else if (conv && t256 >= kCUs / 2 && t256 < kCUs) tile = 7;
    else if (t256 >= kCUs / 2) tile = 3;
    else tile = 1;
  }
  if (tile == 8 && conv) tile = 3;
  if (geglu && (tile == 2 || tile == 6)) tile = 1;
  const int t160 = mb * ((N + 159) / 160);
  const int t192 = ((M + 191) / 192) * ((N + 255) / 256);
  const int tiles = tile == 1 ? t128 : tile == 2 ? t64 : (tile == 3 || tile == 8) ? t256 : tile == 6 ? t160
                    : tile == 7 ? t192 : t256n;
  if (splits == 0) {
    splits = 1;
    if (tiles < kCUs / 2 && nk32 >= 8) {
      splits = std::min(std::min((2 * kCUs + tiles - 1) / tiles, nk32 / 4), 16);
      if (splits < 2) splits = 1;
    }
  }
  if (tile == 8) splits = 1;  // the 8-phase kernel has no split-K slab epilogue
  if (splits > nk32) splits = nk32;
  if (splits > 1) {
    const size_t need = (size_t)splits * M * N * sizeof(float);
    if (need > ws_bytes) splits = 1;
    if (splits > nk) splits = nk;
  }
}

int launch_gemm_ring(const GemmArgs& a, int amode, int epi, int tile, int splits, hipStream_t s);
int launch_gemm_p8(const GemmArgs& a, int epi, int bn, hipStream_t s);
bool p8_persist_applies(int M, int N, int K, int epi, int bn);
bool p8_lora_persist_on();
int launch_gemm_p8_tattn(const GemmArgs& a, hipStream_t s);
int launch_gemm_p8_lora(const GemmArgs& a, int bn, hipStream_t s);
int launch_gemm_p8_xattn(const GemmArgs& a, hipStream_t s);
int launch_gemm_p8_conv(const GemmArgs& a, int bn, hipStream_t s);

// 8-phase 256x256x64 kernel (gemm_p8.hip) for plain / LoRA-augmented projections and GEGLU (see p8_auto).
static int gemm_p8_env() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("VST_GEMM_P8");
    v = e ? atoi(e) : -1;
  }
  return v;
}

// Automatic choice of the 8-phase kernel (tile 0).  Measured in the denoise step (tools/ab_bench.sh, VST_BENCH_SHAPES,
// one MI355X): it beats the ring on every projection / GEGLU shape -- first at K < 2048 (the 16x16-level
// out-projection 8192x1280x1312 9.53 -> 8.55 ms per step, GEGLU 8192x10240x1280 14.29 -> 13.93, the K = 320 shapes of
// the 64x64 level 3-7 %), and since its loop lost the per-piece K checks also at K >= 2048 (ff.net.2: ring 10.6 ->
// 9.1 ms per step, profiles/r2_ab_p8_all_k.txt).
// VST_GEMM_P8 = 0 off, unset / 1 every shape with at least half a wave of 256x256 tiles.
static int device_cus();
static bool p8_auto(int M, int N, int K, bool geglu) {
  (void)geglu;
  const int e = gemm_p8_env();
  if (e == 0) return false;
  const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
  return t256 >= kCUs / 2 && K >= 128;
}

// 256x192 tiles for the 8-phase kernel (tile code 9, and tile 0 wherever it wins the round count): N = 1280 gives
// 7 column tiles (224 workgroups at M = 8192) instead of 5 (160 of 256 CUs), N = 640 two full rounds instead of
// 1.5, N = 320 a 192 + 128 split instead of 256 + 64.  A 256x192 tile costs ~0.8 of a 256x256 one (its fill and
// epilogue do not shrink with it), so it is taken when ceil(tiles192 / CUs) * 0.8 beats ceil(tiles256 / CUs).
// VST_P8_BN=256 keeps every shape on 256x256 (A/B).
// Forced 8-phase tile width (256 / 192 / 320, 0 = the policy below): VST_P8_BN, or vst_p8_force_bn (tests, A/B).
static int g_p8_force_bn = -1;
static int p8_forced_bn() {
  if (g_p8_force_bn < 0) {
    const char* e = getenv("VST_P8_BN");
    g_p8_force_bn = e ? atoi(e) : 0;
  }
  return g_p8_force_bn;
}

static bool p8_bn192(int M, int N, bool geglu) {
  const int env = p8_forced_bn();
  if (geglu || env == 256 || env == 320) return false;
  const int mb = (M + 255) / 256, cus = device_cus();
  const int r256 = (mb * ((N + 255) / 256) + cus - 1) / cus, r192 = (mb * ((N + 191) / 192) + cus - 1) / cus;
  return env == 192 || 0.8 * r192 < 0.97 * r256;
}

// 128x320 tiles of the 8-phase kernel (tile code 10): every SDXL width (320 / 640 / 1280 / 1920 / 3840) splits into
// 320-column tiles without padding, and M = 8192 gives exactly one full round (256 tiles on 256 CUs) where 256x192
// gives 224.  A 128x320 tile is 0.625 of a 256x256 one in work.  VST_P8_320 = 1 takes it wherever its round count
// times 0.7 beats the 256 / 192 choice; VST_P8_BN = 320 wherever it is legal (A/B).
static bool p8_320_on() {
  static const int on = [] {
    const char* e = getenv("VST_P8_320");
    return e ? atoi(e) : 0;
  }();
  return on != 0;
}

static bool p8_bn320(int M, int N, bool geglu) {
  const int env = p8_forced_bn();
  if (geglu || N % 320) return false;
  if (env == 320) return true;
  if (!p8_320_on() || env == 256 || env == 192) return false;
  const int cus = device_cus();
  const int mb = (M + 255) / 256;
  const int r256 = (mb * ((N + 255) / 256) + cus - 1) / cus, r192 = (mb * ((N + 191) / 192) + cus - 1) / cus;
  const int r320 = (((M + 127) / 128) * (N / 320) + cus - 1) / cus;
  const double best = p8_bn192(M, N, false) ? 0.8 * r192 : r256;
  return 0.7 * r320 < 0.97 * best;
}

static int g_p8_conv = -1;  // VST_P8_CONV, or vst_p8_conv (tests, A/B)
static bool p8_conv_env() {
  if (g_p8_conv < 0) {
    const char* e = getenv("VST_P8_CONV");
    g_p8_conv = e ? atoi(e) : 1;
  }
  return g_p8_conv != 0;
}

static int p8_bn(int M, int N, bool geglu) {
  return p8_bn320(M, N, geglu) ? 320 : p8_bn192(M, N, geglu) ? 192 : 256;
}


// Convs whose Cout is a multiple of 128 (not of 320) on which the 8-phase policy would take 192-wide tiles -- the VAE's
// Cout = 128 convs at 512^2 (a third of every 192-wide tile padding) and its Cout = 512 convs at 64^2 (256x128 tiles fill
// exactly one round of 256 CUs) -- run on the ring kernel's 256x128 tiles: same k order, same bits, 10-12 % faster
// per launch (tools/vae_conv_ab.py, profiles/r6_vae_conv_ab.txt).  No UNet conv qualifies (Cout 320 / 640 / 1280 / 4).
static bool conv_ring128(int M, int N) { return N % 128 == 0 && N % 320 != 0 && p8_bn(M, N, false) == 192; }

}  // namespace vst

// Force the 8-phase kernel's tile width for every later GEMM of this process (256 / 192 / 320 where legal; 0 = the
// automatic policy); returns the previous setting.  For tests and A/B runs.
extern "C" int vst_p8_force_bn(int bn) {
  const int prev = vst::p8_forced_bn();
  vst::g_p8_force_bn = (bn == 256 || bn == 192 || bn == 320) ? bn : 0;
  return prev;
}

// Route 3x3 convs with 64-multiple channel sources to the 8-phase kernel (1) or the ring kernel (0) for every later
// conv of this process; returns the previous setting.  For tests and A/B runs.
extern "C" int vst_p8_conv(int on) {
  const int prev = vst::p8_conv_env() ? 1 : 0;
  vst::g_p8_conv = on ? 1 : 0;
  return prev;
}

namespace vst {

// tile code 8: AMODE 0, no split-K, a 64-aligned A source split, 256x256 tiles
static bool p8_applies(int M, int N, int K1, bool two_src) {
  (void)M; (void)N;
  return !two_src || (K1 & 63) == 0;
}
// Workspace (caller-owned): the fp32 split-K slabs [splits][M][N].

static int device_cus() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = kCUs;
  }
  return n;
}

// Stream-K (one workgroup per CU over equal shares of the (tile, k-step) space, partial tiles summed by their
// owner) was built for both the ring and the 8-phase kernel in rounds 1-3 and measured slower on every shape of this
// path (8192x1280x1312: 8.56 -> 11.1 ms per step).  Its cross-workgroup hand-off also depended on
// every workgroup being resident at once, which concurrent streams do not guarantee, so it was removed.

static int gemm_ablate_env() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("VST_GEMM_ABLATE");
    v = e ? atoi(e) : 0;
  }
  return v;
}

static int gemm_group_env() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("VST_GEMM_GROUP_M");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// Persistent launch: measured (tools/gemm_persist.sh) 4-10 % faster for the GEGLU epilogue and neutral for
// the others, so it is the default for GEGLU only.  VST_GEMM_PERSIST=1 forces it on, =0 off.
static int gemm_persist_env() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("VST_GEMM_PERSIST");
    v = e ? atoi(e) : -1;
  }
  return v;
}

static int run_gemm(GemmArgs& a, int amode, int geglu, int tile, int splits, hipStream_t s) {
  a.ablate = gemm_ablate_env();
  a.group_m = gemm_group_env();
  const int pe = gemm_persist_env();
  a.persist = (pe > 0 || (pe < 0 && geglu)) ? device_cus() : 0;
  if (tile == 5) return launch_skinny(a, s);
  if (tile == 8) {
    if (amode != 0 || splits > 1) return VST_ERR_ARG;
    a.splits = 1;
    return launch_gemm_p8(a, geglu ? 1 : (a.act ? 3 : 0), a.p8_bn == 192 || a.p8_bn == 320 ? a.p8_bn : 256, s);
  }
  if (amode == 2) {  // scalar-gather conv (conv_in): register-staged kernel, no split
    a.splits = 1;
    return launch_one<2, 0, 64>(a, s, 1);
  }
  a.splits = splits;
  if (splits > 1) {
    const int rc = launch_gemm_ring(a, amode, 2, tile, splits, s);
    if (rc) return rc;
    const int Nout = geglu ? a.N / 2 : a.N;
    const size_t chunks = (size_t)a.M * ((Nout + 7) / 8);
    const int grid = (int)std::min<size_t>((chunks + 255) / 256, 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, a, geglu);
    return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
  }
  return launch_gemm_ring(a, amode, geglu ? 1 : (a.act ? 3 : 0), tile, 1, s);
}

}  // namespace vst

using namespace vst;

extern "C" size_t vst_gemm_workspace_bytes(int M, int N, int K) {
  int tile = 0, splits = 0;
  choose(M, N, K, 0, 0, (size_t)-1, tile, splits);
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

// ---- fused base + LoRA projection with the down-projection inside the 8-phase GEMM (gemm_p8.hip LORA) ----
// VST_LORA_INGEMM=0 turns it off (the host then runs the separate down-projection pass, A/B).
static bool lora_ingemm_env() {
  static const int v = [] {
    const char* e = getenv("VST_LORA_INGEMM");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}

// 0 = not supported (the host falls back to u = x.Acat^T + vst_gemm_ex), else the 8-phase tile width (256 / 192 /
// 320).  Every tile's output columns must need u columns inside one 16-aligned block of 16.  Whether the in-GEMM
// path is taken depends on the SHAPE only (N, K, the projection groups), never on M: it runs whenever some tile width
// keeps every tile inside one u block (the policy's width first, then 192, 256, 320 -- every SDXL width is a multiple
// of 320, so the 32x32 q/k/v, which straddles q/k on 256-wide tiles, runs on 128x320 tiles).  So a frame-sharded rank
// (fewer rows) takes the same path as the unsharded forward, and the two agree bit for bit: the tile width itself
// does not change any output bit (same k order).
static bool lora_tiles_ok(int N, int P, int gn, int gr, int bn) {
  for (int n0 = 0; n0 < N; n0 += bn) {
    const int g0 = n0 / gn, g1 = (std::min(n0 + bn, N) - 1) / gn;
    const int lo = (g0 * gr) & ~15, hi = (g1 + 1) * gr;
    if (hi > lo + 16 || lo + 16 > P) return false;
  }
  return true;
}

static int lora_ingemm_bn(int M, int N, int K, int P, int gn, int gr, int force_bn = 0) {
  if (!lora_ingemm_env() || M <= 0 || N <= 0 || K < 128 || (K & 7) || P <= 0 || (P & 15) || P > 256 || gn <= 0 ||
      gr <= 0 || N % gn || (N / gn) * gr > P)
    return 0;
  if (force_bn) return lora_tiles_ok(N, P, gn, gr, force_bn) && (force_bn != 320 || N % 320 == 0) ? force_bn : 0;
  const int cand[4] = {p8_bn(M, N, false), 192, 256, 320};
  int bn = 0;
  for (int c : cand)
    if ((c != 320 || N % 320 == 0) && lora_tiles_ok(N, P, gn, gr, c)) {
      bn = c;
      break;
    }
  // a multi-round grid of 256-row tiles (the 32x32 out-projection) moves to the persistent LoRA grid, which runs
  // 128x320 tiles only (gemm_p8.hip, p8_lora_persist_env); a grid under two rounds keeps its tiles (the 16x16 q/k/v:
  // 480 tiles of 256x256, 76 us against 89 on 128x320 persistent, profiles/r5_ab_lora_persist.txt)
  if (bn && bn != 320 && p8_lora_persist_on() && N % 320 == 0 && lora_tiles_ok(N, P, gn, gr, 320) &&
      (long)((M + 255) / 256) * ((N + bn - 1) / bn) >= 2L * device_cus() && p8_persist_applies(M, N, K, 0, 320))
    bn = 320;
  return bn;
}

extern "C" int vst_gemm_lora_supported(int M, int N, int K, int P, int group_n, int group_r) {
  return lora_ingemm_bn(M, N, K, P, group_n, group_r);
}

extern "C" int vst_gemm_lora(const void* x, int ldx, const void* Acat, int ld_acat, int P, int group_n, int group_r,
                             const void* W, int ldw, int M, int N, int K, const float* bias, const void* R, int ldr,
                             void* C, int ldc, void* stream) {
  Fit31 fit;
  if (!x || !Acat || !W || !C || M <= 0 || N <= 0 || K <= 0) return VST_ERR_ARG;
  if ((ldx & 7) || (ld_acat & 7) || (ldw & 7) || (ldc & 7) || ldx < K || ld_acat < K || ldw < K + P) return VST_ERR_ARG;
  if (R && ((ldr & 7) || ldr < N)) return VST_ERR_ARG;
  const int bn = lora_ingemm_bn(M, N, K, P, group_n, group_r);
  if (!bn) return VST_ERR_UNSUPPORTED;
  GemmArgs a{};
  a.A1 = (const bf16_t*)x; a.A2 = nullptr; a.lda1 = ldx; a.lda2 = 0; a.K1 = K;
  a.Wt = (const bf16_t*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.bias = bias; a.R = (const bf16_t*)R; a.ldr = ldr; a.C = (bf16_t*)C; a.ldc = ldc;
  a.a1_bytes = fit(((size_t)(M - 1) * ldx + K) * 2);
  a.w_bytes = fit(((size_t)(N - 1) * ldw + K) * 2);
  a.wtail_bytes = fit(((size_t)(N - 1) * ldw + K + P) * 2);
  a.r_bytes = R ? fit(((size_t)(M - 1) * ldr + N) * 2) : 0;
  a.la = (const bf16_t*)Acat; a.lda_la = ld_acat; a.la_p = P; a.la_gn = group_n; a.la_gr = group_r;
  a.la_bytes = fit((size_t)P * ld_acat * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets (not chunked here): refuse
  a.stride = 1; a.splits = 1;
  a.p8_bn = bn;
  a.ablate = gemm_ablate_env();  // (reaches the kernel in the diagnostics build only, -DVST_P8_TRACE)
  a.group_m = gemm_group_env();
  return launch_gemm_p8_lora(a, bn, (hipStream_t)stream);
}

// ---- attn2: q projection (+ in-GEMM LoRA) with the cross-attention over the text tokens as its epilogue ----
// VST_XATTN_FUSE=0 turns it off (the host then runs the q GEMM and vst_spatial_attention, A/B).
static bool xattn_env() {
  static const int v = [] {
    const char* e = getenv("VST_XATTN_FUSE");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}

// Shape-only decision (not M: a frame-sharded rank fuses exactly where the unsharded forward does).
static bool xattn_ok(int M, int N, int K, const void* Acat, int P, int gn, int gr, int Nq, int Nk) {
  if (!xattn_env() || M <= 0 || N <= 0 || N % 64 || K < 128 || (K & 7) || Nq <= 0 || Nq % 256 || M % Nq || Nk < 1 ||
      Nk > 80)
    return false;
  return !Acat || lora_ingemm_bn(M, N, K, P, gn, gr, 192) == 192;
}

extern "C" int vst_gemm_cross_attention_supported(int M, int N, int K, int lora, int P, int group_n, int group_r,
                                                  int Nq, int Nk) {
  return xattn_ok(M, N, K, lora ? (const void*)1 : nullptr, P, group_n, group_r, Nq, Nk) ? 1 : 0;
}

extern "C" int vst_gemm_cross_attention(const void* x, int ldx, const void* Acat, int ld_acat, int P, int group_n,
                                        int group_r, const void* W, int ldw, const float* bias, int M, int N, int K,
                                        const void* Kt, const void* Vt, int ldkv, int nkv_rows, int Nq, int Nk,
                                        int kv_div, float scale, void* O, int ldo, void* stream) {
  Fit31 fit;
  if (!x || !W || !Kt || !Vt || !O || M <= 0 || N <= 0 || K <= 0 || kv_div <= 0 || nkv_rows <= 0) return VST_ERR_ARG;
  if ((ldx & 7) || (ldw & 7) || (ldo & 7) || (ldkv & 7) || ldx < K || ldo < N || ldkv < N) return VST_ERR_ARG;
  if (Acat && ((ld_acat & 7) || ld_acat < K || ldw < K + P)) return VST_ERR_ARG;
  if (!Acat && ldw < K) return VST_ERR_ARG;
  if (!xattn_ok(M, N, K, Acat, P, group_n, group_r, Nq, Nk)) return VST_ERR_UNSUPPORTED;
  if ((M / Nq - 1) / kv_div >= nkv_rows / Nk) return VST_ERR_ARG;  // every frame's text batch inside K/V
  GemmArgs a{};
  a.A1 = (const bf16_t*)x; a.lda1 = ldx; a.K1 = K;
  a.Wt = (const bf16_t*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.bias = bias; a.C = (bf16_t*)O; a.ldc = ldo;
  a.a1_bytes = fit(((size_t)(M - 1) * ldx + K) * 2);
  a.w_bytes = fit(((size_t)(N - 1) * ldw + K) * 2);
  if (Acat) {
    a.wtail_bytes = fit(((size_t)(N - 1) * ldw + K + P) * 2);
    a.la = (const bf16_t*)Acat; a.lda_la = ld_acat; a.la_p = P; a.la_gn = group_n; a.la_gr = group_r;
    a.la_bytes = fit((size_t)P * ld_acat * 2);
  }
  a.xa_k = (const bf16_t*)Kt; a.xa_v = (const bf16_t*)Vt; a.xa_ldkv = ldkv; a.xa_nk = Nk; a.xa_nq = Nq;
  a.xa_kvdiv = kv_div; a.xa_scale_log2 = scale * 1.4426950408889634f;
  a.xa_kv_bytes = fit(((size_t)(nkv_rows - 1) * ldkv + N) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets (not chunked here): refuse
  a.stride = 1; a.splits = 1; a.p8_bn = 192;
  a.ablate = gemm_ablate_env();  // (diagnostics build only)
  return launch_gemm_p8_xattn(a, (hipStream_t)stream);
}

// The motion modules' q/k/v projection + frame-axis attention in one launch (EPI 5 of the 8-phase kernel): 16 frames
// per clip, heads of 40 (two per 256-column tile: an even head count) or 80 (one per tile), pixels per frame a
// multiple of 16.
static int tattn_hpt(int head_dim) { return head_dim == 40 ? 2 : head_dim == 80 ? 1 : 0; }
static bool tattn_ok(int M, int K, int nclip, int F, int HW, int heads, int head_dim) {
  const int hpt = tattn_hpt(head_dim);
  if (!hpt || F != 16 || heads <= 0 || heads % hpt || HW <= 0 || (HW & 15) || nclip <= 0) return false;
  // (shape-only, like the other fused paths: a frame-sharded rank decides as the unsharded forward does)
  return (long)M == (long)nclip * F * HW && !(K & 63) && K >= 128 && gemm_p8_env() != 0;
}

extern "C" int vst_gemm_temporal_attention_supported(int M, int K, int nclip, int F, int HW, int heads,
                                                     int head_dim) {
  return tattn_ok(M, K, nclip, F, HW, heads, head_dim) ? 1 : 0;
}

extern "C" int vst_gemm_temporal_attention(const void* x, int ldx, const void* Wt, int ldw, const float* bias, int M,
                                           int K, int nclip, int F, int HW, int heads, int head_dim, float scale,
                                           void* O, int ldo, void* stream) {
  Fit31 fit;
  if (!x || !Wt || !O || M <= 0 || K <= 0) return VST_ERR_ARG;
  if ((ldx & 7) || (ldw & 7) || (ldo & 7) || ldx < K || ldw < K || ldo < heads * head_dim) return VST_ERR_ARG;
  if (!tattn_ok(M, K, nclip, F, HW, heads, head_dim)) return VST_ERR_UNSUPPORTED;
  const int N = heads / tattn_hpt(head_dim) * 256;
  GemmArgs a{};
  a.A1 = (const bf16_t*)x; a.lda1 = ldx; a.K1 = K;
  a.Wt = (const bf16_t*)Wt; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.bias = bias; a.C = (bf16_t*)O; a.ldc = ldo;
  a.a1_bytes = fit(((size_t)(M - 1) * ldx + K) * 2);
  a.w_bytes = fit(((size_t)(N - 1) * ldw + K) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets (not chunked here): refuse
  a.ta_hw = HW; a.ta_heads = heads; a.ta_d = head_dim; a.ta_scale_log2 = scale * 1.4426950408889634f;
  a.stride = 1; a.splits = 1; a.p8_bn = 256;
  return launch_gemm_p8_tattn(a, (hipStream_t)stream);
}

// Name of the kernel a vst_gemm_ex / vst_conv3x3_ex call with these arguments launches (the
// symbol rocprofv3 reports), so per-launch timings can be attributed to kernels.  kind: 0 linear,
// 1 GEGLU linear, 2 vectorized conv, 3 scalar-gather conv.  Returns a static string.
extern "C" const char* vst_gemm_kernel_name(int M, int N, int K, int kind, int tile, int splits, size_t ws_bytes) {
  static const char* names[7][3] = {
      {"gemm_ring<128x128>", "gemm_ring<128x128,geglu>", "gemm_ring<128x128,conv>"},
      {"gemm_ring<128x64>", "gemm_ring<128x64,geglu>", "gemm_ring<128x64,conv>"},
      {"gemm_ring<256x256>", "gemm_ring<256x256,geglu>", "gemm_ring<256x256,conv>"},
      {"gemm_ring<256x128>", "gemm_ring<256x128,geglu>", "gemm_ring<256x128,conv>"},
      {"", "", ""},
      {"gemm_ring<256x160>", "", "gemm_ring<256x160,conv>"},
      {"gemm_ring<192x256>", "gemm_ring<192x256,geglu>", "gemm_ring<192x256,conv>"}};
  static const char* split_names[7] = {"gemm_ring<128x128,splitk>", "gemm_ring<128x64,splitk>",
                                       "gemm_ring<256x256,splitk>", "gemm_ring<256x128,splitk>", "",
                                       "gemm_ring<256x160,splitk>", "gemm_ring<192x256,splitk>"};
  if (kind == 3) return "gemm_kernel<conv_in>";
  if (kind == 2 && tile == 0 && splits <= 1 && p8_conv_env() && K % 576 == 0 && N % 64 == 0 &&
      p8_auto(M, N, K, false)) {
    if (conv_ring128(M, N)) return "gemm_ring<256x128,conv>";
    const int bn = N % 320 == 0 ? 320 : p8_bn(M, N, false) == 192 ? 192 : 256;
    return bn == 320 ? "gemm_p8<128x320,conv>" : bn == 192 ? "gemm_p8<256x192,conv>" : "gemm_p8<256x256,conv>";
  }
  if (kind == 0 && tile == 0 && rows_applies(M, N, K)) return "gemm_rows";
  if (kind == 0 && (tile == 5 || (tile == 0 && N <= 64 && M >= 1024))) return "gemm_skinny";  // no-epilogue calls
  if (kind < 0 || kind > 3 || tile < 0 || tile > 10 || tile == 5 || splits < 0) return "";
  // the 8-phase kernel, persistent where p8_persist_applies (kind 0 is reported with its plain epilogue)
  auto p8name = [&](int bn, bool geglu) -> const char* {
    const bool pe = p8_persist_applies(M, N, K, geglu ? 1 : 0, bn);
    if (bn == 320) return pe ? "gemm_p8<128x320,persist>" : "gemm_p8<128x320>";
    if (bn == 192) return pe ? "gemm_p8<256x192,persist>" : "gemm_p8<256x192>";
    if (geglu) return pe ? "gemm_p8<256x256,geglu,persist>" : "gemm_p8<256x256,geglu>";
    return pe ? "gemm_p8<256x256,persist>" : "gemm_p8<256x256>";
  };
  if (tile == 9) return kind == 0 ? p8name(192, false) : "";
  if (tile == 10) return kind == 0 ? p8name(320, false) : "";
  if (tile == 0 && kind <= 1 && p8_auto(M, N, K, kind == 1)) {
    if (splits <= 1 && kind == 0 && p8_bn(M, N, false) == 320) return p8name(320, false);
    if (splits <= 1 && kind == 0 && p8_bn192(M, N, false)) return p8name(192, false);
    tile = 8;
  }
  choose(M, N, K, kind == 1, kind == 2, ws_bytes, tile, splits);
  if (tile == 8) return p8name(256, kind == 1);
  if (splits > 1) return split_names[tile - 1];
  return names[tile - 1][kind == 2 ? 2 : kind];
}

// The kernels address A, A2 and the residual through buffer descriptors with 32-bit byte offsets (Fit31): an
// operand whose byte extent passes 2^31 - 1 would read zeros past that point.  Such a call (e.g. the motion modules'
// ff.net.2 at the 64^2 level of an 8-clip CFG batch, A = 1M x 1280 bf16 = 2.7 GB) runs as equal row chunks with
// offset pointers instead.  The kernels' per-row k order does not depend on M, and chunks this large take the same
// kernels (no split-K), so every row gets the bits of one launch (test_kernels_gpu.py::test_gemm_rows_past_2gb).
static size_t row_extent(size_t rows, int ld, int cols) { return ((rows - 1) * (size_t)ld + (size_t)cols) * 2; }
static int row_chunk(int M, size_t row_bytes, int align) {  // balanced rows per chunk (a multiple of align), 0: none
  const size_t lim = 0x7fffffffULL;
  const size_t fit = (lim / row_bytes) / (size_t)align * (size_t)align;
  if (fit == 0) return 0;
  const size_t n = ((size_t)M + fit - 1) / fit;
  const size_t rows = (((size_t)M + n - 1) / n + align - 1) / align * align;
  return rows <= fit ? (int)rows : (int)fit;
}
static int gcd_int(int a, int b) { return b ? gcd_int(b, a % b) : a; }

extern "C" int vst_gemm_ex(const void* A, int lda, const void* A2, int lda2, int K1, const void* W, int ldw, int M,
                           int N, int K, const float* bias, const float* row_bias, int row_bias_div, int ld_row_bias,
                           const void* R, int ldr, void* C, int ldc, int epilogue, int tile, int splits,
                           void* workspace, size_t ws_bytes, void* stream) {
  Fit31 fit;
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0) return VST_ERR_ARG;
  if ((K & 7) || (lda & 7) || (ldw & 7) || (ldc & 7)) return VST_ERR_ARG;
  if (A2) {
    if (K1 <= 0 || K1 % BK || K1 >= K || (lda2 & 7)) return VST_ERR_ARG;
  } else {
    K1 = K;
  }
  if (epilogue < 0 || epilogue > 2) return VST_ERR_ARG;
  if (epilogue == 1 && (N % 64)) return VST_ERR_ARG;
  if (epilogue == 2 && (R || row_bias)) return VST_ERR_ARG;  // GELU: bias only
  if (R && (ldr & 7)) return VST_ERR_ARG;
  if (row_bias && row_bias_div <= 0) return VST_ERR_ARG;
  {
    const int nout = epilogue == 1 ? N / 2 : N;
    const size_t lim = 0x7fffffffULL;
    if (row_extent(M, lda, K1) > lim || (A2 && row_extent(M, lda2, K - K1) > lim) ||
        (R && row_extent(M, ldr, nout) > lim) || row_extent(M, ldc, nout) > lim) {
      const int wide = max(max(lda, A2 ? lda2 : 0), max(R ? ldr : 0, ldc));
      const int align = row_bias ? 256 / gcd_int(256, row_bias_div) * row_bias_div : 256;
      const int rows = align > 0 ? row_chunk(M, (size_t)wide * 2, align) : 0;
      if (rows <= 0) return VST_ERR_ARG;
      const int ldrb = ld_row_bias ? ld_row_bias : N;
      for (int m0 = 0; m0 < M; m0 += rows) {
        const int mc = min(rows, M - m0);
        const int st = vst_gemm_ex(
            (const char*)A + (size_t)m0 * lda * 2, lda, A2 ? (const char*)A2 + (size_t)m0 * lda2 * 2 : nullptr, lda2,
            A2 ? K1 : 0, W, ldw, mc, N, K, bias, row_bias ? row_bias + (size_t)(m0 / row_bias_div) * ldrb : nullptr,
            row_bias_div, ld_row_bias, R ? (const char*)R + (size_t)m0 * ldr * 2 : nullptr, ldr,
            (char*)C + (size_t)m0 * ldc * 2, ldc, epilogue, tile, splits, workspace, ws_bytes, stream);
        if (st != VST_OK) return st;
      }
      return VST_OK;
    }
  }
  if (tile < 0 || tile > 10 || splits < 0) return VST_ERR_ARG;
  if ((tile == 8 || tile == 9 || tile == 10) && !p8_applies(M, N, K1, A2 != nullptr)) return VST_ERR_ARG;
  if ((tile == 9 || tile == 10) && epilogue == 1) return VST_ERR_ARG;  // GEGLU needs the 256-wide tiles
  if (tile == 10 && N % 320) return VST_ERR_ARG;
  const bool skinny_ok = N <= 64 && !A2 && !bias && !row_bias && !R && epilogue == 0;
  if (tile == 5 && !skinny_ok) return VST_ERR_ARG;
  GemmArgs a{};
  a.A1 = (const bf16_t*)A; a.A2 = (const bf16_t*)A2; a.lda1 = lda; a.lda2 = lda2; a.K1 = K1;
  a.Wt = (const bf16_t*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.bias = bias; a.rbias = row_bias; a.rbias_div = row_bias_div; a.ldrb = ld_row_bias;
  a.R = (const bf16_t*)R; a.ldr = ldr; a.C = (bf16_t*)C; a.ldc = ldc;
  a.ws = (float*)workspace;
  a.a1_bytes = fit(((size_t)(M - 1) * lda + K1) * 2);
  a.a2_bytes = A2 ? fit(((size_t)(M - 1) * lda2 + (K - K1)) * 2) : 0;
  a.w_bytes = fit(((size_t)(N - 1) * ldw + K) * 2);
  a.r_bytes = R ? fit(((size_t)(M - 1) * ldr + N) * 2) : 0;
  if (fit.over) return VST_ERR_ARG;  // (A / R / C are chunked above; a weight past 2^31 - 1 bytes is refused)
  a.C1 = 0; a.C2 = 0; a.stride = 1; a.up = 0;
  a.act = epilogue == 2 ? 1 : 0;
  if (epilogue == 2) epilogue = 0;
  if (tile == 0 && !A2 && epilogue != 1 && rows_applies(M, N, K)) return launch_rows(a, (hipStream_t)stream);
  if (tile == 0 && skinny_ok && M >= 1024) tile = 5;  // LoRA down-projection: skinny kernel
  if (tile == 5) return run_gemm(a, 0, 0, 5, 1, (hipStream_t)stream);
  const size_t slab_bytes = workspace ? ws_bytes : 0;
  // splits 1 = no split-K (a row's bits then never depend on M: the denoise forward's row-invariant policy); the
  // 8-phase kernel, which never splits, is chosen the same way under 0 and 1
  if (tile == 0 && splits <= 1 && p8_auto(M, N, K, epilogue == 1) && p8_applies(M, N, K1, A2 != nullptr))
    tile = p8_bn(M, N, epilogue == 1) == 320 ? 10 : p8_bn192(M, N, epilogue == 1) ? 9 : 8;
  if (tile == 9 || tile == 10) {  // the 8-phase kernel at 256x192 / 128x320
    a.p8_bn = tile == 9 ? 192 : 320;
    return run_gemm(a, 0, 0, 8, 1, (hipStream_t)stream);
  }
  choose(M, N, K, epilogue == 1, 0, slab_bytes, tile, splits);
  return run_gemm(a, 0, epilogue == 1, tile, splits, (hipStream_t)stream);
}

extern "C" int vst_gemm(const void* A, int lda, const void* A2, int lda2, int K1, const void* W, int ldw, int M, int N,
                        int K, const float* bias, const float* row_bias, int row_bias_div, int ld_row_bias,
                        const void* R, int ldr, void* C, int ldc, int epilogue, void* stream) {
  return vst_gemm_ex(A, lda, A2, lda2, K1, W, ldw, M, N, K, bias, row_bias, row_bias_div, ld_row_bias, R, ldr, C, ldc,
                     epilogue, 0, 1, nullptr, 0, stream);
}

// 3x3 conv, padding 1, NHWC.  x1: [nimg,H,W,C1], optional x2: [nimg,H,W,C2] concatenated
// on channels.  Wt: [Cout][3][3][C1+C2].  stride 1 or 2; upsample=1 applies nearest 2x to
// the input first (output 2H x 2W).  Output [nimg, OH, OW, Cout] with row stride ldc.

static int conv3x3_impl(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride,
                        int upsample, int pad0, const void* Wt, int Cout, const float* bias, const float* row_bias,
                        int row_bias_div, int ld_row_bias, const void* R, int ldr, void* out, int ldc, int tile,
                        int splits, void* workspace, size_t ws_bytes, void* stream, float* colstat = nullptr) {
  Fit31 fit;
  if (!x1 || !Wt || !out || nimg <= 0 || H <= 0 || W <= 0 || Cout <= 0) return VST_ERR_ARG;
  if (pad0 && (stride != 2 || H < 2 || W < 2)) return VST_ERR_ARG;
  if (stride != 1 && stride != 2) return VST_ERR_ARG;
  if (upsample && stride != 1) return VST_ERR_ARG;
  if (tile < 0 || tile > 7 || tile == 5 || splits < 0) return VST_ERR_ARG;
  const int Ct = C1 + (x2 ? C2 : 0);
  const bool vec = (Ct % BK == 0) && (C1 % 8 == 0);
  if (x2 && !vec) return VST_ERR_ARG;
  GemmArgs a{};
  a.OH = upsample ? 2 * H : pad0 ? (H - 2) / 2 + 1 : (stride == 2 ? (H + 1) / 2 : H);
  a.OW = upsample ? 2 * W : pad0 ? (W - 2) / 2 + 1 : (stride == 2 ? (W + 1) / 2 : W);
  {  // byte extents past the 32-bit buffer offsets (vst_gemm_ex): chunks of whole images (a 3x3 tap never leaves its
     // image), equal in size
    const size_t lim = 0x7fffffffULL, hw = (size_t)H * W, ohw = (size_t)a.OH * a.OW;
    const size_t img_bytes = max(max(hw * C1, x2 ? hw * C2 : 0), max(R ? ohw * ldr : 0, ohw * ldc)) * 2;
    if ((size_t)nimg * img_bytes > lim) {
      if (colstat || (row_bias && row_bias_div != (int)ohw)) return VST_ERR_UNSUPPORTED;
      const int per = (int)(lim / img_bytes);
      if (per <= 0) return VST_ERR_ARG;
      const int nch = (nimg + per - 1) / per, ipc = (nimg + nch - 1) / nch;
      const int ldrb = ld_row_bias ? ld_row_bias : Cout;
      for (int i0 = 0; i0 < nimg; i0 += ipc) {
        const int ni = min(ipc, nimg - i0);
        const int st = conv3x3_impl(
            (const char*)x1 + (size_t)i0 * hw * C1 * 2, C1, x2 ? (const char*)x2 + (size_t)i0 * hw * C2 * 2 : nullptr,
            C2, ni, H, W, stride, upsample, pad0, Wt, Cout, bias, row_bias ? row_bias + (size_t)i0 * ldrb : nullptr,
            row_bias_div, ld_row_bias, R ? (const char*)R + (size_t)i0 * ohw * ldr * 2 : nullptr, ldr,
            (char*)out + (size_t)i0 * ohw * ldc * 2, ldc, tile, splits, workspace, ws_bytes, stream);
        if (st != VST_OK) return st;
      }
      return VST_OK;
    }
  }
  a.pad0 = pad0;
  a.A1 = (const bf16_t*)x1; a.A2 = (const bf16_t*)x2; a.C1 = C1; a.C2 = x2 ? C2 : 0;
  a.H = H; a.W = W; a.stride = stride; a.up = upsample;
  a.K = 9 * Ct; a.K1 = a.K;
  a.M = nimg * a.OH * a.OW; a.N = Cout;
  if (!vec) a.K = (a.K + 7) & ~7;  // scalar gather: pad K to a chunk; weight rows padded too
  a.Wt = (const bf16_t*)Wt; a.ldw = a.K;
  if (row_bias && (row_bias_div <= 0 || (ld_row_bias && ld_row_bias < Cout) || ((ld_row_bias ? ld_row_bias : Cout) & 3)))
    return VST_ERR_ARG;
  a.bias = bias; a.rbias = row_bias; a.rbias_div = row_bias_div; a.ldrb = ld_row_bias ? ld_row_bias : Cout;
  a.R = (const bf16_t*)R; a.ldr = ldr; a.C = (bf16_t*)out; a.ldc = ldc;
  a.ws = (float*)workspace;
  a.a1_bytes = fit((size_t)nimg * H * W * C1 * 2);
  a.a2_bytes = x2 ? fit((size_t)nimg * H * W * C2 * 2) : 0;
  a.w_bytes = fit((size_t)Cout * a.K * 2);
  a.r_bytes = R ? fit(((size_t)(a.M - 1) * ldr + Cout) * 2) : 0;
  if (fit.over) return VST_ERR_ARG;  // (A / R / C are chunked above; a weight past 2^31 - 1 bytes is refused)
  if ((ldc & 7) && Cout >= 8) return VST_ERR_ARG;
  if (!vec) { tile = 2; splits = 1; }
  // 3x3 convs with both sources a multiple of 64 channels run on the 8-phase kernel (implicit im2col; 128x320 tiles
  // where Cout is a multiple of 320, else the projection policy's width); VST_P8_CONV=0 restores the ring kernel
  bool p8 = vec && tile == 0 && splits <= 1 && p8_conv_env() && !(C1 & 63) && !((x2 ? C2 : 0) & 63) &&
            !(a.N & 63) && p8_auto(a.M, a.N, a.K, false);
  if (p8 && !colstat && conv_ring128(a.M, a.N)) {
    p8 = false;
    tile = 4;
    splits = 1;
  }
  if (colstat) {  // column statistics come from the 128x320 tiles' epilogue only
    if (!p8 || a.N % 320) return VST_ERR_UNSUPPORTED;
    a.colstat = colstat;
  }
  if (p8) {
    a.splits = 1;
    a.ablate = 0;
    a.group_m = gemm_group_env();
    return launch_gemm_p8_conv(a, a.N % 320 == 0 ? 320 : p8_bn(a.M, a.N, false), (hipStream_t)stream);
  }
  const size_t slab_bytes = workspace ? ws_bytes : 0;
  choose(a.M, a.N, a.K, 0, 1, slab_bytes, tile, splits);
  return run_gemm(a, vec ? 1 : 2, 0, tile, splits, (hipStream_t)stream);
}

extern "C" int vst_conv3x3_ex(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride,
                              int upsample, const void* Wt, int Cout, const float* bias, const float* row_bias,
                              int row_bias_div, int ld_row_bias, const void* R, int ldr, void* out, int ldc, int tile,
                              int splits, void* workspace, size_t ws_bytes, void* stream) {
  return conv3x3_impl(x1, C1, x2, C2, nimg, H, W, stride, upsample, 0, Wt, Cout, bias, row_bias, row_bias_div,
                      ld_row_bias, R, ldr, out, ldc, tile, splits, workspace, ws_bytes, stream);
}

// vst_conv3x3_ex + the GroupNorm column statistics of the output for a following vst_groupnorm_colstat:
// colstat [ceil(M / 128)][Cout][2] fp32 = (sum, sum of squares) over each 128-row output tile of the stored bf16
// values.  VST_ERR_UNSUPPORTED (nothing launched) unless the conv runs on the 8-phase kernel's 128x320 tiles
// (Cout % 320 == 0, both sources multiples of 64 channels, default policy).
extern "C" int vst_conv3x3_colstat(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride,
                                   int upsample, const void* Wt, int Cout, const float* bias, const float* row_bias,
                                   int row_bias_div, int ld_row_bias, const void* R, int ldr, void* out, int ldc,
                                   float* colstat, void* stream) {
  if (!colstat) return VST_ERR_ARG;
  return conv3x3_impl(x1, C1, x2, C2, nimg, H, W, stride, upsample, 0, Wt, Cout, bias, row_bias, row_bias_div,
                      ld_row_bias, R, ldr, out, ldc, 0, 1, nullptr, 0, stream, colstat);
}

// 3x3 stride-2 conv with padding (0,1,0,1): diffusers Downsample2D(padding=0) = F.pad(x, (0, 1, 0, 1)) + conv(k3, s2,
// p0), the downsampler of the SDXL VAE encoder's DownEncoderBlock2D.  Output [nimg, (H-2)/2+1, (W-2)/2+1, Cout].
extern "C" int vst_conv3x3_down_pad0(const void* x, int C, int nimg, int H, int W, const void* Wt, int Cout,
                                     const float* bias, void* out, int ldc, void* workspace, size_t ws_bytes,
                                     void* stream) {
  return conv3x3_impl(x, C, nullptr, 0, nimg, H, W, 2, 0, 1, Wt, Cout, bias, nullptr, 1, 0, nullptr, 0, out, ldc, 0,
                      0, workspace, ws_bytes, stream);
}

// C[M][N] (fp32, row stride N) = A[M][K] . W[N][K]^T with no rounding of the accumulator: the ring kernel's split-K slab
// epilogue with one split.  For attention scores whose softmax must see fp32 logits (the SDXL VAE mid-block attention,
// head_dim 512, fp32 in the reference: inference_animatediff.py:164-169).
extern "C" int vst_gemm_f32out(const void* A, int lda, const void* W, int ldw, int M, int N, int K, float* C,
                               void* stream) {
  Fit31 fit;
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0) return VST_ERR_ARG;
  if ((K & 7) || (lda & 7) || (ldw & 7) || (N & 3)) return VST_ERR_ARG;
  GemmArgs a{};
  a.A1 = (const bf16_t*)A; a.lda1 = lda; a.lda2 = lda; a.K1 = K;
  a.Wt = (const bf16_t*)W; a.ldw = ldw; a.M = M; a.N = N; a.K = K;
  a.C = nullptr; a.ldc = N; a.ws = C; a.splits = 1; a.stride = 1;
  a.a1_bytes = fit(((size_t)(M - 1) * lda + K) * 2);
  a.w_bytes = fit(((size_t)(N - 1) * ldw + K) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets (not chunked here): refuse
  int tile = 0, splits = 1;
  choose(M, N, K, 0, 0, 0, tile, splits);
  if (tile == 8) tile = 3;
  a.ablate = gemm_ablate_env();
  a.group_m = gemm_group_env();
  return launch_gemm_ring(a, 0, 2, tile, 1, (hipStream_t)stream);
}

extern "C" int vst_conv3x3(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride,
                           int upsample, const void* Wt, int Cout, const float* bias, const float* row_bias,
                           int row_bias_div, const void* R, int ldr, void* out, int ldc, void* stream) {
  return vst_conv3x3_ex(x1, C1, x2, C2, nimg, H, W, stride, upsample, Wt, Cout, bias, row_bias, row_bias_div, 0, R,
                        ldr, out, ldc, 0, 1, nullptr, 0, stream);
}
