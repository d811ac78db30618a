// Token-contracted GEMM for the training step's weight gradients: C[N][K] = A^T B with A [M][N] and B [M][K] both
// row-major over M tokens (dW = g^T x of every trainable linear, dA = s v^T x and dB = s g^T u of the temporal
// LoRA, dW of the GEGLU projection; autograd.py, the reference's backward of train_animatediff.py:265-319).
//
// Why a kernel of its own: the projection GEMMs contract over their row-major K, so a weight gradient through them
// needed both operands transposed to [N][M] / [K][M] first (two vst_transpose launches per gradient, 420 per
// training step) and then ran a split-K GEMM over the token axis.  Here the tokens ARE the contraction axis: a stage
// of 64 tokens x 128 columns of each operand is staged in LDS as it lies in memory ([token][column] sub-tiles of
// 64 x 64, the V-tile swizzle of the attention kernels), and both MFMA operands are read transposed with
// ds_read_b64_tr_b16 (the O^T = V^T P^T read of spatial attention), so no transposed copy is ever written.
//
// Workgroup: 4 waves (2 x 2) over a 128 (n) x 128 (k) output tile, wave tile 64 x 64 = 4 x 4 accumulators of
// 16 x 16; one 32-KiB LDS stage (the next stage waits in registers), so three workgroups share a CU (3-10 % faster
// per shape than two double-buffered ones, profiles/r6_gemm_tn.txt); the token range splits over `splits`
// workgroups per tile so the grid fills the chip (the weight grids are
// 3 x 3 .. 80 x 10 tiles against 20k-260k tokens).  splits == 1 writes bf16 directly; otherwise each split writes
// its fp32 partial tile and gemm_tn_reduce_kernel sums the splits in index order (deterministic bits).
#include "attn_common.h"

namespace vst {

constexpr int TN_T = 64;                 // tokens per stage
constexpr int TN_SUB = TN_T * 64 * 2;    // one [64 tokens][64 columns] bf16 sub-tile: 8 KiB
constexpr int TN_STAGE = 4 * TN_SUB;     // A: columns n0 .. n0+127 (2 sub-tiles), B: k0 .. k0+127 (2)
constexpr int TN_LDS = TN_STAGE;         // one stage (the next one waits in registers): 32 KiB, three workgroups per CU

__global__ __launch_bounds__(256, 3) void gemm_tn_kernel(const bf16_t* __restrict__ A, int lda,
                                                         const bf16_t* __restrict__ B, int ldb, int M, int N, int K,
                                                         int tokens_per_split, uint32_t a_bytes, uint32_t b_bytes,
                                                         bf16_t* __restrict__ C, int ldc, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wk = wid & 1;
  const int ntn = (N + 127) / 128, ntk = (K + 127) / 128;
  const int tile = blockIdx.x % (ntn * ntk), split = blockIdx.x / (ntn * ntk);
  const int n0 = (tile / ntk) * 128, k0 = (tile % ntk) * 128;
  const int m_begin = split * tokens_per_split;
  const int m_end = min(M, m_begin + tokens_per_split);
  const int nstage = (m_end - m_begin + TN_T - 1) / TN_T;
  const auto ra = make_rsrc(A, a_bytes), rb = make_rsrc(B, b_bytes);

  // loader: sub-tile s (0, 1: A columns n0 + 64 s; 2, 3: B columns k0 + 64 (s - 2)), rows sr and sr + 32, 16-B chunk sc
  const int sc = tid & 7, sr = tid >> 3;
  u32x4 reg[4][2];
  auto load = [&](int t) {
    const int m0 = m_begin + t * TN_T;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int col = (s < 2 ? n0 + 64 * s : k0 + 64 * (s - 2)) + sc * 8;
      const bool cok = col < (s < 2 ? N : K);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m0 + sr + 32 * i;
        const bool ok = cok && m < m_end;
        if (s < 2) reg[s][i] = buf_load16(ra, ok ? (m * lda + col) * 2 : kOOB);
        else reg[s][i] = buf_load16(rb, ok ? (m * ldb + col) * 2 : kOOB);
      }
    }
  };
  auto store = [&](int buf) {
    char* base = smem + buf * TN_STAGE;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<u32x4*>(base + s * TN_SUB + v_off(sr + 32 * i, sc)) = reg[s][i];
  };

  // transposed fragment reads (spatial attention's V^T pattern): column block cb (16 columns) x token half st
  const int fr = lane & 15, g = lane >> 4;
  int toff[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int r0 = g * 4 + (fr >> 2), col = cb * 16 + (fr & 3) * 4;
    toff[cb] = v_off(r0, col >> 3) + (col & 7) * 2;
  }
  f32x4 acc[4][4];  // [k block][n block]: lane holds C[n = .. + fr][k = .. + 4 g + e]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nstage > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < nstage; ++t) {
    const int cur = 0;
    if (t + 1 < nstage) load(t + 1);
    const char* As = smem + cur * TN_STAGE + wn * TN_SUB;
    const char* Bs = smem + cur * TN_STAGE + (2 + wk) * TN_SUB;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const char* pa = As + toff[cb] + st * 4096;
        const char* pb = Bs + toff[cb] + st * 4096;
        fa[cb] = cat_tr(ds_read_tr(pa), ds_read_tr(pa + 2048));
        fb[cb] = cat_tr(ds_read_tr(pb), ds_read_tr(pb + 2048));
      }
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[kb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kb], fa[nb], acc[kb][nb], 0, 0, 0);
    }
    __syncthreads();  // every wave's reads of the stage done
    if (t + 1 < nstage) {
      store(0);
      __syncthreads();
    }
  }

#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = n0 + wn * 64 + nb * 16 + fr;
    if (n >= N) continue;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int k = k0 + wk * 64 + kb * 16 + 4 * g;
      if (k >= K) continue;  // (K % 8 == 0: a 4-column group is wholly in or out)
      const f32x4 v = acc[kb][nb];
      if (ws) {
        *reinterpret_cast<f32x4*>(ws + ((size_t)split * N + n) * K + k) = v;
      } else {
        *reinterpret_cast<u32x2*>(C + (size_t)n * ldc + k) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    }
  }
}

// C[n][k] = bf16(sum over splits s = 0, 1, ... of ws[s][n][k]), 4 columns per thread
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(const float* __restrict__ ws, int splits, int N, int K,
                                                             bf16_t* __restrict__ C, int ldc) {
  const size_t q = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t nq = (size_t)N * K / 4;
  if (q >= nq) return;
  const size_t e = q * 4;
  const int n = (int)(e / K), k = (int)(e % K);
  f32x4 s = *reinterpret_cast<const f32x4*>(ws + e);
  for (int i = 1; i < splits; ++i) s += *reinterpret_cast<const f32x4*>(ws + (size_t)i * N * K + e);
  *reinterpret_cast<u32x2*>(C + (size_t)n * ldc + k) = u32x2{pack2bf(s[0], s[1]), pack2bf(s[2], s[3])};
}

static int tn_splits(int M, int N, int K) {
  const int tiles = ((N + 127) / 128) * ((K + 127) / 128);
  const int want = (768 + tiles - 1) / tiles;             // about three workgroups per CU
  const int most = max(1, (M + 2047) / 2048);             // at least 2048 tokens per split
  return max(1, min(want, most));
}

}  // namespace vst

using namespace vst;

extern "C" size_t vst_gemm_tn_workspace_bytes(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int s = tn_splits(M, N, K);
  return s > 1 ? (size_t)s * N * K * sizeof(float) : 0;
}

extern "C" int vst_gemm_tn(const void* A, int lda, const void* B, int ldb, int M, int N, int K, void* C, int ldc,
                           void* workspace, size_t ws_bytes, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0) return VST_ERR_ARG;
  if ((N & 7) || (K & 7) || (lda & 7) || (ldb & 7) || (ldc & 3) || lda < N || ldb < K || ldc < K) return VST_ERR_ARG;
  Fit31 fit;
  const uint32_t ab = fit(((size_t)(M - 1) * lda + N) * 2);
  const uint32_t bb = fit(((size_t)(M - 1) * ldb + K) * 2);
  if (fit.over) return VST_ERR_ARG;  // past the 32-bit buffer offsets: refuse (the caller splits the tokens)
  const int splits = tn_splits(M, N, K);
  const size_t need = splits > 1 ? (size_t)splits * N * K * sizeof(float) : 0;
  if (need && (!workspace || ws_bytes < need)) return VST_ERR_ARG;
  int tps = (M + splits - 1) / splits;
  tps = (tps + TN_T - 1) / TN_T * TN_T;
  const int tiles = ((N + 127) / 128) * ((K + 127) / 128);
  hipStream_t s = (hipStream_t)stream;
  static const bool attr = hipFuncSetAttribute((const void*)gemm_tn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               TN_LDS) == hipSuccess;
  if (!attr) return VST_ERR_LAUNCH;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3(tiles * splits), dim3(256), TN_LDS, s, (const bf16_t*)A, lda,
                     (const bf16_t*)B, ldb, M, N, K, tps, ab, bb, (bf16_t*)C, ldc,
                     splits > 1 ? (float*)workspace : (float*)nullptr);
  if (splits > 1) {
    const size_t nq = (size_t)N * K / 4;
    hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s,
                       (const float*)workspace, splits, N, K, (bf16_t*)C, ldc);
  }
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}
