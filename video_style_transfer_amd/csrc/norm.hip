// Normalisations on NHWC / token-major activations ([rows, C], C contiguous).
//
// GroupNorm (32 groups) as used by the denoise path:
//   * ResnetBlock2D norm1/norm2 (eps 1e-5, + SiLU), per frame;
//   * Transformer2DModel.norm (eps 1e-6), per frame (unziplora_unet/transformer_2d.py:222-235);
//   * motion-module norm (eps 1e-6) over the 5-D (B,C,F,H,W) tensor, i.e. statistics span
//     every frame of a clip (diffusers AnimateDiffTransformer3D);
//   * conv_norm_out (eps 1e-5, + SiLU).
// A "sample" is `rows_per_sample` consecutive rows (H*W for per-frame, F*H*W per clip).
// Three launches: partial (sum, sumsq) per (sample, chunk, group) -> merge to (mean, rstd)
// with Chan's parallel-variance combine -> apply (+optional SiLU), bf16 out.  The input may
// be two channel-concatenated sources (up-block skip concat), so the concat is never
// materialised for the normalised branch.
//
// LayerNorm over C per row (BasicTransformerBlock norm1/2/3, eps 1e-5), optionally adding the
// sinusoidal frame position table pe[(row / pe_div) % pe_mod] after the affine transform
// (motion-module blocks add the PE to the normed input before attn1 and attn2).
#include "vst_common.h"

namespace vst {

// Launch geometry shared by the stats and apply passes: grid (nchunk, nsamples), each workgroup owns
// `rpc` consecutive rows of one sample and has rps x CH threads (CH = C/8 16-B channel chunks per row,
// rps = 512 / CH rows in flight per step), so no lane idles whatever C is, and `rpc` is chosen by the
// host so that every launch has >= ~256 workgroups (the 16x16-latent GroupNorms have only 256 rows
// per frame: one 256-row chunk per sample gave 32 workgroups and 0.7 TB/s).
__host__ __device__ inline int gn_rps(int C) { return max(1, 512 / (C / 8)); }

// x1: [rows, C1] (ld1), x2: [rows, C2] (ld2): base pointer / stride of the source holding channel c
__device__ __forceinline__ void gn_src(const bf16_t* x1, int ld1, int C1, const bf16_t* x2, int ld2, int c,
                                       const bf16_t*& base, int& ld) {
  if (c < C1) { base = x1 + c; ld = ld1; }
  else { base = x2 + (c - C1); ld = ld2; }
}

__global__ __launch_bounds__(512) void gn_stats_kernel(const bf16_t* __restrict__ x1, int ld1, int C1,
                                                       const bf16_t* __restrict__ x2, int ld2, int C2,
                                                       int rows_per_sample, int rpc, int groups,
                                                       float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float gsm[];  // [rps][C] sums then sumsqs
  const int C = C1 + C2;
  const int CH = C / 8;
  const int rps = blockDim.x / CH;
  const int s = blockIdx.y, chunk = blockIdx.x;
  const int nchunk = gridDim.x;
  const int r_beg = chunk * rpc;
  const int r_end = min(rows_per_sample, r_beg + rpc);
  const int tid = threadIdx.x;
  const int cch = tid % CH, rph = tid / CH, c = cch * 8;
  const bf16_t* base;
  int ld;
  gn_src(x1, ld1, C1, x2, ld2, c, base, ld);
  base += (size_t)s * rows_per_sample * ld;
  float a[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { a[e] = 0.f; q[e] = 0.f; }
  // GN_UNROLL independent 16-B loads in flight per thread
#ifndef VST_GN_STATS_U
#define VST_GN_STATS_U 8
#endif
  constexpr int GN_UNROLL = VST_GN_STATS_U;
  for (int r = r_beg + rph; r < r_end; r += GN_UNROLL * rps) {
    u32x4 v[GN_UNROLL];
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) {
      const int rr = r + u * rps;
      v[u] = rr < r_end ? *reinterpret_cast<const u32x4*>(base + (size_t)rr * ld) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += f[e]; q[e] += f[e] * f[e]; }
    }
  }
  float* ssum = gsm;
  float* ssq = gsm + rps * C;
#pragma unroll
  for (int e = 0; e < 8; ++e) { ssum[rph * C + c + e] = a[e]; ssq[rph * C + c + e] = q[e]; }
  __syncthreads();
  // fold the row phases column-parallel into row 0, then one wave per group sums its Cg columns by
  // shuffles (a serial per-group loop over rps x Cg LDS reads was ~10 us of latency per workgroup)
  for (int cc = tid; cc < C; cc += blockDim.x) {
    float sa = ssum[cc], sq = ssq[cc];
    for (int rr = 1; rr < rps; ++rr) { sa += ssum[rr * C + cc]; sq += ssq[rr * C + cc]; }
    ssum[cc] = sa;
    ssq[cc] = sq;
  }
  __syncthreads();
  const int Cg = C / groups;
  const int lane = tid & 63, wave = tid >> 6, nwave = blockDim.x >> 6;  // full waves only
  for (int gi = wave; wave < nwave && gi < groups; gi += nwave) {
    float sa = 0.f, sq = 0.f;
    for (int cc = lane; cc < Cg; cc += 64) { sa += ssum[gi * Cg + cc]; sq += ssq[gi * Cg + cc]; }
    sa = wave_sum(sa);
    sq = wave_sum(sq);
    if (lane == 0) {
      float* o = part + (((size_t)s * nchunk + chunk) * groups + gi) * 2;
      o[0] = sa;
      o[1] = sq;
    }
  }
}

// one 64-thread block per (sample, group): merge the chunk partials (sum, sumsq) in double, then
// emit the per-channel affine  y = x * scale[s,c] + shift[s,c]  (scale = rstd*gamma,
// shift = beta - mean*rstd*gamma) so the apply pass is one FMA per element.
__global__ __launch_bounds__(64) void gn_finalize_kernel(const float* __restrict__ part, int nchunk,
                                                         int rows_per_sample, int groups, int Cg, float eps,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ scale,
                                                         float* __restrict__ shift, int C,
                                                         float* __restrict__ stats = nullptr) {
  const int s = blockIdx.x / groups, gi = blockIdx.x - s * groups;
  const int lane = threadIdx.x;
  double a = 0.0, q = 0.0;
  for (int c = lane; c < nchunk; c += 64) {
    const float* p = part + (((size_t)s * nchunk + c) * groups + gi) * 2;
    a += p[0];
    q += p[1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    q += __shfl_xor(q, o);
  }
  const double n = (double)rows_per_sample * Cg;
  const double mean = a / n;
  const double var = fmax(q / n - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int c = gi * Cg + lane; c < (gi + 1) * Cg; c += 64) {
    const float sc = rstd * gamma[c];
    scale[(size_t)s * C + c] = sc;
    shift[(size_t)s * C + c] = beta[c] - (float)mean * sc;
  }
  if (stats != nullptr && lane == 0) {  // backward: (mean, rstd) per (sample, group)
    stats[(size_t)blockIdx.x * 2] = (float)mean;
    stats[(size_t)blockIdx.x * 2 + 1] = rstd;
  }
}

// Column statistics of a bf16 tensor x [M, C] in the arithmetic of the 128x320 conv tiles' epilogue
// (gemm_epilogue.h, p.colstat): per 128-row chunk and channel, 12 row groups (rows g, g + 12, ...) summed in row order
// (sum += x, sumsq = fma(x, x, sumsq) in fp32), then the 12 groups added in order -- so a GroupNorm gets the same
// statistics bits whether its input's producer wrote them or this kernel did.  Workgroup: 128 rows x 320 channels.
__global__ __launch_bounds__(512) void gn_colstat_kernel(const bf16_t* __restrict__ x, int ldx, int M, int C,
                                                         float* __restrict__ cs) {
  constexpr int CPR = 40, RG = 12, RPT = 11;
  __shared__ f32x2 part[RG][320];
  const int tid = threadIdx.x, cc = tid % CPR, rg = tid / CPR;
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 320, n = n0 + cc * 8;
  float a[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = q[e] = 0.f;
  if (rg < RG && n < C) {
    u32x4 v[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int row = rg + RG * j, m = m0 + row;
      v[j] = row < 128 && m < M ? *reinterpret_cast<const u32x4*>(x + (size_t)m * ldx + n) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int row = rg + RG * j;
      if (row >= 128 || m0 + row >= M) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(v[j][e] << 16), hi = __uint_as_float(v[j][e] & 0xffff0000u);
        a[2 * e] += lo;
        q[2 * e] = fmaf(lo, lo, q[2 * e]);
        a[2 * e + 1] += hi;
        q[2 * e + 1] = fmaf(hi, hi, q[2 * e + 1]);
      }
    }
  }
  if (rg < RG) {
#pragma unroll
    for (int e = 0; e < 8; ++e) part[rg][cc * 8 + e] = f32x2{a[e], q[e]};
  }
  __syncthreads();
  if (tid < 320 && n0 + tid < C) {
    f32x2 t = part[0][tid];
#pragma unroll
    for (int g = 1; g < RG; ++g) t += part[g][tid];
    *reinterpret_cast<f32x2*>(cs + ((size_t)blockIdx.x * C + n0 + tid) * 2) = t;
  }
}

// GroupNorm statistics from the producing conv's column statistics (vst_conv3x3_colstat: per 128-row output tile and
// channel, the sum and sum of squares of the stored bf16 values), so the GroupNorm's own statistics pass over x
// disappears.  One 64-thread block per (sample, group) merges the sample's nchunk tiles x Cg channels in double,
// in a fixed order (lane-strided, then the xor butterfly), and emits the same per-channel affine as
// gn_finalize_kernel.  x2 (the channel concat of an up block): channels >= C1 read cs2.
__global__ __launch_bounds__(64) void gn_finalize_colstat_kernel(const float* __restrict__ cs1, int C1,
                                                                 const float* __restrict__ cs2, int C2, int nchunk,
                                                                 int rows_per_sample, int groups, int Cg, float eps,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 float* __restrict__ scale, float* __restrict__ shift) {
  const int s = blockIdx.x / groups, gi = blockIdx.x - s * groups;
  const int lane = threadIdx.x;
  const int C = C1 + C2;
  double a = 0.0, q = 0.0;
  for (int e = lane; e < nchunk * Cg; e += 64) {
    const int ck = e / Cg, c = gi * Cg + e - ck * Cg;
    const int row = s * nchunk + ck;
    const float* p = c < C1 ? cs1 + ((size_t)row * C1 + c) * 2 : cs2 + ((size_t)row * C2 + c - C1) * 2;
    a += p[0];
    q += p[1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    q += __shfl_xor(q, o);
  }
  const double n = (double)rows_per_sample * Cg;
  const double mean = a / n;
  const double var = fmax(q / n - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int c = gi * Cg + lane; c < (gi + 1) * Cg; c += 64) {
    const float sc = rstd * gamma[c];
    scale[(size_t)s * C + c] = sc;
    shift[(size_t)s * C + c] = beta[c] - (float)mean * sc;
  }
}

// ---- GroupNorm backward (training path) ----
// z = x * scale + shift (the forward's affine, recomputed), dz = g (or g * silu'(z) with the fused SiLU).
// Pass 1 (gn_bwd_sums): per (sample, chunk) and channel, sum dz and dz * x (same geometry as gn_stats).
// Pass 2 (gn_bwd_finalize): per (sample, group), A = mean(gamma dz), B = mean(gamma dz x^) ->
//   dx = a_c dz + b0 + b1 x  with a_c = rstd gamma_c, b0 = rstd^2 mean B - rstd A, b1 = -rstd^2 B,
//   and the per-(sample, channel) sums for dgamma / dbeta.  Pass 3 (gn_bwd_apply) writes dx; gn_bwd_param sums
//   dgamma_c = sum_s rstd (S_dzx - mean S_dz), dbeta_c = sum_s S_dz in a fixed order.
__device__ __forceinline__ float silu_grad(float z) {
  const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * 1.4426950408889634f));
  return sg * (1.0f + z * (1.0f - sg));
}

__global__ __launch_bounds__(512) void gn_bwd_sums_kernel(const bf16_t* __restrict__ x, int ldx,
                                                          const bf16_t* __restrict__ g, int ldg, int C,
                                                          int rows_per_sample, int rpc, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int act,
                                                          float* __restrict__ part2) {
  extern __shared__ __attribute__((aligned(16))) float bsm[];  // [rps][C] sum dz, then [rps][C] sum dz*x
  const int CH = C / 8;
  const int rps = blockDim.x / CH;
  const int s = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int r_beg = chunk * rpc, r_end = min(rows_per_sample, r_beg + rpc);
  const int tid = threadIdx.x, cch = tid % CH, rph = tid / CH, c = cch * 8;
  const size_t row0 = (size_t)s * rows_per_sample;
  float sc[8], sh[8], a[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[(size_t)s * C + c + e];
    sh[e] = shift[(size_t)s * C + c + e];
    a[e] = 0.f;
    q[e] = 0.f;
  }
  for (int r = r_beg + rph; r < r_end; r += rps) {
    float xv[8], gv[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + (row0 + r) * ldx + c), xv);
    unpack8(*reinterpret_cast<const u32x4*>(g + (row0 + r) * ldg + c), gv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dz = act ? gv[e] * silu_grad(xv[e] * sc[e] + sh[e]) : gv[e];
      a[e] += dz;
      q[e] += dz * xv[e];
    }
  }
  float* s1 = bsm;
  float* s2 = bsm + rps * C;
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[rph * C + c + e] = a[e]; s2[rph * C + c + e] = q[e]; }
  __syncthreads();
  for (int cc = tid; cc < C; cc += blockDim.x) {
    float u = 0.f, v = 0.f;
    for (int rr = 0; rr < rps; ++rr) { u += s1[rr * C + cc]; v += s2[rr * C + cc]; }
    part2[(((size_t)s * nchunk + chunk) * 2) * C + cc] = u;
    part2[(((size_t)s * nchunk + chunk) * 2 + 1) * C + cc] = v;
  }
}

__global__ __launch_bounds__(64) void gn_bwd_finalize_kernel(const float* __restrict__ part2, int nchunk, int C,
                                                             int groups, int rows_per_sample,
                                                             const float* __restrict__ stats,
                                                             const float* __restrict__ gamma,
                                                             float* __restrict__ chsum, float* __restrict__ coef) {
  const int s = blockIdx.x / groups, gi = blockIdx.x - s * groups;
  const int lane = threadIdx.x;
  const int Cg = C / groups;
  const float mean = stats[(size_t)blockIdx.x * 2], rstd = stats[(size_t)blockIdx.x * 2 + 1];
  double A = 0.0, Bq = 0.0;
  for (int c = gi * Cg + lane; c < (gi + 1) * Cg; c += 64) {
    double sdz = 0.0, sdzx = 0.0;
    for (int ch = 0; ch < nchunk; ++ch) {
      sdz += part2[(((size_t)s * nchunk + ch) * 2) * C + c];
      sdzx += part2[(((size_t)s * nchunk + ch) * 2 + 1) * C + c];
    }
    chsum[((size_t)s * 2) * C + c] = (float)sdz;
    chsum[((size_t)s * 2 + 1) * C + c] = (float)(rstd * (sdzx - (double)mean * sdz));  // sum dz * x^
    A += gamma[c] * sdz;
    Bq += gamma[c] * (sdzx - (double)mean * sdz);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    A += __shfl_xor(A, o);
    Bq += __shfl_xor(Bq, o);
  }
  const double n = (double)rows_per_sample * Cg;
  const double Am = A / n, Bm = (double)rstd * Bq / n;
  const float b0 = (float)((double)rstd * rstd * mean * Bm - (double)rstd * Am);
  const float b1 = (float)(-(double)rstd * rstd * Bm);
  for (int c = gi * Cg + lane; c < (gi + 1) * Cg; c += 64) {
    coef[((size_t)s * C + c) * 3] = rstd * gamma[c];
    coef[((size_t)s * C + c) * 3 + 1] = b0;
    coef[((size_t)s * C + c) * 3 + 2] = b1;
  }
}

__global__ __launch_bounds__(512) void gn_bwd_apply_kernel(const bf16_t* __restrict__ x, int ldx,
                                                           const bf16_t* __restrict__ g, int ldg, int C,
                                                           int rows_per_sample, int rpc,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int act,
                                                           const float* __restrict__ coef, bf16_t* __restrict__ dx,
                                                           int lddx) {
  const int CH = C / 8;
  const int rps = blockDim.x / CH;
  const int s = blockIdx.y;
  const int r_beg = blockIdx.x * rpc, r_end = min(rows_per_sample, r_beg + rpc);
  const int tid = threadIdx.x, cch = tid % CH, rph = tid / CH, c = cch * 8;
  const size_t row0 = (size_t)s * rows_per_sample;
  float sc[8], sh[8], ca[8], c0[8], c1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[(size_t)s * C + c + e];
    sh[e] = shift[(size_t)s * C + c + e];
    ca[e] = coef[((size_t)s * C + c + e) * 3];
    c0[e] = coef[((size_t)s * C + c + e) * 3 + 1];
    c1[e] = coef[((size_t)s * C + c + e) * 3 + 2];
  }
  for (int r = r_beg + rph; r < r_end; r += rps) {
    float xv[8], gv[8], o[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + (row0 + r) * ldx + c), xv);
    unpack8(*reinterpret_cast<const u32x4*>(g + (row0 + r) * ldg + c), gv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dz = act ? gv[e] * silu_grad(xv[e] * sc[e] + sh[e]) : gv[e];
      o[e] = ca[e] * dz + c0[e] + c1[e] * xv[e];
    }
    *reinterpret_cast<u32x4*>(dx + (row0 + r) * lddx + c) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void gn_bwd_param_kernel(const float* __restrict__ chsum, int nsamples, int C,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float db = 0.f, dg = 0.f;
  for (int s = 0; s < nsamples; ++s) {
    db += chsum[((size_t)s * 2) * C + c];
    dg += chsum[((size_t)s * 2 + 1) * C + c];
  }
  dgamma[c] = dg;
  dbeta[c] = db;
}

__global__ __launch_bounds__(512) void gn_apply_kernel(const bf16_t* __restrict__ x1, int ld1, int C1,
                                                       const bf16_t* __restrict__ x2, int ld2, int C2,
                                                       int rows_per_sample, int rpc, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int act,
                                                       bf16_t* __restrict__ y, int ldy) {
  const int C = C1 + C2;
  const int CH = C / 8;
  const int rps = blockDim.x / CH;
  const int s = blockIdx.y;
  const int r_beg = blockIdx.x * rpc;
  const int r_end = min(rows_per_sample, r_beg + rpc);
  const int cch = threadIdx.x % CH, rph = threadIdx.x / CH, c = cch * 8;
  const bf16_t* base;
  int ld;
  gn_src(x1, ld1, C1, x2, ld2, c, base, ld);
  const size_t row0 = (size_t)s * rows_per_sample;
  base += row0 * ld;
  bf16_t* yb = y + row0 * ldy + c;
  // this thread's 8 channels of one sample: the affine is loaded once
  const f32x4* sc = reinterpret_cast<const f32x4*>(scale + (size_t)s * C + c);
  const f32x4* sh = reinterpret_cast<const f32x4*>(shift + (size_t)s * C + c);
  const f32x4 a0 = sc[0], a1 = sc[1], b0 = sh[0], b1 = sh[1];
#ifndef VST_GN_APPLY_U
#define VST_GN_APPLY_U 4
#endif
  constexpr int U = VST_GN_APPLY_U;  // loads in flight per thread
  for (int r = r_beg + rph; r < r_end; r += U * rps) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rps;
      v[u] = rr < r_end ? *reinterpret_cast<const u32x4*>(base + (size_t)rr * ld) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + u * rps;
      if (rr >= r_end) break;
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = f[e] * a0[e] + b0[e];
        f[e + 4] = f[e + 4] * a1[e] + b1[e];
      }
      if (act) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = silu(f[e]);
      }
      *reinterpret_cast<u32x4*>(yb + (size_t)rr * ldy) = pack8(f);
    }
  }
}

// Motion-module GroupNorm (statistics over every frame of a clip), frame-sharded or not.  The statistics are
// built from per-FRAME chunk partials (gn_stats_kernel with one sample per frame, chunking that depends only on
// the frame's row count), so a rank holding some frames of a clip produces exactly the partials the unsharded
// forward produces for those frames.  The finalize merges the clip's F x nck partials in one fixed order, read
// from the rank-major layout [P][clips][F/P][nck][G][2] an all-gather leaves (P = 1: the unsharded layout), so the
// sharded and unsharded statistics are the same bits whatever P is.
__global__ __launch_bounds__(64) void gn_finalize_parts_kernel(const float* __restrict__ part, int P, int nclips,
                                                               int Fl, int nck, int groups, int Cg, double count,
                                                               float eps, const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* __restrict__ scale,
                                                               float* __restrict__ shift, int C) {
  const int b = blockIdx.x / groups, gi = blockIdx.x - b * groups;
  const int lane = threadIdx.x;
  const int per_clip = P * Fl * nck;  // partials of one clip, in (global frame, chunk) order
  double a = 0.0, q = 0.0;
  for (int c = lane; c < per_clip; c += 64) {
    const int f = c / nck, k = c - f * nck;
    const int r = f / Fl, fl = f - r * Fl;
    const float* p = part + (((((size_t)r * nclips + b) * Fl + fl) * nck + k) * groups + gi) * 2;
    a += p[0];
    q += p[1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    q += __shfl_xor(q, o);
  }
  const double mean = a / count;
  const double var = fmax(q / count - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int c = gi * Cg + lane; c < (gi + 1) * Cg; c += 64) {
    const float sc = rstd * gamma[c];
    scale[(size_t)b * C + c] = sc;
    shift[(size_t)b * C + c] = beta[c] - (float)mean * sc;
  }
}

// LayerNorm: each wave normalises ROWS rows (all their 16-B loads issued before any reduction, so
// ROWS x MAXCH loads are in flight per lane), up to MAXCH 8-channel chunks per lane and row.
template <int MAXCH, int ROWS>
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16_t* __restrict__ x, int ldx, int C, int rows,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        float eps, const float* __restrict__ pe, int pe_div, int pe_mod,
                                                        bf16_t* __restrict__ y, int ldy) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * ROWS;
  if (row0 >= rows) return;
  const int CH = C / 8;
  float v[ROWS][MAXCH][8];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int row = row0 + r;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int cc = lane + 64 * i;
      u32x4 raw = u32x4{0u, 0u, 0u, 0u};
      if (cc < CH && row < rows) raw = *reinterpret_cast<const u32x4*>(x + (size_t)row * ldx + cc * 8);
      unpack8(raw, v[r][i]);
    }
  }
  float gg[MAXCH][8], bb[MAXCH][8];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int cc = lane + 64 * i;
    if (cc < CH) {
      const f32x4* g4 = reinterpret_cast<const f32x4*>(gamma + cc * 8);
      const f32x4* b4 = reinterpret_cast<const f32x4*>(beta + cc * 8);
      const f32x4 g0 = g4[0], g1 = g4[1], b0 = b4[0], b1 = b4[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) { gg[i][e] = g0[e]; gg[i][e + 4] = g1[e]; bb[i][e] = b0[e]; bb[i][e + 4] = b1[e]; }
    }
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int row = row0 + r;
    if (row >= rows) break;
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[r][i][e];  // zero-filled past C
    const float mean = wave_sum(sum) / C;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      if (lane + 64 * i < CH) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[r][i][e] - mean; sq += d * d; }
      }
    }
    const float rstd = rsqrtf(wave_sum(sq) / C + eps);
    const float* pr = pe ? pe + (size_t)((row / pe_div) % pe_mod) * C : nullptr;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int cc = lane + 64 * i;
      if (cc < CH) {
        float o[8];
        if (pr) {
          const f32x4* p4 = reinterpret_cast<const f32x4*>(pr + cc * 8);
          const f32x4 p0 = p4[0], p1 = p4[1];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = (v[r][i][e] - mean) * (rstd * gg[i][e]) + bb[i][e] + p0[e];
            o[e + 4] = (v[r][i][e + 4] - mean) * (rstd * gg[i][e + 4]) + bb[i][e + 4] + p1[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (v[r][i][e] - mean) * (rstd * gg[i][e]) + bb[i][e];
        }
        *reinterpret_cast<u32x4*>(y + (size_t)row * ldy + cc * 8) = pack8(o);
      }
    }
  }
}

// LayerNorm for C = 40 * LPR (320 / 640 / 1280): LPR lanes per row, each holding CPL = 5 interleaved 16-B chunks
// (lane l of a row reads chunks l, l + LPR, ...: every load instruction covers whole 128-B+ row segments), so all 64
// lanes work for every C (the generic kernel above idles 37 % of its lanes at C = 320) and a wave normalises
// 64 / LPR rows per pass; RIT passes' loads are all issued before the first reduction.  Row statistics are two-pass
// (mean, then squared deviations), reduced over the row's LPR lanes by xor shuffles.
template <int LPR, int RIT>
__global__ __launch_bounds__(256) void layernorm_g_kernel(const bf16_t* __restrict__ x, int ldx, int C, int rows,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          const float* __restrict__ pe, int pe_div, int pe_mod,
                                                          bf16_t* __restrict__ y, int ldy) {
  constexpr int CPL = 5, RPW = 64 / LPR;
  __shared__ f32x4 sgb[2][CPL * LPR * 2];  // gamma, beta of the row (C = 40 LPR floats = 10 LPR f32x4)
  const int lane = threadIdx.x & 63, l = lane % LPR, rsub = lane / LPR;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW * RIT;
  float v[RIT][CPL][8];
#pragma unroll
  for (int it = 0; it < RIT; ++it) {
    const int row = row0 + it * RPW + rsub;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      u32x4 raw = u32x4{0u, 0u, 0u, 0u};
      if (row < rows) raw = *reinterpret_cast<const u32x4*>(x + (size_t)row * ldx + (l + LPR * i) * 8);
      unpack8(raw, v[it][i]);
    }
  }
  // gamma / beta staged once per workgroup (every wave of it used to fetch the whole row's 10 LPR x 32 B through the
  // vector memory path per row pass: 4x the row's own bytes)
  for (int i = threadIdx.x; i < CPL * LPR * 2; i += 256) {
    sgb[0][i] = reinterpret_cast<const f32x4*>(gamma)[i];
    sgb[1][i] = reinterpret_cast<const f32x4*>(beta)[i];
  }
  __syncthreads();
  if (row0 >= rows) return;
  const float invc = 1.0f / (float)C;
#pragma unroll
  for (int it = 0; it < RIT; ++it) {
    const int row = row0 + it * RPW + rsub;
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[it][i][e];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float mean = sum * invc;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[it][i][e] - mean; sq = fmaf(d, d, sq); }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    const float rstd = rsqrtf(fmaf(sq, invc, eps));  // (explicit fmas: codegen-independent rounding)
    if (row >= rows) continue;
    const float* pr = pe ? pe + (size_t)((row / pe_div) % pe_mod) * C : nullptr;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c0 = (l + LPR * i) * 8;
      const f32x4 g0 = sgb[0][c0 / 4], g1 = sgb[0][c0 / 4 + 1];
      const f32x4 b0 = sgb[1][c0 / 4], b1 = sgb[1][c0 / 4 + 1];
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = fmaf(v[it][i][e] - mean, rstd * g0[e], b0[e]);
        o[e + 4] = fmaf(v[it][i][e + 4] - mean, rstd * g1[e], b1[e]);
      }
      if (pr) {
        const f32x4 p0 = *reinterpret_cast<const f32x4*>(pr + c0), p1 = *reinterpret_cast<const f32x4*>(pr + c0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] += p0[e]; o[e + 4] += p1[e]; }
      }
      *reinterpret_cast<u32x4*>(y + (size_t)row * ldy + c0) = pack8(o);
    }
  }
}

// LayerNorm fused with the UnZipLoRA down-projection of the projections that consume its output
// (BasicTransformerBlock norm1 -> attn1 q/k/v, norm2 -> attn2 q): y = LN(x) (bf16, as the reference's
// LayerNorm output) and u = y . Acat^T (Acat: [R, C] bf16, R <= 64 a multiple of 16), reading x once.
// A workgroup = 8 waves owns 32 rows; wave w holds the k32-chunks w, w+8, ... of both 16-row
// fragments in registers in the 16x16x32 MFMA operand layout (lane l: row l&15, 8 channels at
// chunk*32 + 8*(l>>4)).  Row statistics are two-pass (mean, then sum of squared deviations) reduced
// over the 4 lanes of a row by shuffles and over the 8 waves through LDS; the normalised bf16 values
// are stored (16 B per lane) and fed straight to the MFMAs; the 8 partial u tiles are summed via LDS.
template <int NJ, int MAXT>
__global__ __launch_bounds__(512, 2) void layernorm_lora_kernel(const bf16_t* __restrict__ x, int ldx, int C, int rows,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps,
                                                                const bf16_t* __restrict__ A, int R,
                                                                bf16_t* __restrict__ y, int ldy, bf16_t* __restrict__ u,
                                                                int ldu) {
#ifndef VST_LNL_MI
#define VST_LNL_MI 2
#endif
  constexpr int MI = VST_LNL_MI, NW = 8;  // MAXT = ceil(C / 256) k32-chunks per wave (C <= 256 * MAXT)
  __shared__ f32x4 red[NW][MI][NJ][64];
  __shared__ float st[NW][MI][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kc = (lane >> 4) * 8;
  const int m0 = blockIdx.x * 16 * MI;
  const int nk = C / 32;
  const auto rx = make_rsrc(x, (uint32_t)min<size_t>(((size_t)(rows - 1) * ldx + C) * 2, 0x7fffffffULL));
  u32x4 raw[MAXT][MI];  // x kept packed (bf16) in registers; unpacked per pass
  bool rowok[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) rowok[i] = m0 + 16 * i + r < rows;
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int ks = w + NW * t;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int off = (ks < nk && rowok[i]) ? ((m0 + 16 * i + r) * ldx + ks * 32 + kc) * 2 : kOOB;
      raw[t][i] = buf_load16(rx, off);
    }
  }
  // ---- mean ----
  float s[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    s[i] = 0.f;
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      float v[8];
      unpack8(raw[t][i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[i] += v[e];  // zero-filled beyond C
    }
    s[i] += __shfl_xor(s[i], 16);
    s[i] += __shfl_xor(s[i], 32);
    if (lane < 16) st[w][i][lane] = s[i];
  }
  __syncthreads();
  float mean[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) a += st[q][i][r];
    mean[i] = a / C;
  }
  __syncthreads();
  // ---- variance (deviations from the mean, only over real channels) ----
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    float q2 = 0.f;
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      if (w + NW * t < nk) {
        float v[8];
        unpack8(raw[t][i], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[e] - mean[i]; q2 += d * d; }
      }
    }
    q2 += __shfl_xor(q2, 16);
    q2 += __shfl_xor(q2, 32);
    if (lane < 16) st[w][i][lane] = q2;
  }
  __syncthreads();
  float rstd[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) a += st[q][i][r];
    rstd[i] = rsqrtf(a / C + eps);
  }
  // ---- normalise, store y, u partials on MFMA ----
  const auto ra = make_rsrc(A, (uint32_t)((size_t)R * C * 2));
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int ks = w + NW * t;
    if (ks >= nk) break;  // wave-uniform
    const int c = ks * 32 + kc;
    const f32x4* g4 = reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4* b4 = reinterpret_cast<const f32x4*>(beta + c);
    const f32x4 g0 = g4[0], g1 = g4[1], b0 = b4[0], b1 = b4[1];
    u32x4 wf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) wf[j] = buf_load16(ra, (16 * j + r) < R ? ((16 * j + r) * C + c) * 2 : kOOB);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v[8], o[8];
      unpack8(raw[t][i], v);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = (v[e] - mean[i]) * (rstd[i] * g0[e]) + b0[e];
        o[e + 4] = (v[e + 4] - mean[i]) * (rstd[i] * g1[e]) + b1[e];
      }
      const u32x4 pk = pack8(o);
      if (rowok[i]) *reinterpret_cast<u32x4*>(y + (size_t)(m0 + 16 * i + r) * ldy + c) = pk;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&wf[j]),
                                                            *reinterpret_cast<const bf16x8*>(&pk), acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) red[w][i][j][lane] = acc[i][j];
  __syncthreads();
  if (w >= MI) return;
  const int i = w;
  const int m = m0 + 16 * i + r;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    f32x4 sum = red[0][i][j][lane];
#pragma unroll
    for (int q = 1; q < NW; ++q) sum += red[q][i][j][lane];
    const int n = 16 * j + 4 * (lane >> 4);  // sum[e] = u[m][n + e]
    if (m < rows && n < R) {
      u32x2 pv;
      pv[0] = pack2bf(sum[0], sum[1]);
      pv[1] = pack2bf(sum[2], sum[3]);
      *reinterpret_cast<u32x2*>(u + (size_t)m * ldu + n) = pv;
    }
  }
}


// LayerNorm backward (training path): one wave per row, grid-stride over rows.
//   x^ = (x - mean) * rstd (recomputed, two-pass), gg = g * gamma,
//   dx = rstd * (gg - mean(gg) - x^ * mean(gg * x^)),  dgamma += g * x^,  dbeta += g.
// The per-channel sums are kept per lane, folded over the 4 waves in LDS and written as one [2][C] partial per
// workgroup; layernorm_bwd_reduce_kernel sums the partials in a fixed order (deterministic).
template <int MAXCH>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const bf16_t* __restrict__ x, int ldx,
                                                            const bf16_t* __restrict__ g, int ldg, int C, int rows,
                                                            const float* __restrict__ gamma, float eps,
                                                            bf16_t* __restrict__ dx, int lddx, float* __restrict__ part) {
  __shared__ float red[4][2][MAXCH * 512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int CH = C / 8;
  float gm[MAXCH][8], dg[MAXCH][8], db[MAXCH][8];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int cc = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) { gm[i][e] = cc < CH ? gamma[cc * 8 + e] : 0.f; dg[i][e] = 0.f; db[i][e] = 0.f; }
  }
  for (int row = blockIdx.x * 4 + w; row < rows; row += gridDim.x * 4) {
    float xv[MAXCH][8], gv[MAXCH][8];
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int cc = lane + 64 * i;
      u32x4 rx = u32x4{0u, 0u, 0u, 0u}, rg = u32x4{0u, 0u, 0u, 0u};
      if (cc < CH) {
        rx = *reinterpret_cast<const u32x4*>(x + (size_t)row * ldx + cc * 8);
        rg = *reinterpret_cast<const u32x4*>(g + (size_t)row * ldg + cc * 8);
      }
      unpack8(rx, xv[i]);
      unpack8(rg, gv[i]);
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += xv[i][e];
    const float mean = wave_sum(sum) / C;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i)
      if (lane + 64 * i < CH) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = xv[i][e] - mean; sq += d * d; }
      }
    const float rstd = rsqrtf(wave_sum(sq) / C + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (xv[i][e] - mean) * rstd;
        const float gg = gv[i][e] * gm[i][e];
        xv[i][e] = xh;
        s1 += gg;
        s2 += gg * xh;
        dg[i][e] += gv[i][e] * xh;
        db[i][e] += gv[i][e];
      }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int cc = lane + 64 * i;
      if (cc < CH) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rstd * (gv[i][e] * gm[i][e] - s1 - xv[i][e] * s2);
        *reinterpret_cast<u32x4*>(dx + (size_t)row * lddx + cc * 8) = pack8(o);
      }
    }
  }
  if (!part) return;  // frozen LayerNorm (spatial path): no dgamma / dbeta
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int cc = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[w][0][cc * 8 + e] = dg[i][e]; red[w][1][cc * 8 + e] = db[i][e]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) { a += red[q][0][c]; b += red[q][1][c]; }
    part[((size_t)blockIdx.x * 2) * C + c] = a;
    part[((size_t)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

// 16 columns per workgroup x 16 partial-block stripes (a stripe reads 64 contiguous bytes), combined in a fixed
// order through LDS (deterministic).
__global__ __launch_bounds__(256) void layernorm_bwd_reduce_kernel(const float* __restrict__ part, int nblk, int C,
                                                                   float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[16][17];
  const int lc = threadIdx.x & 15, q = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lc;
  float a = 0.f;
  if (c < 2 * C) {
    const int which = c / C, cc = c - which * C;
    for (int b = q; b < nblk; b += 16) a += part[((size_t)b * 2 + which) * C + cc];
  }
  red[q][lc] = a;
  __syncthreads();
  if (q == 0 && c < 2 * C) {
    const int which = c / C, cc = c - which * C;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lc];
    (which ? dbeta : dgamma)[cc] = t;
  }
}

}  // namespace vst

using namespace vst;

// rows per workgroup.  Forward GroupNorms: a function of the sample's (frame's) row count only -- never of how many
// samples share the launch -- so a frame's statistics are the same bits in a batch of any size (the frame-sharded
// forward runs 1/P of the frames per rank, tests/test_frame_shard.py asserts equality); rows / 8 gives >= 8 chunks
// per frame, >= 256 workgroups at the denoise step's 32 frames (the same chunking the old total-rows rule picked
// there: 32 / 128 / 256 rows at 16x16 / 32x32 / 64x64).  Backward (vst_groupnorm_bwd, per-clip samples of the
// training step): >= ~256 workgroups over the whole launch (swept 256..4096 with tools/norm_bench.py).
static inline int gn_rpc_rows(int rows_per_sample) {
  return std::max(8, std::min(256, (rows_per_sample + 7) / 8));
}
static inline int gn_rpc(int nsamples, int rows_per_sample) {
  static const long long target = [] {
    const char* e = getenv("VST_GN_TARGET");  // tuning only (tools/norm_bench.py)
    return e ? std::max(1LL, atoll(e)) : 256LL;
  }();
  const long long total = (long long)nsamples * rows_per_sample;
  return (int)std::max<long long>(8, std::min<long long>(256, (total + target - 1) / target));
}
static inline int gn_nchunk(int nsamples, int rows_per_sample) {
  const int rpc = gn_rpc(nsamples, rows_per_sample);
  return (rows_per_sample + rpc - 1) / rpc;
}
static inline int gn_nchunk_rows(int rows_per_sample) {
  const int rpc = gn_rpc_rows(rows_per_sample);
  return (rows_per_sample + rpc - 1) / rpc;
}
static inline size_t gn_part_floats(int nsamples, int rows_per_sample, int groups) {
  const int nchunk = gn_nchunk(nsamples, rows_per_sample);
  return ((size_t)nsamples * nchunk * groups * 2 + 3) & ~(size_t)3;  // keep scale/shift 16-B aligned
}
static inline size_t gn_part_floats_rows(int nsamples, int rows_per_sample, int groups) {
  return ((size_t)nsamples * gn_nchunk_rows(rows_per_sample) * groups * 2 + 3) & ~(size_t)3;
}

extern "C" size_t vst_groupnorm_workspace_bytes(int nsamples, int rows_per_sample, int groups, int C) {
  return (gn_part_floats_rows(nsamples, rows_per_sample, groups) + (size_t)2 * nsamples * C) * sizeof(float);
}

extern "C" int vst_groupnorm(const void* x1, int ld1, int C1, const void* x2, int ld2, int C2, int nsamples,
                             int rows_per_sample, int groups, float eps, const float* gamma, const float* beta,
                             int silu_act, void* y, int ldy, void* workspace, void* stream) {
  const int C = C1 + (x2 ? C2 : 0);
  if (!x1 || !y || !workspace || !gamma || !beta || nsamples <= 0 || rows_per_sample <= 0 || groups <= 0)
    return VST_ERR_ARG;
  if (C % groups || C % 8 || C1 % 8 || (ld1 & 7) || (ldy & 7) || (x2 && (ld2 & 7))) return VST_ERR_ARG;
  if (C > 4096) return VST_ERR_ARG;
  if (!x2) C2 = 0;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = gn_rpc_rows(rows_per_sample);
  const int nchunk = gn_nchunk_rows(rows_per_sample);
  float* part = (float*)workspace;
  float* scale = part + gn_part_floats_rows(nsamples, rows_per_sample, groups);
  float* shift = scale + (size_t)nsamples * C;
  const int CH = C / 8;
  const int rps = gn_rps(C);
  const size_t lds = (size_t)2 * rps * C * sizeof(float);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(nchunk, nsamples), dim3(rps * CH), lds, s, (const bf16_t*)x1, ld1, C1,
                     (const bf16_t*)x2, ld2, C2, rows_per_sample, rpc, groups, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(nsamples * groups), dim3(64), 0, s, part, nchunk, rows_per_sample,
                     groups, C / groups, eps, gamma, beta, scale, shift, C);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(nchunk, nsamples), dim3(rps * CH), 0, s, (const bf16_t*)x1, ld1, C1,
                     (const bf16_t*)x2, ld2, C2, rows_per_sample, rpc, scale, shift, silu_act, (bf16_t*)y, ldy);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// Column statistics of x [M, C] (C % 8 == 0) as the 128x320 conv epilogue writes them: cs [ceil(M / 128)][C][2].
extern "C" int vst_colstat(const void* x, int ldx, int M, int C, float* cs, void* stream) {
  if (!x || !cs || M <= 0 || C <= 0 || C % 8 || (ldx & 7)) return VST_ERR_ARG;
  hipLaunchKernelGGL(gn_colstat_kernel, dim3((M + 127) / 128, (C + 319) / 320), dim3(512), 0, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, M, C, cs);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// vst_groupnorm with the statistics from column statistics of x1 (and x2) written by the producing conv
// (vst_conv3x3_colstat, 128-row tiles): rows_per_sample % 128 == 0.  workspace: vst_groupnorm_workspace_bytes.
extern "C" int vst_groupnorm_colstat(const void* x1, int ld1, int C1, const float* cs1, const void* x2, int ld2, int C2,
                                     const float* cs2, int nsamples, int rows_per_sample, int groups, float eps,
                                     const float* gamma, const float* beta, int silu_act, void* y, int ldy,
                                     void* workspace, void* stream) {
  const int C = C1 + (x2 ? C2 : 0);
  if (!x1 || !cs1 || !y || !workspace || !gamma || !beta || nsamples <= 0 || rows_per_sample <= 0 || groups <= 0)
    return VST_ERR_ARG;
  if ((x2 && !cs2) || rows_per_sample % 128) return VST_ERR_ARG;
  if (C % groups || C % 8 || C1 % 8 || (ld1 & 7) || (ldy & 7) || (x2 && (ld2 & 7))) return VST_ERR_ARG;
  if (C > 4096) return VST_ERR_ARG;
  if (!x2) C2 = 0;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = gn_rpc_rows(rows_per_sample);
  const int nchunk = gn_nchunk_rows(rows_per_sample);
  float* scale = (float*)workspace + gn_part_floats_rows(nsamples, rows_per_sample, groups);
  float* shift = scale + (size_t)nsamples * C;
  hipLaunchKernelGGL(gn_finalize_colstat_kernel, dim3(nsamples * groups), dim3(64), 0, s, cs1, C1, cs2, C2,
                     rows_per_sample / 128, rows_per_sample, groups, C / groups, eps, gamma, beta, scale, shift);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(nchunk, nsamples), dim3(gn_rps(C) * (C / 8)), 0, s, (const bf16_t*)x1,
                     ld1, C1, (const bf16_t*)x2, ld2, C2, rows_per_sample, rpc, scale, shift, silu_act, (bf16_t*)y,
                     ldy);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

static int gn_check(const void* x1, int ld1, int C1, const void* x2, int ld2, int C2, int nsamples,
                    int rows_per_sample, int groups) {
  const int C = C1 + (x2 ? C2 : 0);
  if (!x1 || nsamples <= 0 || rows_per_sample <= 0 || groups <= 0) return VST_ERR_ARG;
  if (C % groups || C % 8 || C1 % 8 || (ld1 & 7) || (x2 && (ld2 & 7))) return VST_ERR_ARG;
  if (C > 4096) return VST_ERR_ARG;
  return VST_OK;
}

extern "C" int vst_groupnorm_frame_chunks(int rows_per_frame) {
  return rows_per_frame > 0 ? gn_nchunk_rows(rows_per_frame) : 0;
}

extern "C" int vst_groupnorm_frame_partials(const void* x1, int ld1, int C1, int nframes, int rows_per_frame,
                                            int groups, float* part, void* stream) {
  if (gn_check(x1, ld1, C1, nullptr, 0, 0, nframes, rows_per_frame, groups) || !part) return VST_ERR_ARG;
  const int C = C1;
  hipStream_t s = (hipStream_t)stream;
  const int rps = gn_rps(C);
  const size_t lds = (size_t)2 * rps * C * sizeof(float);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(gn_nchunk_rows(rows_per_frame), nframes), dim3(rps * (C / 8)), lds, s,
                     (const bf16_t*)x1, ld1, C1, (const bf16_t*)nullptr, 0, 0, rows_per_frame,
                     gn_rpc_rows(rows_per_frame), groups, part);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

extern "C" int vst_groupnorm_apply_partials(const void* x1, int ld1, int C1, int nclips, int frames_local,
                                            int rows_per_frame, int groups, const float* part, int nranks, float eps,
                                            const float* gamma, const float* beta, int silu_act, void* y, int ldy,
                                            float* scale_shift, void* stream) {
  if (gn_check(x1, ld1, C1, nullptr, 0, 0, nclips * frames_local, rows_per_frame, groups) || nclips <= 0 ||
      frames_local <= 0 || nranks <= 0 || !part || !y || !gamma || !beta || !scale_shift || (ldy & 7) ||
      ((uintptr_t)scale_shift & 15) || (nclips * C1) % 4)
    return VST_ERR_ARG;
  const int C = C1;
  hipStream_t s = (hipStream_t)stream;
  float* scale = scale_shift;
  float* shift = scale + (size_t)nclips * C;
  const int nck = gn_nchunk_rows(rows_per_frame);
  const double count = (double)nranks * frames_local * rows_per_frame * (C / groups);
  hipLaunchKernelGGL(gn_finalize_parts_kernel, dim3(nclips * groups), dim3(64), 0, s, part, nranks, nclips,
                     frames_local, nck, groups, C / groups, count, eps, gamma, beta, scale, shift, C);
  const int rows_per_clip = frames_local * rows_per_frame;
  const int rpc = gn_rpc_rows(rows_per_frame);
  hipLaunchKernelGGL(gn_apply_kernel, dim3((rows_per_clip + rpc - 1) / rpc, nclips), dim3(gn_rps(C) * (C / 8)), 0, s,
                     (const bf16_t*)x1, ld1, C1, (const bf16_t*)nullptr, 0, 0, rows_per_clip, rpc, scale, shift,
                     silu_act, (bf16_t*)y, ldy);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

extern "C" int vst_layernorm(const void* x, int ldx, int C, int rows, const float* gamma, const float* beta,
                             float eps, const float* pe, int pe_div, int pe_mod, void* y, int ldy, void* stream) {
  if (!x || !y || !gamma || !beta || rows <= 0 || C <= 0 || C % 8 || (ldx & 7) || (ldy & 7)) return VST_ERR_ARG;
  if (pe && (pe_div <= 0 || pe_mod <= 0)) return VST_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int CH = C / 8;
  const dim3 blk(256);
#define VST_LNG(LPR, RIT)                                                                                      \
  hipLaunchKernelGGL((layernorm_g_kernel<LPR, RIT>), dim3((rows + 4 * (64 / LPR) * RIT - 1) / (4 * (64 / LPR) * RIT)), \
                     blk, 0, s, (const bf16_t*)x, ldx, C, rows, gamma, beta, eps, pe, pe_div, pe_mod, (bf16_t*)y, ldy)
  static const bool generic_only = getenv("VST_LN_GENERIC") != nullptr;  // A/B switch (tools/ab_bench.sh)
  const bool g16 = !generic_only && ((uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)pe) % 16 == 0;
  // RIT = row passes per wave whose loads are all in flight before the first reduction.  C = 1280 (M = 8192 rows in the
  // step): 1 pass, 1024 workgroups: 9.8 -> 9.2 us per launch graph-timed, step -0.15..-0.2 ms same-box
  // (profiles/r3_ab_ln_rit.txt); VST_LN_RIT (1 / 2 / 4) overrides every width for A/B.
  static const int rit_env = [] {
    const char* e = getenv("VST_LN_RIT");
    return e ? atoi(e) : 0;
  }();
#define VST_LNG_RIT(LPR, DEF)                                        \
  {                                                                  \
    const int rit = rit_env ? rit_env : (DEF);                       \
    if (rit == 1) VST_LNG(LPR, 1);                                   \
    else if (rit == 4) VST_LNG(LPR, 4);                              \
    else VST_LNG(LPR, 2);                                            \
    return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH; \
  }
  if (g16 && C == 320) VST_LNG_RIT(8, 2)
  if (g16 && C == 640) VST_LNG_RIT(16, 2)
  if (g16 && C == 1280) VST_LNG_RIT(32, 1)
#undef VST_LNG_RIT
#undef VST_LNG
#define VST_LN(MC, R)                                                                                          \
  hipLaunchKernelGGL((layernorm_kernel<MC, R>), dim3((rows + 4 * R - 1) / (4 * R)), blk, 0, s, (const bf16_t*)x, ldx, \
                     C, rows, gamma, beta, eps, pe, pe_div, pe_mod, (bf16_t*)y, ldy)
  if (CH <= 64)
    VST_LN(1, 4);
  else if (CH <= 128)
    VST_LN(2, 2);
  else if (CH <= 256)
    VST_LN(4, 2);
#undef VST_LN
  else
    return VST_ERR_ARG;
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

extern "C" int vst_layernorm_lora(const void* x, int ldx, int C, int rows, const float* gamma, const float* beta,
                                  float eps, const void* A, int R, void* y, int ldy, void* u, int ldu, void* stream) {
  if (!x || !y || !u || !A || !gamma || !beta || rows <= 0 || C <= 0 || (C & 31) || C > 1280) return VST_ERR_ARG;
  if (R <= 0 || R > 64 || (R & 15) || (ldx & 7) || (ldy & 7) || (ldu & 3) || ldu < R) return VST_ERR_ARG;
  if (((size_t)(rows - 1) * ldx + C) * 2 > 0x7fffffffULL) return VST_ERR_ARG;  // x through a 32-bit buffer offset
  const dim3 grid((rows + 16 * VST_LNL_MI - 1) / (16 * VST_LNL_MI)), blk(512);
  hipStream_t s = (hipStream_t)stream;
#define VST_LNL(NJ, MT)                                                                                         \
  hipLaunchKernelGGL((layernorm_lora_kernel<NJ, MT>), grid, blk, 0, s, (const bf16_t*)x, ldx, C, rows, gamma, beta, \
                     eps, (const bf16_t*)A, R, (bf16_t*)y, ldy, (bf16_t*)u, ldu)
#define VST_LNL_T(NJ)             \
  if (C <= 256) VST_LNL(NJ, 1);   \
  else if (C <= 512) VST_LNL(NJ, 2); \
  else if (C <= 768) VST_LNL(NJ, 3); \
  else VST_LNL(NJ, 5);
  switch (R / 16) {
    case 1: VST_LNL_T(1); break;
    case 2: VST_LNL_T(2); break;
    case 3: VST_LNL_T(3); break;
    default: VST_LNL_T(4); break;
  }
#undef VST_LNL_T
#undef VST_LNL
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// fp32 residual stream + LayerNorm (the CLIP text encoders, text_encoder.py): h_out = h + y (y bf16, optional),
// n = LN(h_out) in bf16 (the projection input).  The reference's text towers are fp32 modules under bf16 autocast:
// their residual stream stays fp32, only the matmul outputs are bf16 -- so this path keeps it fp32 too.  One
// workgroup of 256 threads per row, two-pass statistics (C <= 2048).
__global__ __launch_bounds__(256) void residual_layernorm_kernel(const float* __restrict__ h, int ldh,
                                                                 const bf16_t* __restrict__ y, int ldy, int C,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float eps,
                                                                 float* __restrict__ ho, int ldho,
                                                                 bf16_t* __restrict__ n, int ldn) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float v[8];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = tid + 256 * e;
    float x = 0.f;
    if (c < C) {
      x = h[(size_t)row * ldh + c];
      if (y) x += bf2f(y[(size_t)row * ldy + c]);
      ho[(size_t)row * ldho + c] = x;
    }
    v[e] = x;
    s += x;
  }
  s = wave_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  const float mean = (red[0] + red[1] + red[2] + red[3]) / C;
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (tid + 256 * e < C) { const float d = v[e] - mean; q += d * d; }
  q = wave_sum(q);
  if (lane == 0) red[w] = q;
  __syncthreads();
  const float rstd = rsqrtf((red[0] + red[1] + red[2] + red[3]) / C + eps);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = tid + 256 * e;
    if (c < C) n[(size_t)row * ldn + c] = f2bf((v[e] - mean) * rstd * gamma[c] + beta[c]);
  }
}

extern "C" int vst_residual_layernorm(const float* h, int ldh, const void* y, int ldy, int rows, int C,
                                      const float* gamma, const float* beta, float eps, float* h_out, int ldho,
                                      void* n, int ldn, void* stream) {
  if (!h || !h_out || !n || !gamma || !beta || rows <= 0 || C <= 0 || C > 2048 || ldh < C || ldho < C || ldn < C ||
      (y && ldy < C))
    return VST_ERR_ARG;
  hipLaunchKernelGGL(residual_layernorm_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, h, ldh,
                     (const bf16_t*)y, ldy, C, gamma, beta, eps, h_out, ldho, (bf16_t*)n, ldn);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// ---- LayerNorm backward (training path) ----
static inline int lnb_grid(int rows) { return std::max(1, std::min(512, (rows + 3) / 4)); }

extern "C" size_t vst_layernorm_bwd_workspace_bytes(int C, int rows) {
  return (size_t)lnb_grid(rows) * 2 * C * sizeof(float);
}

extern "C" int vst_layernorm_bwd(const void* x, int ldx, const void* g, int ldg, int C, int rows, const float* gamma,
                                 float eps, void* dx, int lddx, float* dgamma, float* dbeta, void* workspace,
                                 void* stream) {
  // dgamma == dbeta == NULL: dx only (frozen affine), no workspace needed
  if (!x || !g || !dx || !gamma || (!dgamma) != (!dbeta) || (dgamma && !workspace) || rows <= 0 || C <= 0 ||
      C % 8 || (ldx & 7) || (ldg & 7) || (lddx & 7) || C > 2048)
    return VST_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int grid = lnb_grid(rows);
  float* part = dgamma ? (float*)workspace : nullptr;
  const int CH = C / 8;
#define VST_LNB(MC)                                                                                            \
  hipLaunchKernelGGL((layernorm_bwd_kernel<MC>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, ldx, (const bf16_t*)g, \
                     ldg, C, rows, gamma, eps, (bf16_t*)dx, lddx, part)
  if (CH <= 64) VST_LNB(1);
  else if (CH <= 128) VST_LNB(2);
  else VST_LNB(4);
#undef VST_LNB
  if (dgamma)
    hipLaunchKernelGGL(layernorm_bwd_reduce_kernel, dim3((2 * C + 15) / 16), dim3(256), 0, s, part, grid, C, dgamma,
                       dbeta);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// ---- GroupNorm backward host side ----
static inline size_t gnb_floats(int nsamples, int rows_per_sample, int groups, int C) {
  const size_t nchunk = gn_nchunk(nsamples, rows_per_sample);
  const size_t a4 = 4;
  auto up = [&](size_t n) { return (n + a4 - 1) / a4 * a4; };
  return up(gn_part_floats(nsamples, rows_per_sample, groups)) + up((size_t)2 * nsamples * C)  // part, scale/shift
         + up((size_t)2 * nsamples * groups) + up((size_t)nsamples * nchunk * 2 * C)           // stats, part2
         + up((size_t)2 * nsamples * C) + up((size_t)3 * nsamples * C);                        // chsum, coef
}

extern "C" size_t vst_groupnorm_bwd_workspace_bytes(int nsamples, int rows_per_sample, int groups, int C) {
  return gnb_floats(nsamples, rows_per_sample, groups, C) * sizeof(float);
}

extern "C" int vst_groupnorm_bwd(const void* x, int ldx, const void* g, int ldg, int C, int nsamples,
                                 int rows_per_sample, int groups, float eps, const float* gamma, const float* beta,
                                 int silu_act, void* dx, int lddx, float* dgamma, float* dbeta, void* workspace,
                                 void* stream) {
  if (!x || !g || !dx || !gamma || !beta || !dgamma || !dbeta || !workspace || nsamples <= 0 ||
      rows_per_sample <= 0 || groups <= 0 || C % groups || C % 8 || C > 4096 || (ldx & 7) || (ldg & 7) || (lddx & 7))
    return VST_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = gn_rpc(nsamples, rows_per_sample);
  const int nchunk = gn_nchunk(nsamples, rows_per_sample);
  const int CH = C / 8, rps = gn_rps(C);
  auto up = [](size_t n) { return (n + 3) / 4 * 4; };
  float* part = (float*)workspace;
  float* scale = part + up(gn_part_floats(nsamples, rows_per_sample, groups));
  float* shift = scale + nsamples * (size_t)C;
  float* stats = scale + up((size_t)2 * nsamples * C);
  float* part2 = stats + up((size_t)2 * nsamples * groups);
  float* chsum = part2 + up((size_t)nsamples * nchunk * 2 * C);
  float* coef = chsum + up((size_t)2 * nsamples * C);
  const size_t lds = (size_t)2 * rps * C * sizeof(float);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(nchunk, nsamples), dim3(rps * CH), lds, s, (const bf16_t*)x, ldx, C,
                     (const bf16_t*)nullptr, 0, 0, rows_per_sample, rpc, groups, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(nsamples * groups), dim3(64), 0, s, part, nchunk, rows_per_sample,
                     groups, C / groups, eps, gamma, beta, scale, shift, C, stats);
  hipLaunchKernelGGL(gn_bwd_sums_kernel, dim3(nchunk, nsamples), dim3(rps * CH), lds, s, (const bf16_t*)x, ldx,
                     (const bf16_t*)g, ldg, C, rows_per_sample, rpc, scale, shift, silu_act, part2);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(nsamples * groups), dim3(64), 0, s, part2, nchunk, C, groups,
                     rows_per_sample, stats, gamma, chsum, coef);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3(nchunk, nsamples), dim3(rps * CH), 0, s, (const bf16_t*)x, ldx,
                     (const bf16_t*)g, ldg, C, rows_per_sample, rpc, scale, shift, silu_act, coef, (bf16_t*)dx, lddx);
  hipLaunchKernelGGL(gn_bwd_param_kernel, dim3((C + 255) / 256), dim3(256), 0, s, chsum, nsamples, C, dgamma, dbeta);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}
