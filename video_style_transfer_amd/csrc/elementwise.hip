// Small element-wise kernels around the UNet: timestep embeddings, latent packing,
// the fused CFG-combine + Euler step of the denoise loop, and glue (silu, add, copy).
// Per-step scalars (timestep, sigma) are read from device tables indexed by a device
// step counter, so one captured HIP graph of a denoise step replays for every step.
#include "vst_common.h"

namespace vst {

// diffusers get_timestep_embedding (max_period 10000): value i -> row (i / per_row),
// columns col0 + (i % per_row)*dim + [0, dim)
__global__ void timestep_embed_kernel(const float* __restrict__ t, const int* __restrict__ step, int n, int dim,
                                      int flip, float shift, bf16_t* __restrict__ out, int ld, int col0,
                                      int per_row) {
  const int half = dim / 2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * half) return;
  const int i = idx / half, j = idx - i * half;
  const float tv = step ? t[*step] : t[i];
  const float freq = expf(-9.210340371976184f * (float)j / ((float)half - shift));  // ln(10000)
  const float a = tv * freq;
  const float s = sinf(a), c = cosf(a);
  bf16_t* o = out + (size_t)(i / per_row) * ld + col0 + (i % per_row) * dim;
  if (flip) { o[j] = f2bf(c); o[half + j] = f2bf(s); }
  else { o[j] = f2bf(s); o[half + j] = f2bf(c); }
}

__global__ void silu_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(silu(bf2f(x[i])));
}

// transformers' quick_gelu (CLIP ViT-L/14 text MLP): x * sigmoid(1.702 x), fp32 math, one rounding
__global__ void quick_gelu_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = bf2f(x[i]);
    y[i] = f2bf(v / (1.f + __expf(-1.702f * v)));
  }
}

// CLIPTextEmbeddings: y[r][c] = token_embedding[ids[r]][c] + position_embedding[r % L][c], fp32 (the text towers'
// residual stream, text_encoder.py)
__global__ void embed_tokens_kernel(const int* __restrict__ ids, int rows, int L, const bf16_t* __restrict__ tok,
                                    const bf16_t* __restrict__ pos, int C, float* __restrict__ y, int ldy) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * C) return;
  const int r = idx / C, c = idx - r * C;
  y[(size_t)r * ldy + c] = bf2f(tok[(size_t)ids[r] * C + c]) + bf2f(pos[(size_t)(r % L) * C + c]);
}

__global__ void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                           size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

__global__ void copy2d_kernel(const bf16_t* __restrict__ x, int ldx, bf16_t* __restrict__ y, int ldy, int rows,
                              int cols) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const int r = idx / cols, c = idx - r * cols;
  y[(size_t)r * ldy + c] = x[(size_t)r * ldx + c];
}

// latents fp32 (B, Cl, F, H, W) -> bf16 NHWC rows ((k*B + b)*F + f)*H*W + p, Cl channels,
// scaled by 1/sqrt(sigma^2 + 1) (EulerDiscreteScheduler.scale_model_input), ncopy copies (CFG).
__global__ void pack_latents_kernel(const float* __restrict__ lat, int B, int Cl, int F, int HW,
                                    const float* __restrict__ sigmas, const int* __restrict__ step, float fixed_scale,
                                    int ncopy, bf16_t* __restrict__ out) {
  const size_t n = (size_t)B * Cl * F * HW;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int p = (int)(idx % HW);
  size_t r = idx / HW;
  const int f = (int)(r % F); r /= F;
  const int c = (int)(r % Cl);
  const int b = (int)(r / Cl);
  float scale = fixed_scale;
  if (sigmas) { const float sg = sigmas[*step]; scale = rsqrtf(sg * sg + 1.0f); }
  const uint16_t v = f2bf(lat[idx] * scale);
  for (int k = 0; k < ncopy; ++k) out[((size_t)((k * B + b) * F + f) * HW + p) * Cl + c] = v;
}

// noise NHWC bf16 rows as above with ncopy=2 (k=0 uncond, k=1 cond) or 1 (no CFG).
// latents += (sigma[step+1] - sigma[step]) * (u + g (c - u))   (Euler, epsilon prediction)
__global__ void euler_cfg_kernel(const bf16_t* __restrict__ noise, int ncopy, float guidance, float* __restrict__ lat,
                                 int B, int Cl, int F, int HW, const float* __restrict__ sigmas,
                                 const int* __restrict__ step) {
  const size_t n = (size_t)B * Cl * F * HW;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int p = (int)(idx % HW);
  size_t r = idx / HW;
  const int f = (int)(r % F); r /= F;
  const int c = (int)(r % Cl);
  const int b = (int)(r / Cl);
  float eps;
  if (ncopy == 2) {
    const float u = bf2f(noise[((size_t)(b * F + f) * HW + p) * Cl + c]);
    const float cc = bf2f(noise[((size_t)((B + b) * F + f) * HW + p) * Cl + c]);
    eps = u + guidance * (cc - u);
  } else {
    eps = bf2f(noise[((size_t)(b * F + f) * HW + p) * Cl + c]);
  }
  const int s = *step;
  lat[idx] += (sigmas[s + 1] - sigmas[s]) * eps;
}

// Row-block permutation for the frame <-> pixel shard exchange of the motion module.  Rows of C
// bf16 are indexed 4-D in the source, (i0, i1, i2, i3) with dims d[0..3]; destination axis k is
// source axis perm[k].  One thread moves 16 B.
__global__ __launch_bounds__(256) void permute_rows_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                           int C, int4 d, int4 perm, size_t total_chunks) {
  const int dd[4] = {d.x, d.y, d.z, d.w};
  const int pp[4] = {perm.x, perm.y, perm.z, perm.w};
  const int CH = C / 8;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total_chunks; idx += (size_t)gridDim.x * 256) {
    size_t row = idx / CH;
    const int c = (int)(idx - row * CH) * 8;
    int j[4], i[4];
#pragma unroll
    for (int k = 3; k >= 0; --k) {
      const int dk = dd[pp[k]];
      j[k] = (int)(row % dk);
      row /= dk;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) i[pp[k]] = j[k];
    const size_t srow = (((size_t)i[0] * dd[1] + i[1]) * dd[2] + i[2]) * dd[3] + i[3];
    const size_t drow = idx / CH;
    *reinterpret_cast<u32x4*>(dst + drow * C + c) = *reinterpret_cast<const u32x4*>(src + srow * C + c);
  }
}

// y[row] = x[row] + table[(row / div) % mod]: the reference TemporalTransformer's PositionalEncoding
// (animatediff/temporal_transformer.py:20-27) on token rows (b*F + f)*HW + p with div = HW, mod = F.
__global__ __launch_bounds__(256) void add_row_table_kernel(const bf16_t* __restrict__ x, int ldx, int C,
                                                            const float* __restrict__ table, int div, int mod,
                                                            bf16_t* __restrict__ y, int ldy, size_t total_chunks) {
  const int CH = C / 8;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total_chunks; idx += (size_t)gridDim.x * 256) {
    const size_t row = idx / CH;
    const int c = (int)(idx - row * CH) * 8;
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + row * ldx + c), f);
    const f32x4* t = reinterpret_cast<const f32x4*>(table + (size_t)((row / div) % mod) * C + c);
    const f32x4 t0 = t[0], t1 = t[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] += t0[e]; f[e + 4] += t1[e]; }
    *reinterpret_cast<u32x4*>(y + row * ldy + c) = pack8(f);
  }
}

// bf16 token rows ((b*F + f)*HW + p, C) -> fp32 (B, C, F, HW): the inverse of pack_latents (the 5-D
// output of UNetMotionModel / TemporalTransformer).  64-pixel x 64-channel tiles transposed through
// LDS so both the 16-B row reads and the fp32 pixel-run writes are coalesced.
__global__ __launch_bounds__(256) void unpack_tokens_kernel(const bf16_t* __restrict__ src, int C, int F, int HW,
                                                            float* __restrict__ out) {
  __shared__ float tile[64][65];
  const int img = blockIdx.z;  // b*F + f
  const int b = img / F, f = img - b * F;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k;
    const int r = idx >> 3, ch = (idx & 7) * 8;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (p0 + r < HW && c0 + ch < C)
      unpack8(*reinterpret_cast<const u32x4*>(src + ((size_t)img * HW + p0 + r) * C + c0 + ch), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[ch + e][r] = v[e];
  }
  __syncthreads();
  const int pl = tid & 63;
  for (int cl = tid >> 6; cl < 64; cl += 4) {
    const int c = c0 + cl, p = p0 + pl;
    if (c < C && p < HW) out[(((size_t)b * C + c) * F + f) * HW + p] = tile[cl][pl];
  }
}

// bf16 transpose y[c][r] = x[r][c] through a 64x64 LDS tile (backward-pass operand layouts: dW = dY^T X needs
// the token axis as the GEMM's K, i.e. row-major [features, tokens] copies of dY and X).
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ x, int ldx, int rows, int cols,
                                                        bf16_t* __restrict__ y, int ldy) {
  __shared__ uint16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  const bool vec_in = (cols & 7) == 0 && (ldx & 7) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k;
    const int r = idx >> 3, ch = (idx & 7) * 8;
    const int gr = r0 + r, gc = c0 + ch;
    uint16_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (gr < rows) {
      if (vec_in && gc + 8 <= cols) {
        const u32x4 w = *reinterpret_cast<const u32x4*>(x + (size_t)gr * ldx + gc);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[2 * e] = (uint16_t)(w[e] & 0xffffu); v[2 * e + 1] = (uint16_t)(w[e] >> 16); }
      } else {
        for (int e = 0; e < 8; ++e)
          if (gc + e < cols) v[e] = x[(size_t)gr * ldx + gc + e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[r][ch + e] = v[e];
  }
  __syncthreads();
  const bool vec_out = (rows & 7) == 0 && (ldy & 7) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k;
    const int c = idx >> 3, rr = (idx & 7) * 8;  // output row c0 + c, output columns r0 + rr .. +7
    const int gc = c0 + c, gr = r0 + rr;
    if (gc >= cols) continue;
    uint16_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[rr + e][c];
    if (vec_out && gr + 8 <= rows) {
      u32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (uint32_t)v[2 * e] | ((uint32_t)v[2 * e + 1] << 16);
      *reinterpret_cast<u32x4*>(y + (size_t)gc * ldy + gr) = w;
    } else {
      for (int e = 0; e < 8; ++e)
        if (gr + e < rows) y[(size_t)gc * ldy + gr + e] = v[e];
    }
  }
}

// GEGLU backward (training path): the FF projection output p is stored in the GEMM's 32-interleaved layout —
// block b = [32 hidden | 32 gate] columns 64b.., producing output columns 32b.. (diffusers GEGLU:
// out = h * gelu(gate)).  Given g = dL/dout:  dh = g * gelu(gate),  dgate = g * h * gelu'(gate),
// gelu'(z) = Phi(z) + z * phi(z).  dp is written in the same interleaved layout (the dX / dW GEMMs use the
// interleaved weights as they are).
__global__ __launch_bounds__(256) void geglu_bwd_kernel(const bf16_t* __restrict__ p, int ldp,
                                                        const bf16_t* __restrict__ g, int ldg, int M, int Nh,
                                                        bf16_t* __restrict__ dp, int lddp) {
  const int cpr = Nh / 8;  // 8-column chunks of g per row
  const size_t total = (size_t)M * cpr;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
    const int m = (int)(idx / cpr);
    const int oc = (int)(idx - (size_t)m * cpr) * 8;
    const int blk = oc >> 5, c = oc & 31;
    const int hcol = blk * 64 + c, gcol = hcol + 32;
    float gv[8], hv[8], zv[8], dh[8], dz[8];
    unpack8(*reinterpret_cast<const u32x4*>(g + (size_t)m * ldg + oc), gv);
    unpack8(*reinterpret_cast<const u32x4*>(p + (size_t)m * ldp + hcol), hv);
    unpack8(*reinterpret_cast<const u32x4*>(p + (size_t)m * ldp + gcol), zv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float z = zv[e];
      const float cdf = 0.5f * (1.0f + erf_fast(z * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.5f * z * z * 1.4426950408889634f);
      dh[e] = gv[e] * z * cdf;
      dz[e] = gv[e] * hv[e] * (cdf + z * pdf);
    }
    *reinterpret_cast<u32x4*>(dp + (size_t)m * lddp + hcol) = pack8(dh);
    *reinterpret_cast<u32x4*>(dp + (size_t)m * lddp + gcol) = pack8(dz);
  }
}

// Conv data-gradient helpers for the down/up samplers (training path):
//  zero_insert: y[n, 2i, 2j, :] = x[n, i, j, :] on a zeroed [n, 2h, 2w, C] grid (stride-2 conv dgrad = stride-1
//               conv of the zero-inserted dY with flipped weights);
//  sumpool2x2:  y[n, i, j, :] = sum of x[n, 2i..2i+1, 2j..2j+1, :] (the adjoint of the nearest-2x upsample).
__global__ __launch_bounds__(256) void zero_insert_kernel(const bf16_t* __restrict__ x, int nimg, int h, int w, int C,
                                                          bf16_t* __restrict__ y) {
  const int CH = C / 8;
  const size_t total = (size_t)nimg * h * w * CH;
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
    const int c = (int)(idx % CH) * 8;
    const size_t pix = idx / CH;
    const int j = (int)(pix % w), i = (int)((pix / w) % h);
    const size_t n = pix / ((size_t)w * h);
    *reinterpret_cast<u32x4*>(y + ((n * 2 * h + 2 * i) * 2 * w + 2 * j) * C + c) =
        *reinterpret_cast<const u32x4*>(x + pix * C + c);
  }
}

__global__ __launch_bounds__(256) void sumpool2x2_kernel(const bf16_t* __restrict__ x, int nimg, int h, int w, int C,
                                                         bf16_t* __restrict__ y) {
  const int CH = C / 8;
  const size_t total = (size_t)nimg * h * w * CH;  // output pixels x chunks (h, w: OUTPUT size)
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
    const int c = (int)(idx % CH) * 8;
    const size_t pix = idx / CH;
    const int j = (int)(pix % w), i = (int)((pix / w) % h);
    const size_t n = pix / ((size_t)w * h);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float v[8];
        unpack8(*reinterpret_cast<const u32x4*>(x + ((n * 2 * h + 2 * i + dy) * 2 * w + 2 * j + dx) * C + c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    *reinterpret_cast<u32x4*>(y + pix * C + c) = pack8(acc);
  }
}

// The counter wraps at num_steps: a graph replayed past the end of the schedule starts it again instead of
// indexing sigmas[] / timesteps[] (num_steps + 1 / num_steps entries) out of bounds.
__global__ void step_advance_kernel(int* step, int num_steps) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const int s = *step + 1;
    *step = (s >= num_steps || s < 0) ? 0 : s;
  }
}


// ---- SDXL VAE (AutoencoderKL) glue: layout conversions at the fp32 NCHW boundary, latent sampling, frame output,
// and the row softmax of the mid-block attention (head_dim 512: scores come fp32 from vst_gemm_f32out) ----

// dst[(img*HW + p)*ldd + c] = bf16(src[(img*C + c)*HW + p] * mul) for c < C, 0 for C <= c < ldd
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ src, int n, int C, int HW, float mul,
                                    bf16_t* __restrict__ dst, int ldd) {
  const size_t total = (size_t)n * HW * ldd;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % ldd);
    const size_t t = i / ldd;  // img * HW + p
    const int p = (int)(t % HW);
    const size_t img = t / HW;
    dst[i] = c < C ? f2bf(src[(img * C + c) * HW + p] * mul) : (bf16_t)0;
  }
}

// dst[(img*C + c)*HW + p] = src[(img*HW + p)*ld + c]  (bf16 NHWC -> fp32 NCHW)
__global__ void nhwc_to_nchw_kernel(const bf16_t* __restrict__ src, int ld, int n, int C, int HW,
                                    float* __restrict__ dst) {
  const size_t total = (size_t)n * C * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % HW);
    const size_t t = i / HW;  // img * C + c
    const int c = (int)(t % C);
    const size_t img = t / C;
    dst[i] = bf2f(src[(img * HW + p) * ld + c]);
  }
}

// inference_animatediff.py:141-143: (x / 2 + 0.5).clamp(0, 1), then (x * 255).astype(np.uint8) (truncation), HWC
__global__ void frames_to_u8_kernel(const bf16_t* __restrict__ src, int ld, int n, int C, int HW,
                                    uint8_t* __restrict__ dst) {
  const size_t total = (size_t)n * HW * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const size_t t = i / C;
    const float v = fminf(fmaxf(bf2f(src[t * ld + c]) / 2.f + 0.5f, 0.f), 1.f);
    dst[i] = (uint8_t)(int)(v * 255.f);
  }
}

// DiagonalGaussianDistribution(moments).sample() * scaling_factor (train_animatediff.py:222-223): moments NHWC
// [n*HW][ld] bf16 with mean = channels 0..3, logvar = 4..7; logvar clamped to [-30, 20]; eps fp32 NCHW (n, 4, HW);
// out fp32 NCHW.  eps == nullptr: the distribution's mode (mean).
__global__ void vae_sample_kernel(const bf16_t* __restrict__ mom, int ld, int n, int HW, const float* __restrict__ eps,
                                  float mul, float* __restrict__ out) {
  const size_t total = (size_t)n * 4 * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % HW);
    const size_t t = i / HW;
    const int c = (int)(t % 4);
    const size_t img = t / 4;
    const bf16_t* m = mom + (img * HW + p) * ld;
    float v = bf2f(m[c]);
    if (eps) {
      const float lv = fminf(fmaxf(bf2f(m[4 + c]), -30.f), 20.f);
      v += expf(0.5f * lv) * eps[i];
    }
    out[i] = v * mul;
  }
}

// P[r][:] = softmax(scale * S[r][:]) in fp32, stored bf16.  One wave per row: an online (max, sum) pass, then the
// normalised exponentials (the second read of the row is an L2 hit).
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ S, int lds, int rows, int n,
                                                           float scale_log2, bf16_t* __restrict__ P, int ldp) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* s = S + (size_t)r * lds;
  float m = -INFINITY, l = 0.f;
  for (int j = lane * 4; j < n; j += 256) {
    float v[4];
    if (j + 4 <= n) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(s + j);
      v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    } else {
      for (int e = 0; e < 4; ++e) v[e] = j + e < n ? s[j + e] : -INFINITY;
    }
    float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])) * scale_log2;
    const float mn = fmaxf(m, mx);
    l *= exp2f(m - mn);
    for (int e = 0; e < 4; ++e) l += exp2f(v[e] * scale_log2 - mn);
    m = mn;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o), lo = __shfl_xor(l, o);
    const float mn = fmaxf(m, mo);
    if (mn != -INFINITY) {  // lanes past n hold (-inf, 0)
      l = (m == -INFINITY ? 0.f : l * exp2f(m - mn)) + (mo == -INFINITY ? 0.f : lo * exp2f(mo - mn));
      m = mn;
    }
  }
  const float inv = 1.f / l;
  bf16_t* p = P + (size_t)r * ldp;
  for (int j = lane * 4; j < n; j += 256) {
    if (j + 4 <= n) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(s + j);
      u32x2 w{pack2bf(exp2f(q[0] * scale_log2 - m) * inv, exp2f(q[1] * scale_log2 - m) * inv),
              pack2bf(exp2f(q[2] * scale_log2 - m) * inv, exp2f(q[3] * scale_log2 - m) * inv)};
      *reinterpret_cast<u32x2*>(p + j) = w;
    } else {
      for (int e = 0; j + e < n; ++e) p[j + e] = f2bf(exp2f(s[j + e] * scale_log2 - m) * inv);
    }
  }
}

}  // namespace vst

using namespace vst;

static inline int ok() { return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH; }

extern "C" int vst_timestep_embedding(const float* t, const int* step_idx, int n, int dim, int flip_sin_to_cos,
                                      float downscale_freq_shift, void* out, int ld, int col0, int per_row,
                                      void* stream) {
  if (!t || !out || n <= 0 || dim <= 0 || (dim & 1) || per_row <= 0) return VST_ERR_ARG;
  const int tot = n * (dim / 2);
  hipLaunchKernelGGL(timestep_embed_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, t, step_idx,
                     n, dim, flip_sin_to_cos, downscale_freq_shift, (bf16_t*)out, ld, col0, per_row);
  return ok();
}

extern "C" int vst_silu(const void* x, void* y, size_t n, void* stream) {
  if (!x || !y) return VST_ERR_ARG;
  const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(silu_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, n);
  return ok();
}

extern "C" int vst_quick_gelu(const void* x, void* y, size_t n, void* stream) {
  if (!x || !y) return VST_ERR_ARG;
  const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(quick_gelu_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y,
                     n);
  return ok();
}

extern "C" int vst_embed_tokens(const int* ids, int rows, int L, const void* tok, const void* pos, int C, float* y,
                                int ldy, void* stream) {
  if (!ids || !tok || !pos || !y || rows <= 0 || L <= 0 || C <= 0 || ldy < C) return VST_ERR_ARG;
  hipLaunchKernelGGL(embed_tokens_kernel, dim3((rows * C + 255) / 256), dim3(256), 0, (hipStream_t)stream, ids, rows,
                     L, (const bf16_t*)tok, (const bf16_t*)pos, C, y, ldy);
  return ok();
}

extern "C" int vst_add(const void* a, const void* b, void* y, size_t n, void* stream) {
  if (!a || !b || !y) return VST_ERR_ARG;
  const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(add_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)a, (const bf16_t*)b,
                     (bf16_t*)y, n);
  return ok();
}

extern "C" int vst_copy2d(const void* x, int ldx, void* y, int ldy, int rows, int cols, void* stream) {
  if (!x || !y || rows <= 0 || cols <= 0) return VST_ERR_ARG;
  const int tot = rows * cols;
  hipLaunchKernelGGL(copy2d_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     ldx, (bf16_t*)y, ldy, rows, cols);
  return ok();
}

extern "C" int vst_pack_latents(const float* lat, int B, int Cl, int F, int HW, const float* sigmas,
                                const int* step_idx, float fixed_scale, int ncopy, void* out, void* stream) {
  if (!lat || !out || B <= 0 || Cl <= 0 || F <= 0 || HW <= 0 || ncopy <= 0) return VST_ERR_ARG;
  if (sigmas && !step_idx) return VST_ERR_ARG;
  const size_t n = (size_t)B * Cl * F * HW;
  hipLaunchKernelGGL(pack_latents_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lat, B,
                     Cl, F, HW, sigmas, step_idx, fixed_scale, ncopy, (bf16_t*)out);
  return ok();
}

extern "C" int vst_euler_cfg_step(const void* noise, int ncopy, float guidance, float* lat, int B, int Cl, int F,
                                  int HW, const float* sigmas, const int* step_idx, void* stream) {
  if (!noise || !lat || !sigmas || !step_idx || (ncopy != 1 && ncopy != 2)) return VST_ERR_ARG;
  const size_t n = (size_t)B * Cl * F * HW;
  hipLaunchKernelGGL(euler_cfg_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)noise, ncopy, guidance, lat, B, Cl, F, HW, sigmas, step_idx);
  return ok();
}

extern "C" int vst_step_advance(int* step_idx, int num_steps, void* stream) {
  if (!step_idx || num_steps <= 0) return VST_ERR_ARG;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step_idx, num_steps);
  return ok();
}

extern "C" int vst_permute_rows(const void* src, void* dst, int C, int d0, int d1, int d2, int d3, int p0, int p1,
                                int p2, int p3, void* stream) {
  if (!src || !dst || src == dst || C <= 0 || (C & 7) || d0 <= 0 || d1 <= 0 || d2 <= 0 || d3 <= 0) return VST_ERR_ARG;
  const int pp[4] = {p0, p1, p2, p3};
  int seen = 0;
  for (int k = 0; k < 4; ++k) {
    if (pp[k] < 0 || pp[k] > 3 || (seen >> pp[k]) & 1) return VST_ERR_ARG;
    seen |= 1 << pp[k];
  }
  const size_t total = (size_t)d0 * d1 * d2 * d3 * (C / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(permute_rows_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)src,
                     (bf16_t*)dst, C, make_int4(d0, d1, d2, d3), make_int4(p0, p1, p2, p3), total);
  return ok();
}

extern "C" int vst_add_row_table(const void* x, int ldx, int C, int rows, const float* table, int div, int mod,
                                 void* y, int ldy, void* stream) {
  if (!x || !y || !table || rows <= 0 || C <= 0 || (C & 7) || (ldx & 7) || (ldy & 7) || div <= 0 || mod <= 0)
    return VST_ERR_ARG;
  const size_t total = (size_t)rows * (C / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(add_row_table_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, C,
                     table, div, mod, (bf16_t*)y, ldy, total);
  return ok();
}

extern "C" int vst_unpack_tokens(const void* src, int B, int C, int F, int HW, float* out, void* stream) {
  if (!src || !out || B <= 0 || C <= 0 || (C & 7) || F <= 0 || HW <= 0 || B * F > 65535) return VST_ERR_ARG;
  const dim3 grid((HW + 63) / 64, (C + 63) / 64, B * F);
  hipLaunchKernelGGL(unpack_tokens_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)src, C, F, HW,
                     out);
  return ok();
}

extern "C" int vst_transpose(const void* x, int ldx, int rows, int cols, void* y, int ldy, void* stream) {
  if (!x || !y || rows <= 0 || cols <= 0 || ldx < cols || ldy < rows) return VST_ERR_ARG;
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (grid.y > 65535) return VST_ERR_ARG;
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, rows, cols,
                     (bf16_t*)y, ldy);
  return ok();
}

extern "C" int vst_geglu_bwd(const void* p, int ldp, const void* g, int ldg, int M, int Nh, void* dp, int lddp,
                             void* stream) {
  if (!p || !g || !dp || M <= 0 || Nh <= 0 || Nh % 32 || (ldp & 7) || (ldg & 7) || (lddp & 7) || ldp < 2 * Nh ||
      lddp < 2 * Nh)
    return VST_ERR_ARG;
  const size_t total = (size_t)M * (Nh / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)p, ldp,
                     (const bf16_t*)g, ldg, M, Nh, (bf16_t*)dp, lddp);
  return ok();
}

extern "C" int vst_zero_insert(const void* x, int nimg, int h, int w, int C, void* y, void* stream) {
  if (!x || !y || nimg <= 0 || h <= 0 || w <= 0 || C <= 0 || C % 8) return VST_ERR_ARG;
  const size_t total = (size_t)nimg * h * w * (C / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(zero_insert_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, nimg, h, w,
                     C, (bf16_t*)y);
  return ok();
}

extern "C" int vst_sumpool2x2(const void* x, int nimg, int h, int w, int C, void* y, void* stream) {
  if (!x || !y || nimg <= 0 || h <= 0 || w <= 0 || C <= 0 || C % 8) return VST_ERR_ARG;
  const size_t total = (size_t)nimg * h * w * (C / 8);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(sumpool2x2_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, nimg, h, w,
                     C, (bf16_t*)y);
  return ok();
}

static inline int grid_for(size_t total) { return (int)std::min<size_t>((total + 255) / 256, 16384); }

extern "C" int vst_nchw_to_nhwc(const float* src, int n, int C, int HW, float mul, void* dst, int ldd, void* stream) {
  if (!src || !dst || n <= 0 || C <= 0 || HW <= 0 || ldd < C) return VST_ERR_ARG;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((size_t)n * HW * ldd)), dim3(256), 0, (hipStream_t)stream, src,
                     n, C, HW, mul, (bf16_t*)dst, ldd);
  return ok();
}

extern "C" int vst_nhwc_to_nchw(const void* src, int ld, int n, int C, int HW, float* dst, void* stream) {
  if (!src || !dst || n <= 0 || C <= 0 || HW <= 0 || ld < C) return VST_ERR_ARG;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for((size_t)n * C * HW)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, ld, n, C, HW, dst);
  return ok();
}

extern "C" int vst_frames_to_u8(const void* src, int ld, int n, int C, int HW, void* dst, void* stream) {
  if (!src || !dst || n <= 0 || C <= 0 || HW <= 0 || ld < C) return VST_ERR_ARG;
  hipLaunchKernelGGL(frames_to_u8_kernel, dim3(grid_for((size_t)n * HW * C)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, ld, n, C, HW, (uint8_t*)dst);
  return ok();
}

extern "C" int vst_vae_sample(const void* moments, int ld, int n, int HW, const float* eps, float mul, float* out,
                              void* stream) {
  if (!moments || !out || n <= 0 || HW <= 0 || ld < 8) return VST_ERR_ARG;
  hipLaunchKernelGGL(vae_sample_kernel, dim3(grid_for((size_t)n * 4 * HW)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)moments, ld, n, HW, eps, mul, out);
  return ok();
}

extern "C" int vst_softmax_rows(const float* S, int lds, int rows, int n, float scale, void* P, int ldp, void* stream) {
  if (!S || !P || rows <= 0 || n <= 0 || lds < n || ldp < n || (lds & 3) || (ldp & 3)) return VST_ERR_ARG;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, lds, rows, n,
                     scale * 1.4426950408889634f, (bf16_t*)P, ldp);
  return ok();
}

extern "C" const char* vst_version(void) { return "vst-hip 0.1 gfx950"; }

// ---- column sums (training path: bias gradients db = g^T 1) ------------------------------------------------------
// bf16 [M, N] row-major view -> fp32 [N], deterministic and graph-safe (no atomics, no memset; a captured HIP graph
// replays it bit for bit; torch's g.float().sum(0) also writes and re-reads an fp32 copy of g):
//   pass 1: R row blocks x (N/512) column blocks; lane = 8-column chunk (16-B loads, 4 rows in flight per lane), the
//           4 waves stride the block's rows and are combined in LDS in wave order -> part1 [R][N];
//   pass 2: part1 summed in groups of 32 rows (unrolled) -> part2 [ceil(R/32)][N];
//   pass 3: part2 summed (<= 32 rows) -> y.  Every pass has fixed summation order and short dependent chains.
namespace {
struct ColsumPlan {
  int gx, R, rows_per_blk, R2;
};
ColsumPlan colsum_plan(int M, int N) {
  ColsumPlan p;
  p.gx = (N / 8 + 63) / 64;
  int R = (2048 + p.gx - 1) / p.gx;                       // ~2048 workgroups in pass 1
  R = std::max(1, std::min(std::min(R, 1024), (M + 63) / 64));  // >= 64 rows per block, R2 <= 32
  p.rows_per_blk = ((M + R - 1) / R + 3) / 4 * 4;
  p.R = (M + p.rows_per_blk - 1) / p.rows_per_blk;
  p.R2 = (p.R + 31) / 32;
  return p;
}
}  // namespace

__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16_t* __restrict__ x, int ldx, int M, int N,
                                                             int rows_per_blk, float* __restrict__ part) {
  __shared__ float red[3][64][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk = blockIdx.x * 64 + lane;
  const bool active = chunk < N / 8;
  const int r0 = blockIdx.y * rows_per_blk;
  const int r1 = min(M, r0 + rows_per_blk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    const bf16_t* base = x + (size_t)chunk * 8;
    int r = r0 + wave;
    for (; r + 12 < r1; r += 16) {  // four rows in flight per lane
      u32x4 a = *reinterpret_cast<const u32x4*>(base + (size_t)r * ldx);
      u32x4 b = *reinterpret_cast<const u32x4*>(base + (size_t)(r + 4) * ldx);
      u32x4 c = *reinterpret_cast<const u32x4*>(base + (size_t)(r + 8) * ldx);
      u32x4 d = *reinterpret_cast<const u32x4*>(base + (size_t)(r + 12) * ldx);
      float va[8], vb[8], vc[8], vd[8];
      unpack8(a, va);
      unpack8(b, vb);
      unpack8(c, vc);
      unpack8(d, vd);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += ((va[e] + vb[e]) + (vc[e] + vd[e]));
    }
    for (; r < r1; r += 4) {
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(base + (size_t)r * ldx), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wave - 1][lane][e] = acc[e];
  }
  __syncthreads();
  if (wave == 0 && active) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = ((acc[e] + red[0][lane][e]) + red[1][lane][e]) + red[2][lane][e];
    float4* dst = reinterpret_cast<float4*>(part + (size_t)blockIdx.y * N + (size_t)chunk * 8);
    dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// y[g][col] = sum of rows 32g .. min(R, 32g + 32) of part[R][N] (in order); grid (ceil(N/256), ceil(R/32))
__global__ __launch_bounds__(256) void colsum_rows32_kernel(const float* __restrict__ part, int R, int N,
                                                            float* __restrict__ y) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  const int r0 = blockIdx.y * 32, n = min(32, R - r0);
  const float* src = part + (size_t)r0 * N + col;
  float v[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) v[r] = r < n ? src[(size_t)r * N] : 0.f;
#pragma unroll
  for (int w = 16; w > 0; w >>= 1)
#pragma unroll
    for (int r = 0; r < w; ++r) v[r] += v[r + w];  // fixed pairwise tree
  y[(size_t)blockIdx.y * N + col] = v[0];
}

extern "C" size_t vst_colsum_workspace_bytes(int M, int N) {
  if (M <= 0 || N <= 0) return 0;
  const ColsumPlan p = colsum_plan(M, N);
  return ((size_t)p.R + p.R2) * N * sizeof(float);
}

extern "C" int vst_colsum(const void* x, int ldx, int M, int N, float* y, void* workspace, void* stream) {
  if (!x || !y || !workspace || M <= 0 || N <= 0 || N % 8 || (ldx & 7) || ldx < N || ((uintptr_t)x & 15))
    return VST_ERR_ARG;  // 16-B vector loads of 8-column chunks
  const ColsumPlan p = colsum_plan(M, N);
  hipStream_t s = (hipStream_t)stream;
  float* part1 = (float*)workspace;
  float* part2 = part1 + (size_t)p.R * N;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(p.gx, p.R), dim3(256), 0, s, (const bf16_t*)x, ldx, M, N,
                     p.rows_per_blk, part1);
  hipLaunchKernelGGL(colsum_rows32_kernel, dim3((N + 255) / 256, p.R2), dim3(256), 0, s, (const float*)part1, p.R, N,
                     part2);
  hipLaunchKernelGGL(colsum_rows32_kernel, dim3((N + 255) / 256, 1), dim3(256), 0, s, (const float*)part2, p.R2, N, y);
  return ok();
}
