// Shared GEMM tile epilogue (gemm_big.hip ring kernel, gemm_p8.hip 8-phase kernel): bias (+GELU), the bf16 tile
// staged once in LDS, then per-frame row bias / residual add (after that rounding, as the reference's separate add
// does) or GEGLU, written as full 16-B chunks.  acc[i][j][r] = C[m0 + wr*WM + i*16 + (lane&15)][n0 + wc*WN + j*16 +
// 4*(lane>>4) + r] (the W fragment is the MFMA's A operand).
#pragma once
#include "gemm_common.h"

namespace vst {

// Tile row (relative to the wave row's first row) of accumulator row block i.  ROT (the 8-phase kernel's in-GEMM
// LoRA variants): wave column wc reads the row blocks of each A quadrant rotated by wc, so block i of quadrant
// i / MQR is ((i mod MQR) + wc) mod MQR (MQR = MI / 2 blocks per quadrant, a power of two there).
template <class Cfg, bool ROT>
__device__ __forceinline__ int p8_acc_row(const int i, const int wc) {
  if constexpr (!ROT) {
    return i * 16;
  } else {
    constexpr int MQR = Cfg::MI / 2;
    static_assert((MQR & (MQR - 1)) == 0, "rotated row blocks: MQR a power of two");
    return (i / MQR) * (MQR * 16) + (((i % MQR) + wc) & (MQR - 1)) * 16;
  }
}

template <class Cfg, int EPI, bool ROT = false, bool CS_OK = false>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& p, char* smem, const int m0, const int n0,
                                              f32x4 (&acc)[Cfg::MI][Cfg::NJ], const int wr, const int wc,
                                              const int tid = threadIdx.x) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN;
  const int lane = tid & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow0 = wr * Cfg::WM + fr;          // + i*16
  const int lcol0 = wc * Cfg::WN + 4 * fq;      // + j*16
  constexpr int LROW = BN * 2 + 16;  // staged bf16 row (16-B pad: conflict-light b64 writes)
  static_assert(BM * LROW <= Cfg::LDS, "epilogue staging must fit in the ring's LDS");
  constexpr int CPR = BN / 8;  // 16-B output chunks per row
  constexpr int TOT = BM * CPR;
  constexpr int ITEMS = (TOT + Cfg::THREADS - 1) / Cfg::THREADS;
  const auto rr = make_rsrc(p.R ? p.R : p.Wt, p.R ? p.r_bytes : 0u);
  // GroupNorm column statistics (128x320 conv tiles, p.colstat; gn_colstat_kernel restates the same arithmetic):
  // the store pass then maps thread t to one 8-channel column (t mod 40) and rows t / 40 + 12 j, sums the stored bf16
  // values and their squares in registers (fixed order), and the 12 row groups are added in order through the LDS.
  // Compiled in only where the caller can ask for it (CS_OK: the 8-phase conv kernels), so the 128x320 projection and
  // in-GEMM LoRA epilogues keep their 10 store items and no runtime branch.
  constexpr bool CSTAT = CS_OK && EPI == 0 && BM == 128 && BN == 320;
  constexpr int CS_RG = Cfg::THREADS / CPR, CS_RPT = (BM + CS_RG - 1) / CS_RG;  // 12 row groups, 11 rows each
  constexpr int NIT = CSTAT && CS_RPT > ITEMS ? CS_RPT : ITEMS;
  const bool cs = CSTAT && p.colstat;
  // store-pass item k -> (tile row, 16-B chunk); false past the tile
  auto item = [&](int k, int& row, int& cc) {
    if (CSTAT && cs) {
      cc = tid % CPR;
      row = tid / CPR + CS_RG * k;
      return tid / CPR < CS_RG && row < BM;
    }
    const int idx = tid + k * Cfg::THREADS;
    row = idx / CPR;
    cc = idx - row * CPR;
    return k < ITEMS && idx < TOT;
  };
  // residual chunks are fetched first (the fragment registers are dead now): their HBM latency
  // overlaps the bias add and the LDS staging below instead of stalling the store pass.
  u32x4 res[EPI == 0 ? NIT : 1];
  if (EPI == 0 && p.R) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      int row, cc;
      const bool ok = item(k, row, cc);
      const int n = n0 + cc * 8, m = m0 + row;
      res[k] = buf_load16(rr, (ok && m < p.M && n + 8 <= p.N) ? (m * p.ldr + n) * 2 : kOOB);
    }
  }
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) {
      const int n = n0 + lcol0 + j * 16;
      f32x4 b4;
      if (n + 4 <= p.N) {
        b4 = *reinterpret_cast<const f32x4*>(p.bias + n);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = n + e < p.N ? p.bias[n + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i) acc[i][j] += b4;
    }
  }
  if constexpr (EPI == 1 && Cfg::WN == 64 && Cfg::NJ == 4) {
    // GEGLU from the registers: a wave's 64 weight rows are one [32 hidden | 32 gate] block, so lane-wise
    // acc[i][j] (j = 0, 1) is the hidden half and acc[i][j + 2] the gate of the same output column.  Both are
    // rounded to bf16 first (the reference's projection output), then h * gelu(g) is rounded once, as the LDS path
    // below does; only the 32-column outputs are staged (half the tile) for full-row stores.
    constexpr int OC = BN / 2;            // output columns of the tile
    constexpr int OROW = OC * 2 + 16;     // staged bf16 output row
    static_assert(BM * OROW <= Cfg::LDS, "GEGLU staging must fit in the ring's LDS");
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        u32x2 v;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t hp = pack2bf(acc[i][j][2 * e], acc[i][j][2 * e + 1]);
          const uint32_t gp = pack2bf(acc[i][j + 2][2 * e], acc[i][j + 2][2 * e + 1]);
          const f32x2 h = {__uint_as_float(hp << 16), __uint_as_float(hp & 0xffff0000u)};
          const f32x2 g = {__uint_as_float(gp << 16), __uint_as_float(gp & 0xffff0000u)};
#ifdef VST_ABL_NOGELU  // diagnostics build only (tools/p8_epi_ablate.sh): the GELU's VALU cost
          const f32x2 o = h * g;
#else
          const f32x2 o = geglu2(h, g);
#endif
          v[e] = pack2bf(o.x, o.y);
        }
        *reinterpret_cast<u32x2*>(smem + (lrow0 + p8_acc_row<Cfg, ROT>(i, wc)) * OROW + (wc * 32 + j * 16 + 4 * fq) * 2) = v;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    constexpr int OCPR = OC / 8;
    constexpr int OTOT = BM * OCPR;
    constexpr int OITEMS = (OTOT + Cfg::THREADS - 1) / Cfg::THREADS;
    const int nout = p.N / 2, c0 = n0 / 2;
#pragma unroll
    for (int k = 0; k < OITEMS; ++k) {
      const int idx = tid + k * Cfg::THREADS;
      const int row = idx / OCPR, cc = idx - row * OCPR;
      const int m = m0 + row, n = c0 + cc * 8;
      if (idx >= OTOT || m >= p.M || n >= nout) continue;
      *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + n) =
          *reinterpret_cast<const u32x4*>(smem + row * OROW + cc * 16);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) {
      f32x4 a4 = acc[i][j];
      if constexpr (EPI == 3) {  // GELU(erf) of the biased fp32 accumulator, before the bf16 rounding
#pragma unroll
        for (int e = 0; e < 4; ++e) a4[e] = gelu_erf(a4[e]);
      }
      u32x2 v;
      v[0] = pack2bf(a4[0], a4[1]);
      v[1] = pack2bf(a4[2], a4[3]);
      *reinterpret_cast<u32x2*>(smem + (lrow0 + p8_acc_row<Cfg, ROT>(i, wc)) * LROW + (lcol0 + j * 16) * 2) = v;
    }
  // publish the staged tile; a raw barrier (no vmcnt drain) keeps the residual loads in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (EPI == 0 || EPI == 3) {
    float csa[CSTAT ? 8 : 1], csq[CSTAT ? 8 : 1];
    if constexpr (CSTAT) {
#pragma unroll
      for (int e = 0; e < 8; ++e) csa[e] = csq[e] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      int row, cc;
      const bool ok = item(k, row, cc);
      const int m = m0 + row, n = n0 + cc * 8;
      const int nv = min(8, p.N - n);
      if (!ok || m >= p.M || nv <= 0) continue;
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(smem + row * LROW + cc * 16), v);
      if (EPI == 0 && p.rbias) {
        const float* rb = p.rbias + (size_t)(m / p.rbias_div) * p.ldrb + n;
        if (nv == 8) {
          const f32x4 r0 = *reinterpret_cast<const f32x4*>(rb);
          const f32x4 r1 = *reinterpret_cast<const f32x4*>(rb + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] += r0[e]; v[e + 4] += r1[e]; }
        } else {
          for (int e = 0; e < nv; ++e) v[e] += rb[e];
        }
      }
      if (nv == 8) {
        if (EPI == 0 && p.R) {
          float r8[8];
          unpack8(res[k], r8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += r8[e];
        }
        const u32x4 w = pack8(v);
        *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + n) = w;
        if (CSTAT && cs) {  // the stored bits
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = __uint_as_float(w[e] << 16), hi = __uint_as_float(w[e] & 0xffff0000u);
            csa[2 * e] += lo;
            csq[2 * e] = fmaf(lo, lo, csq[2 * e]);
            csa[2 * e + 1] += hi;
            csq[2 * e + 1] = fmaf(hi, hi, csq[2 * e + 1]);
          }
        }
      } else {
        for (int e = 0; e < nv; ++e) {
          float x = v[e];
          if (EPI == 0 && p.R) x += bf2f(p.R[(size_t)m * p.ldr + n + e]);
          p.C[(size_t)m * p.ldc + n + e] = f2bf(x);
        }
      }
    }
    if constexpr (CSTAT) {
      if (cs) {
        float* part = reinterpret_cast<float*>(smem);  // [CS_RG][BN][2], over the staged tile once every wave read it
        static_assert(CS_RG * BN * 8 <= BM * LROW, "column partials over the staged tile");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int cc = tid % CPR, rg = tid / CPR;
        if (rg < CS_RG) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            *reinterpret_cast<f32x2*>(part + (rg * BN + cc * 8 + e) * 2) = f32x2{csa[e], csq[e]};
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (tid < BN && n0 + tid < p.N) {
          f32x2 t = *reinterpret_cast<const f32x2*>(part + tid * 2);
#pragma unroll
          for (int g = 1; g < CS_RG; ++g) t += *reinterpret_cast<const f32x2*>(part + (g * BN + tid) * 2);
          *reinterpret_cast<f32x2*>(p.colstat + ((size_t)(m0 / BM) * p.N + n0 + tid) * 2) = t;
        }
      }
    }
  } else {  // GEGLU: per 64 weight rows [32 hidden | 32 gate] -> 32 outputs, bias already in
    constexpr int GPR = BN / 16;                // 8-output chunks per row
    constexpr int RSTEP = Cfg::THREADS / GPR;
    constexpr int GITEMS = BM / RSTEP;
    static_assert(Cfg::THREADS % GPR == 0 && BM % RSTEP == 0, "item split");
    const int oc = tid % GPR, row0 = tid / GPR;
    const int blk = oc >> 2, c = (oc & 3) * 8;
    const int nh = n0 + blk * 64 + c;
#pragma unroll
    for (int k = 0; k < GITEMS; ++k) {
      const int row = row0 + k * RSTEP, m = m0 + row;
      if (m >= p.M || nh >= p.N) continue;
      float h[8], g[8], v[8];
      unpack8(*reinterpret_cast<const u32x4*>(smem + row * LROW + (blk * 64 + c) * 2), h);
      unpack8(*reinterpret_cast<const u32x4*>(smem + row * LROW + (blk * 64 + 32 + c) * 2), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = h[e] * gelu_erf(g[e]);
      *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + (n0 >> 1) + blk * 32 + c) = pack8(v);
    }
  }
}

}  // namespace vst
