// 8-phase 256x256x64 GEMM (projections / GEGLU FF of the denoise path; same GemmArgs contract and epilogues as the
// ring kernel in gemm_big.hip, AMODE 0 only: A = [A1 | A2] split at K1, W row-major [N][K]).
//
// Why: the ring kernel runs 32-deep k-steps with two barriers per 32 MFMAs per wave; its MFMA + barrier skeleton
// alone reaches ~60 % of peak.  This kernel takes 64-deep k-tiles, two LDS buffers, and splits each
// buffer into four half-tile SLOTS so a slot is refilled as soon as its last reader is done, which keeps every
// operand byte ~6 phases (≈1.5 k-tiles) ahead of its use with 128 KiB of LDS:
//   slot Amq0 = A rows {0-63, 128-191}   (the first 64-row quadrant of both wave rows)
//   slot Amq1 = A rows {64-127, 192-255}
//   slot Bnq0 = W rows {wc*64 + 0..31}   (the first 32 output columns of every wave column)
//   slot Bnq1 = W rows {wc*64 + 32..63}
// each [128 rows][64 k] bf16, 128-B rows, 16-B chunk c of row r at (c ^ ((r >> 1) & 7)) (conflict-free
// ds_read_b128 fragment reads), filled by `buffer_load ... lds` (16 B per lane, lane-linear 1-KiB pieces, the
// inverse permutation applied to the source address).
//
// 8 waves = 2 (M) x 4 (N), wave tile 128 x 64 = 8 x 4 accumulators (16x16).  A k-tile is three barrier intervals
// over the quadrants Q(mq, nq) of the wave tile (16 MFMAs of 16x16x32 per quadrant):
//   I0: read A(mq0) + B(nq0), Q(0,0) + Q(0,1)      I1: read A(mq1), Q(1,1)      I2: read B(nq1) of t+1, Q(1,0)
// Each interval = {fragment reads, counted vmcnt wait, LDS-DMA issue} barrier {MFMAs} barrier; waves 4-7 run one
// barrier behind waves 0-3, so on every SIMD one wave's MFMAs overlap its partner's reads and DMA issue.
// A slot is refilled two intervals after the one that reads it (every wave's reads retired: WAR) and waited for
// (counted s_waitcnt vmcnt, 2 DMAs per slot per wave) in the interval before its first read (RAW).  Past the last
// k-tile the same DMAs are issued with out-of-range offsets (zeros), so the counts are the same in every interval;
// they are drained before the epilogue reuses the LDS.
#include "attn_common.h"
#include "gemm_common.h"
#include "gemm_epilogue.h"

#include <type_traits>

namespace vst {

// BM x BN tiles, 8 waves as 2 (M) x 4 (N), wave tile WM x WN = BM/2 x BN/4:
//   256 x 256 (128 x 64), 256 x 192 (128 x 48: the N = 1280 / 640 / 320 grids in fewer-padded, fuller rounds), and
//   128 x 320 (64 x 80: every SDXL width is a multiple of 320, so N = 320 / 640 / 1280 / 1920 / 3840 split without
//   padding and M = 8192 gives exactly one full round of 256 tiles on 256 CUs).
// Slot A0 / A1 hold the first / second half of every wave row's WM rows; slot B0 the first 32 columns of every wave
// column, B1 the remaining WN - 32 (32, 16 or 48).
template <int BN_, int BM_ = 256>
struct P8Cfg {  // the epilogue's view of the tile (same wave tiling as RingCfg<BM, BN, 2, 4, S>)
  static constexpr int BM = BM_, BN = BN_, WAVES_M = 2, WAVES_N = 4, NWAVES = 8, THREADS = 512;
  static constexpr int WM = BM / 2, WN = BN / 4, MI = WM / 16, NJ = WN / 16;
  static constexpr int HALF = WM / 2;               // rows of a wave row in one A slot
  static constexpr int MQR = HALF / 16;             // 16-row blocks per A quadrant (4 or 2)
  static constexpr int NPA = BM / 128;              // A slot 1-KiB pieces per wave (2 or 1)
  static constexpr int RB1 = WN - 32;               // B1 rows per wave column
  static constexpr int NJ1 = RB1 / 16;              // B1 fragments per wave
  static constexpr int NPB1 = 4 * RB1 / 64;         // B1 1-KiB pieces per wave (2, 1 or 3)
  static constexpr int SLOT_A = BM / 2 * 128;       // A0, A1
  static constexpr int SLOT_B0 = 128 * 128;         // B0: 4 wave columns x 32 rows
  static constexpr int SLOT_B1 = 4 * RB1 * 128;     // B1
  static constexpr int BUF = 2 * SLOT_A + SLOT_B0 + SLOT_B1;
  static constexpr int EPI_BYTES = BM * (BN * 2 + 16);
  static constexpr int LDS = 2 * BUF > EPI_BYTES ? 2 * BUF : EPI_BYTES;
  // LORA: two 2-KiB Acat slots ([16 u columns][64 k] per k-tile) + 1 KiB sink for the waves without a piece, then
  // the tile's up-projection columns V [BN rows][16] (32-B rows), staged once in the prologue
  static constexpr int LORA_OFF = 2 * BUF, V_OFF = 2 * BUF + 5 * 1024, LORA_END = V_OFF + BN * 32;
  static constexpr int LDS_LORA = LORA_END > EPI_BYTES ? LORA_END : EPI_BYTES;
  // PERSIST: the epilogue stages through the LDS past the ring (the ring holds the next tile's first k-tiles)
  static constexpr int EPI_OFF = 2 * BUF, EPI_REGION = 160 * 1024 - 2 * BUF;
  // PERSIST + LORA (128x320 tiles): u exchanged at U_OFF past V; the epilogue stages over V and U (both dead once the
  // tile's u . V step is done), never over the Acat slots, which hold the next tile's first two k-tiles by then
  static constexpr int U_OFF = LORA_END, U_END = U_OFF + BM * 32;
  static constexpr int EPI_OFF_L = V_OFF, EPI_REGION_L = 160 * 1024 - V_OFF;
  static_assert((BM == 256 && (BN == 256 || BN == 192)) || (BM == 128 && BN == 320), "tile shape");
  static_assert(LDS <= 160 * 1024 && LDS_LORA <= 160 * 1024, "LDS budget");
};

template <int N>
__device__ __forceinline__ void p8_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

typedef __attribute__((address_space(3))) void p8_lds_void;

#ifdef VST_P8_TRACE
// diagnostics build only (tools/p8_trace.py): per-workgroup wall-clock (100 MHz) and shader-clock stamps at
// kernel entry, first operands landed, k-loop done, epilogue done
__device__ unsigned long long vst_p8_trace_buf[8192 * 8];
#define VST_P8_STAMP(I)                                                                    \
  if (threadIdx.x == 0 && blockIdx.x < 8192) {                                             \
    vst_p8_trace_buf[blockIdx.x * 8 + 2 * (I)] = __builtin_amdgcn_s_memrealtime();         \
    vst_p8_trace_buf[blockIdx.x * 8 + 2 * (I) + 1] = __builtin_readcyclecounter();         \
  }
#else
#define VST_P8_STAMP(I)
#endif

__device__ __forceinline__ void p8_dma16(__amdgpu_buffer_rsrc_t r, char* lds_piece, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (p8_lds_void*)((__attribute__((address_space(3))) char*)(uintptr_t)lds_piece), 16, off, 0, 0, 0);
}

__device__ __forceinline__ int p8_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// scheduling hint for an MFMA segment that also issues NV LDS-DMAs (VMEM) among its NM MFMAs: one DMA after every
// NM / (NV + 1) MFMAs, the rest of the MFMAs after the last one
template <int NM, int NV>
__device__ __forceinline__ void p8_interleave_dma() {
  constexpr int PER = NM / (NV + 1) > 0 ? NM / (NV + 1) : 1;
#pragma unroll
  for (int g = 0; g < NV; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);    // VMEM read (buffer_load ... lds)
  }
  __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
}

__device__ __forceinline__ void p8_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// EPI 4: cross-attention over the text tokens as the epilogue of the attn2 q projection (BasicTransformerBlock,
// unziplora_unet/unzip_attention.py:188-212; the SDPA core of AnimateDiffAttnProcessor2_0,
// animatediff/attention_processor.py:78-80).  A 256-row tile lies inside one frame (HW % 256 == 0) and its 192
// columns are 3 heads of 64, so the tile holds every query of those (frame, head) pairs: the q tile is staged once
// in LDS as bf16 (the reference's rounding point of to_q's output), the heads' K/V (<= 80 text keys each, zero rows
// past Nk) are brought in by LDS-DMA, and each wave computes 32 queries x 3 heads of softmax(q K^T / 8) V with
// S^T = K.Q^T and O^T = V^T.P^T on MFMA (the spatial_attn_kernel layouts, one pass over all keys).  q is never
// written to HBM and read back, and the separate attention launch disappears.  LDS: 256 x 400 B of q + 3 x 20 KiB of
// K/V = 160 KiB exactly.
template <class Cfg, bool ROT>
__device__ __forceinline__ void xattn_epilogue(const GemmArgs& p, char* smem, const int m0, const int n0,
                                               f32x4 (&acc)[Cfg::MI][Cfg::NJ], const int wr, const int wc) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN, NH = BN / 64;
  constexpr int LROW = BN * 2 + 16;
  constexpr int KVH = 80 * 128;  // one operand of one head: [80 keys][64 d] bf16, 128-B rows
  constexpr int KV_OFF = BM * LROW;
  static_assert(BN == 192 && KV_OFF + NH * 2 * KVH <= 160 * 1024, "q tile + 3 heads of K/V in 160 KiB");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int bkv = __builtin_amdgcn_readfirstlane((m0 / p.xa_nq) / p.xa_kvdiv);
  const int h0 = n0 / 64, nh = min(NH, (p.N - n0) / 64);
  // K/V pieces first (their latency overlaps the q staging): 20 per head (10 x 8 rows of K, then of V), the tile
  // swizzles k_off / v_off applied to the source chunk (the DMA writes lane-linearly); keys >= Nk read as zeros
  {
    const auto rk = make_rsrc(p.xa_k, p.xa_kv_bytes), rv = make_rsrc(p.xa_v, p.xa_kv_bytes);
    for (int pc = wid; pc < NH * 20; pc += 8) {
      const int hh = pc / 20, q = pc - hh * 20, op = q / 10, r8 = q - op * 10;
      const int row = r8 * 8 + (lane >> 3), slot = lane & 7;
      const int c = op == 0 ? slot ^ ((row >> 1) & 7) : slot ^ (((row >> 1) & 3) << 1);
      const bool ok = hh < nh && row < p.xa_nk;
      const int off = ok ? ((bkv * p.xa_nk + row) * p.xa_ldkv + (h0 + hh) * 64 + c * 8) * 2 : kOOB;
      char* dst = smem + KV_OFF + hh * 2 * KVH + op * KVH + r8 * 1024;
      if (op == 0) p8_dma16(rk, dst, off); else p8_dma16(rv, dst, off);
    }
  }
  // q (+ bias) -> bf16 tile [256][BN] in LDS
  {
    const int lrow0 = wr * Cfg::WM + fr, lcol0 = wc * Cfg::WN + 4 * fq;
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) {
      f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
        const int n = n0 + lcol0 + j * 16;
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = n + e < p.N ? p.bias[n + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i) {
        const f32x4 a4 = acc[i][j] + b4;
        u32x2 v;
        v[0] = pack2bf(a4[0], a4[1]);
        v[1] = pack2bf(a4[2], a4[3]);
        *reinterpret_cast<u32x2*>(smem + (lrow0 + p8_acc_row<Cfg, ROT>(i, wc)) * LROW + (lcol0 + j * 16) * 2) = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // wave w: queries [32 w, 32 w + 32) of the tile, every head of it
  const float sl2 = p.xa_scale_log2;
  const int qbase = 32 * wid;
  int voff[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    const int r0 = fq * 4 + (fr >> 2), col = db * 16 + (fr & 3) * 4;
    voff[db] = v_off(r0, col >> 3) + (col & 7) * 2;
  }
  for (int hh = 0; hh < nh; ++hh) {
    const char* Ks = smem + KV_OFF + hh * 2 * KVH;
    const char* Vs = Ks + KVH;
    bf16x8 qf[2][2];  // Q^T fragments: lane (q, g) holds Q[q][32 kk + 8 g .. +7]
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        qf[qb][kk] = *reinterpret_cast<const bf16x8*>(smem + (qbase + qb * 16 + fr) * LROW + (hh * 64 + kk * 32 + fq * 8) * 2);
    f32x4 s[5][2];  // S^T: lane col q, rows key = 16 kt + 4 g + i
#pragma unroll
    for (int kt = 0; kt < 5; ++kt) {
      bf16x8 kf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) kf[kk] = *reinterpret_cast<const bf16x8*>(Ks + k_off(kt * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 a{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[0], qf[qb][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[1], qf[qb][1], a, 0, 0, 0);
        s[kt][qb] = a;
      }
    }
    // softmax in the standalone kernel's order (spatial_attn_kernel, PRE tiles of 64 keys): keys 0-63 with their own
    // max, then keys 64-79 with an online rescale, P rounded to bf16 unnormalised, 1/l at the end -- the same bf16
    // roundings as the two-launch path, so the fused and unfused attn2 agree to fp32 summation order
    float m0r[2], lrun[2], alpha[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (kt * 16 + fq * 4 + i >= p.xa_nk) s[kt][qb][i] = -INFINITY;
          mx = fmaxf(mx, s[kt][qb][i]);
        }
      mx = group_max(mx);
      m0r[qb] = mx;
      const float mb = mx * sl2;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = fast_exp2(s[kt][qb][i] * sl2 - mb);
          s[kt][qb][i] = pv;
          ls += pv;
        }
      lrun[qb] = ls;
      // second key tile (64-79 live): its max, the rescale of the first tile's state, its P
      float mx1 = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (64 + fq * 4 + i >= p.xa_nk) s[4][qb][i] = -INFINITY;
        mx1 = fmaxf(mx1, s[4][qb][i]);
      }
      mx1 = group_max(mx1);
      const float mnew = fmaxf(mx, mx1);
      alpha[qb] = fast_exp2((mx - mnew) * sl2);
      const float mb1 = mnew * sl2;
      float ls1 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = fast_exp2(s[4][qb][i] * sl2 - mb1);
        s[4][qb][i] = pv;
        ls1 += pv;
      }
      lrun[qb] = lrun[qb] * alpha[qb] + ls1;
    }
    (void)m0r;
    // O^T = V^T P^T: keys 0-31 and 32-63 as two 32-deep steps (P blocks 2 st, 2 st + 1), rescaled by alpha, then
    // keys 64-79 as one 16-deep step
    f32x4 o[4][2];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) o[db][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        pf[qb] = pack_p8(s[2 * st][qb][0], s[2 * st][qb][1], s[2 * st][qb][2], s[2 * st][qb][3], s[2 * st + 1][qb][0],
                         s[2 * st + 1][qb][1], s[2 * st + 1][qb][2], s[2 * st + 1][qb][3]);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8 vf = cat_tr(ds_read_tr(Vs + voff[db] + st * 4096), ds_read_tr(Vs + voff[db] + st * 4096 + 2048));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qb], o[db][qb], 0, 0, 0);
      }
    }
    {
      s16x4 p4[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const u32x2 w{pack2bf(s[4][qb][0], s[4][qb][1]), pack2bf(s[4][qb][2], s[4][qb][3])};
        p4[qb] = __builtin_bit_cast(s16x4, w);
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db][qb] *= alpha[qb];
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const s16x4 vf = ds_read_tr(Vs + voff[db] + 2 * 4096);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, p4[qb], o[db][qb], 0, 0, 0);
      }
    }
    float inv[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float l = lrun[qb];
      l += __shfl_xor(l, 16);
      l += __shfl_xor(l, 32);
      inv[qb] = 1.0f / l;
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int m = m0 + qbase + qb * 16 + fr;
      if (m >= p.M) continue;
      bf16_t* orow = p.C + (size_t)m * p.ldc + n0 + hh * 64;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const f32x4 v = o[db][qb] * inv[qb];
        const u32x2 w{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
        *reinterpret_cast<u32x2*>(orow + db * 16 + fq * 4) = w;
      }
    }
  }
}

// PERSIST epilogue (EPI 0 bias / row bias / residual, 1 GEGLU, 3 bias + GELU): the same rounding points as
// tile_epilogue.  EPI 0 / 3 stage through the EPI_REGION bytes past the ring in passes of 32 * IPP tile rows (IPP
// 16-row accumulator blocks of both wave rows), so the ring's buffers keep the next tile's first k-tiles in flight;
// staged rows are unpadded, 16-B chunk c of staged row r at chunk c ^ (r & 7) (rows hold a multiple of 8 chunks).
// GEGLU stores its half-width output straight from the accumulators, as unconditional buffer stores (out-of-range
// chunks get out-of-range offsets), so every wave issues exactly p8_epi_stores<Cfg, EPI>() of them.  pre() runs after
// the bias add (the caller's next-tile DMAs, issued before any store).  GEGLU reads its bias from R, where the k-loop
// brought it by LDS-DMA.
template <class Cfg, int EPI, int REGION = Cfg::EPI_REGION>
constexpr int p8_epi_ipp() {  // 16-row accumulator blocks per staged pass (both wave rows)
  constexpr int ROWB = (EPI == 1 ? Cfg::BN / 2 : Cfg::BN) * 2, MI = Cfg::MI;
  return (MI >= 8 && 256 * ROWB <= REGION) ? 8
         : (MI >= 4 && 128 * ROWB <= REGION) ? 4
         : (MI >= 2 && 64 * ROWB <= REGION) ? 2 : 1;
}
template <class Cfg, int EPI, int REGION = Cfg::EPI_REGION>
constexpr int p8_epi_items() {  // 16-B output chunks per thread per staged pass
  return 32 * p8_epi_ipp<Cfg, EPI, REGION>() * ((EPI == 1 ? Cfg::BN / 2 : Cfg::BN) / 8) / Cfg::THREADS;
}
template <class Cfg, int EPI, int REGION = Cfg::EPI_REGION>
constexpr int p8_epi_stores() {
#ifdef VST_ABL_NOEPI
  return 0;
#else
  return EPI == 1 ? 2 * Cfg::MI : p8_epi_items<Cfg, EPI, REGION>() * (Cfg::MI / p8_epi_ipp<Cfg, EPI, REGION>());
#endif
}

// ROT (the in-GEMM LoRA kernels): acc[mq MQR + i] holds row block (i + wc) mod MQR of quadrant mq (p8_acc_row), so a
// pass stages whole quadrants (IPP == MQR) and each wave writes its blocks at their rotated rows.
template <class Cfg, int EPI, int REGION = Cfg::EPI_REGION, bool ROT = false, class Pre>
__device__ __forceinline__ void p8_epilogue_passes(const GemmArgs& p, char* R, const int m0, const int n0,
                                                   f32x4 (&acc)[Cfg::MI][Cfg::NJ], const int wr, const int wc,
                                                   Pre&& pre) {
  constexpr int MI = Cfg::MI, NJ = Cfg::NJ, WM = Cfg::WM, THREADS = Cfg::THREADS;
  constexpr int OC = EPI == 1 ? Cfg::BN / 2 : Cfg::BN;  // output columns of the tile
  constexpr int ROWB = OC * 2;
  constexpr int IPP = p8_epi_ipp<Cfg, EPI, REGION>();
  constexpr int PR = 32 * IPP, NPASS = MI / IPP, CPR = OC / 8, ITEMS = PR * CPR / THREADS;
  static_assert(ITEMS == p8_epi_items<Cfg, EPI, REGION>(), "store count");
  static_assert(!ROT || IPP == Cfg::MQR, "rotated row blocks: one quadrant per pass");
  static_assert(PR * ROWB <= REGION && (PR * CPR) % THREADS == 0 && CPR % 8 == 0 && MI % IPP == 0, "pass split");
  static_assert(EPI != 1 || (Cfg::WN == 64 && NJ == 4), "GEGLU: [32 hidden | 32 gate] per wave column");
  const int tid = threadIdx.x, lane = tid & 63, fr = lane & 15, fq = lane >> 4;
  const int lcol0 = wc * Cfg::WN + 4 * fq;
  auto swz = [](int lr, int byte) { return lr * ROWB + (((byte >> 4) ^ (lr & 7)) << 4) + (byte & 15); };
  if (EPI == 1 && p.bias) {  // (the k-loop's LDS-DMA put the tile's bias at R: no global load waits here)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(R + (lcol0 + j * 16) * 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[i][j] += b4;
    }
  } else if (p.bias) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + lcol0 + j * 16;
      f32x4 b4;
      if (n + 4 <= p.N) {
        b4 = *reinterpret_cast<const f32x4*>(p.bias + n);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = n + e < p.N ? p.bias[n + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[i][j] += b4;
    }
  }
  pre();
  const auto rr = make_rsrc(p.R ? p.R : p.Wt, p.R ? p.r_bytes : 0u);
  const auto rc = make_rsrc(p.C, (uint32_t)((size_t)p.M * p.ldc * 2));  // (launch_p8_epi: < 2^31 bytes)
  const int nout = EPI == 1 ? p.N / 2 : p.N, c0 = EPI == 1 ? n0 / 2 : n0;
  if constexpr (EPI == 1) {
    // GEGLU: no staging -- each lane's 4 output columns (8 B) of its 16-row blocks go straight out (the 64-B row
    // segments of a wave column merge in L2; staged through the LDS in passes measured 0.15 ms per step slower,
    // profiles/r4_ab_geglu_direct.txt)
    {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wr * WM + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x2 v;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t hp = pack2bf(acc[i][j][2 * e], acc[i][j][2 * e + 1]);
            const uint32_t gp = pack2bf(acc[i][j + 2][2 * e], acc[i][j + 2][2 * e + 1]);
            const f32x2 h = {__uint_as_float(hp << 16), __uint_as_float(hp & 0xffff0000u)};
            const f32x2 g = {__uint_as_float(gp << 16), __uint_as_float(gp & 0xffff0000u)};
            const f32x2 o = geglu2(h, g);
            v[e] = pack2bf(o.x, o.y);
          }
          const int n = c0 + wc * 32 + j * 16 + 4 * fq;
          __builtin_amdgcn_raw_buffer_store_b64(v, rc, m < p.M && n < nout ? (m * p.ldc + n) * 2 : kOOB, 0, 0);
        }
      }
      return;
    }
  } else {
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    // residual chunks of this pass first: their latency overlaps the staging
    u32x4 res[EPI == 0 ? ITEMS : 1];
    if (EPI == 0 && p.R) {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        const int idx = tid + k * THREADS, lr = idx / CPR, cc = idx - lr * CPR;
        const int row = (lr / (16 * IPP)) * WM + q * IPP * 16 + lr % (16 * IPP), m = m0 + row, n = n0 + cc * 8;
        res[k] = buf_load16(rr, (m < p.M && n + 8 <= p.N) ? (m * p.ldr + n) * 2 : kOOB);
      }
    }
#pragma unroll
    for (int ii = 0; ii < IPP; ++ii) {
      const int i = q * IPP + ii, lr = wr * 16 * IPP + (ROT ? ((ii + wc) & (Cfg::MQR - 1)) : ii) * 16 + fr;
      {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          f32x4 a4 = acc[i][j];
          if constexpr (EPI == 3) {
#pragma unroll
            for (int e = 0; e < 4; ++e) a4[e] = gelu_erf(a4[e]);
          }
          const u32x2 v{pack2bf(a4[0], a4[1]), pack2bf(a4[2], a4[3])};
          *reinterpret_cast<u32x2*>(R + swz(lr, (lcol0 + j * 16) * 2)) = v;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const int idx = tid + k * THREADS, lr = idx / CPR, cc = idx - lr * CPR;
      const int row = (lr / (16 * IPP)) * WM + q * IPP * 16 + lr % (16 * IPP), m = m0 + row, n = c0 + cc * 8;
      const bool ok = m < p.M && n < nout;  // (nout % 8 == 0: the launcher's condition)
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(R + swz(lr, cc * 16)), v);
      if constexpr (EPI == 0) {
        if (p.rbias && ok) {
          const float* rb = p.rbias + (size_t)(m / p.rbias_div) * p.ldrb + n;
          const f32x4 r0 = *reinterpret_cast<const f32x4*>(rb), r1 = *reinterpret_cast<const f32x4*>(rb + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] += r0[e]; v[e + 4] += r1[e]; }
        }
        if (p.R) {
          float r8[8];
          unpack8(res[k], r8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += r8[e];
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(pack8(v), rc, ok ? (m * p.ldc + n) * 2 : kOOB, 0, 0);
    }
    if (q + 1 < NPASS) {  // every wave's reads of this pass done before the next pass restages the region
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  }
}

// EPI 5: the motion modules' frame-axis self-attention as the epilogue of their fused q/k/v projection (AttnProcessor2_0
// on the AnimateDiffTransformer3D blocks: to_q / to_k / to_v, then F.scaled_dot_product_attention over the frames of
// every pixel; animatediff/temporal_transformer.py:40-71 restates the same attention).  The GEMM takes its rows in
// (clip, 16-pixel group, pixel, frame) order (setup_tile's row map), so a 256-row tile holds all 16 frames of 16
// pixels, and the host lays the weight rows out so a 256-column tile is [q k v] of 256 / (3 d) heads (two of 40 or
// one of 80; zero rows pad to 256).  (acc + bias) is rounded to bf16 into LDS (the projections' rounding point), then
// the waves compute the tile's (pixel, head) units on MFMA in temporal_attn_kernel's arithmetic: S^T = K Q^T (32-deep
// steps, d >= head_dim zeroed), softmax over the 16 keys (exp2, P rounded to bf16 unnormalised, 1/l at the end),
// O^T = V^T P^T (16x16x16 steps over 16-wide d blocks).  q / k / v never reach HBM: their write and the separate
// attention launch's read (2 x 252 MB per motion block at the 64^2 level of 16x512^2) are gone.
template <class Cfg>
__device__ __forceinline__ void tattn_epilogue(const GemmArgs& p, char* smem, const int m0, const int n0,
                                               f32x4 (&acc)[Cfg::MI][Cfg::NJ], const int wr, const int wc) {
  constexpr int LROW = Cfg::BN * 2 + 16, TF = 16;
  static_assert(Cfg::BM == 256 && Cfg::BN == 256 && Cfg::BM * LROW <= 160 * 1024, "256x256 tiles");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  {
    const int lrow0 = wr * Cfg::WM + fr, lcol0 = wc * Cfg::WN + 4 * g;
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) {
      f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
        const int n = n0 + lcol0 + j * 16;
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = n + e < p.N ? p.bias[n + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i) {
        const f32x4 a4 = acc[i][j] + b4;
        const u32x2 v{pack2bf(a4[0], a4[1]), pack2bf(a4[2], a4[3])};
        *reinterpret_cast<u32x2*>(smem + (lrow0 + i * 16) * LROW + (lcol0 + j * 16) * 2) = v;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const int TD = p.ta_d, HPT = 256 / (3 * TD), KS = (TD + 31) / 32, DB = (TD + 15) / 16;
  const int ngrp = p.ta_hw / 16, mt = m0 / 256;
  const int b = mt / ngrp, pg = mt - b * ngrp;
  const float sl2 = p.ta_scale_log2;
  for (int u = wid; u < 16 * HPT; u += 8) {
    const int pl = u / HPT, hh = u - pl * HPT, h = (n0 / 256) * HPT + hh;
    if (h >= p.ta_heads) continue;  // (wave-uniform)
    const char* R = smem + pl * TF * LROW;  // the 16 frame rows of pixel pl
    const int cq = hh * 3 * TD, ck = cq + TD, cv = cq + 2 * TD;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};  // S^T: lane (query fr) holds keys 4g + i
    for (int kk = 0; kk < KS; ++kk) {
      const int d0 = kk * 32 + g * 8;
      bf16x8 kf = bf16x8{}, qf = bf16x8{};
      if (d0 < TD) {
        kf = *reinterpret_cast<const bf16x8*>(R + fr * LROW + (ck + d0) * 2);
        qf = *reinterpret_cast<const bf16x8*>(R + fr * LROW + (cq + d0) * 2);
      }
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, s, 0, 0, 0);
    }
    float mx = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mb = mx * sl2;
    float ls = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[i] = fast_exp2(s[i] * sl2 - mb);
      ls += s[i];
    }
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    const float inv = 1.0f / ls;
    const u32x2 pw{pack2bf(s[0], s[1]), pack2bf(s[2], s[3])};
    const s16x4 pb = __builtin_bit_cast(s16x4, pw);  // B = P^T: keys 4g .. 4g+3 of query fr
    bf16_t* orow = p.C + (size_t)((b * TF + fr) * p.ta_hw + pg * 16 + pl) * p.ldc + h * TD;
    for (int db = 0; db < DB; ++db) {
      const int d = db * 16 + fr;  // A = V^T: row d, keys 4g .. 4g+3
      s16x4 va = s16x4{0, 0, 0, 0};
      if (d < TD) {
#pragma unroll
        for (int i = 0; i < 4; ++i) va[i] = *reinterpret_cast<const short*>(R + (4 * g + i) * LROW + (cv + d) * 2);
      }
      const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0) * inv;
      // o[i] = O^T[d = 16 db + 4g + i][query fr]
      if (db * 16 + 4 * g < TD)
        *reinterpret_cast<u32x2*>(orow + db * 16 + 4 * g) = u32x2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
    }
  }
}

// LORA (vst_gemm_lora, UnZipLoRA / LoRA projections): the down-projection u = x . Acat^T is accumulated inside the
// k-loop from the A fragments already in registers, so no separate pass over x produces it.  Each k-tile also
// stages Acat's 16 u columns of this tile ([16][64] bf16, one extra DMA per wave issued with slot Amq0: waves 0-1
// move the two 1-KiB pieces, the others a zero piece into a sink, so every wave's vmcnt counts stay uniform); in I0
// and I1 every wave adds one 16-row block of u (row block wc of the current row quadrant: 2 MFMAs each).  After the
// loop u is rounded to bf16 (the reference's rounding point of lora_layer's down output), exchanged through LDS and
// multiplied by the tile's up-projection columns of W (K + ub0 ...) as one extra 16x16x32 step per accumulator —
// the same operands, in the same order, as the [x | u] . [W | V]^T k-tile it replaces.
// CONV: the A operand is the implicit im2col of an NHWC 3x3 conv (pad 1; stride 2, nearest-2x upsample, the VAE's
// (0,1,0,1) padding; x2 = the up path's skip concat), K ordered (tap, channel) with Ctot = C1 + C2 a multiple of 64,
// so a 64-deep k-tile is one tap of one source.  Each A slot's DMAs are issued for consecutive k-tiles, so a (tap,
// channel) cursor per slot advances by 64 per issue and its pieces' row bases are recomputed only when the tap or the
// source changes (padding rows read out of range: zeros).  Same k order as the ring kernel's conv: same bits.
template <int EPI, int BN, bool LORA = false, int PH = 3, int BM = 256, bool CONV = false, bool PERSIST = false>
__global__ __launch_bounds__(512, 1) void gemm_p8_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Cfg = P8Cfg<BN, BM>;
  static_assert(!CONV || (!LORA && EPI == 0), "conv: plain epilogue");
  static_assert(EPI != 1 || BN == 256, "GEGLU needs 64-column [hidden | gate] blocks");
  static_assert(!LORA || EPI != 1, "in-GEMM LoRA: linear epilogue");
  static_assert(!PERSIST || (!CONV && EPI != 4 && EPI != 5 && PH == 2 && (!LORA || (EPI == 0 && BN == 320))),
                "persistent tiles: plain / GEGLU / GELU, and the in-GEMM LoRA on 128x320 tiles; PH 2");
  static_assert(!(PERSIST && LORA) || Cfg::U_END <= 160 * 1024, "LoRA persistent LDS");
  static_assert(EPI != 5 || (BN == 256 && BM == 256 && !LORA && !CONV), "temporal attention epilogue: 256x256 tiles");
  static_assert(EPI != 4 || (BN == 192 && BM == 256), "cross-attention epilogue: 256 x 192 tiles (3 heads)");
  // LORA: the Acat DMA of a k-tile is issued by waves 0-1 only (one 1-KiB piece each), so their counted vmcnt waits
  // count it and the other waves' do not (VST_P8_VMWAIT_LX; rounds 3-4 had waves 2-7 DMA a zero piece into a sink
  // to keep one count: 6 extra LDS writes and DMA issues per k-tile)
#define VST_P8_VMWAIT_LX(X)                  \
  do {                                       \
    if (LORA && wid < 2) p8_vmwait<(X) + 1>(); \
    else p8_vmwait<(X)>();                   \
  } while (0)
  // one A source (the launchers of the persistent, LoRA, cross- and temporal-attention variants pass no A2): the
  // loader's per-k-tile source selection is compiled out
  constexpr bool ONE_A = PERSIST || LORA || EPI == 4 || EPI == 5;
  // DMM (A/B build VST_P8_DMM): a k-tile interval's LDS-DMAs issued inside the wave's MFMA segment, interleaved with
  // its MFMAs, instead of in its load segment after the fragment reads (an LDS-DMA costs its wave ~60 cycles among
  // bare MFMAs and 100-185 in a segment that carries 16 ds_read_b128, MI355X_MICROARCH.md constants table; the loop
  // ablations put the load segments, not the MFMAs, on the critical path).  Same DMAs in the same order per wave, so
  // every counted wait keeps its count; the slots they refill were read one interval earlier still.
  // Off: in isolation the LoRA kernels gained 1-2 % per launch with it and the plain GEMMs lost 1-22 %
  // (profiles/r5_ab_dma_in_mfma_negative.txt); on the LoRA kernels alone the whole step was 0.2 ms slower in two
  // alternations (profiles/r5_ab_dma_in_mfma_lora_negative.txt).  VST_P8_DMM builds it everywhere (A/B).
#if defined(VST_P8_DMM)
  constexpr bool DMM = true;
#else
  constexpr bool DMM = false;
#endif
#ifdef VST_P8_LORA_B1E  // (A/B build: the in-GEMM LoRA kernels with the B1 placement of the plain GEMMs)
  constexpr bool B1E = EPI != 1;
#else
  constexpr bool B1E = EPI != 1 && !LORA;  // PH = 2: B1 fragments read in J1's MFMA segment (run_segment2)
#endif
  constexpr int BUF = Cfg::BUF, RB1 = Cfg::RB1, NJ1 = Cfg::NJ1, NPB1 = Cfg::NPB1, NPA = Cfg::NPA;
  constexpr int HALF = Cfg::HALF, MQR = Cfg::MQR;
  // slot offsets inside a buffer: A0, A1, B0, B1
  auto slot_off = [](int s_) { return s_ < 2 ? s_ * Cfg::SLOT_A : (s_ == 2 ? 2 * Cfg::SLOT_A : 2 * Cfg::SLOT_A + Cfg::SLOT_B0); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int ntiles = nbm * nbn;
  // grouped order: GROUP_M row panels sweep N together (p.group_m: VST_GEMM_GROUP_M, A/B only; default 8)
  const int GROUP_M = p.group_m > 0 ? p.group_m : 8;
  auto tile_origin = [&](int t, int& m0, int& n0) {
    const int in_group = GROUP_M * nbn;
    const int gid = t / in_group, first_m = gid * GROUP_M;
    const int gsize = min(nbm - first_m, GROUP_M);
    m0 = (first_m + (t - gid * in_group) % gsize) * BM;
    n0 = ((t - gid * in_group) / gsize) * BN;
  };
  const auto ra1 = make_rsrc(p.A1, p.a1_bytes);
  const auto ra2 = make_rsrc(p.A2 ? p.A2 : p.A1, p.A2 ? p.a2_bytes : 0u);
  const auto rw = make_rsrc(p.Wt, p.w_bytes);
  const int nk = (p.K + 63) / 64;
  const bool ktail = !PERSIST && (p.K & 63) != 0;  // (PERSIST: K % 64 == 0 and one A source, the launcher's terms)
  const bool late = wid >= 4;
#ifdef VST_P8_TRACE
  // diagnostics build only (VST_GEMM_ABLATE): 1 no loop DMA, 2 no MFMA, 4 no loop vmcnt waits, 16 no fragment reads,
  // 64 no W-operand traffic in the loop (its DMAs and fragment reads; the upper bound of taking W out of the LDS),
  // 128 no A-operand traffic in the loop
  const int abl = p.ablate;
#else
  constexpr int abl = 0;
#endif

  // ---- per-lane DMA descriptors: slot s in {Amq0, Amq1, Bnq0, Bnq1}; 1-KiB piece q = PB + PS*pc of a slot holds slot
  //      rows 8q .. 8q+7 (row 8q + (lane >> 3)); this lane moves chunk c = (lane & 7) ^ ((row >> 1) & 7) of that row.
  constexpr int NPC = NPB1 > 2 ? NPB1 : 2, PS = 8;  // pieces per wave of the largest slot (B0: 2, B1: up to 3)
  const int PB = wid;
  uint32_t base1[4][NPC], base2[2][NPC];
  int c8[4][NPC];
  // CONV: output pixel (image, oy, ox) of each A piece's row; per-slot (tap, channel) cursor and source
  int cv_img[2][NPA], cv_oy[2][NPA], cv_ox[2][NPA];
  int cv_tap[2] = {0, 0}, cv_ci[2] = {0, 0}, cv_ci0[2] = {0, 0};
  bool cv_second[2] = {false, false}, cv_rebase[2] = {true, true};
  const int Ctot = p.C1 + p.C2;
  const auto rl = make_rsrc(LORA ? p.la : p.Wt, LORA ? p.la_bytes : 0u);
  int ub0 = 0, lc8 = 0;          // LORA: the tile's first u column (16-aligned); this lane's Acat chunk * 8
  uint32_t lbase = (uint32_t)kOOB;  // LORA: this lane's Acat source row / chunk (waves 0-1)
  int n0_tile = 0;
  // PERSIST: global index of the current tile's first k-tile (the LDS buffer of k-tile kt is (kofs + kt) & 1), and
  // the next tile of this workgroup, whose first two k-tiles are streamed in by the current tile's last two
  int kofs = 0, nm0 = 0, nn0 = 0;
  bool has_next = false;
  int bias_n0 = 0;  // PERSIST GEGLU: the current tile's first column (its bias DMA at J0(ke - 2))
  auto setup_tile = [&](int m0, int n0) {
    n0_tile = n0;
    if constexpr (LORA) {
      ub0 = __builtin_amdgcn_readfirstlane(((n0 / p.la_gn) * p.la_gr) & ~15);
      const int r = 8 * wid + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      lc8 = c * 8;
      lbase = wid < 2 ? (uint32_t)((ub0 + r) * p.lda_la + c * 8) * 2u : (uint32_t)kOOB;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc) {
        const int r = 8 * (PB + PS * pc) + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        c8[s][pc] = c * 8;
        if (s < 2) {
          const int m = m0 + (r / HALF) * Cfg::WM + s * HALF + (r % HALF);
          if constexpr (CONV) {
            if (pc < NPA) {
              const int hw = p.OH * p.OW;
              const int img = m / hw, rem = m - img * hw;
              cv_img[s][pc] = m < p.M ? img : -1;
              cv_oy[s][pc] = rem / p.OW;
              cv_ox[s][pc] = rem - cv_oy[s][pc] * p.OW;
            }
            base1[s][pc] = base2[s][pc] = (uint32_t)kOOB;
          } else {
            int src = m;
            if constexpr (EPI == 5) {  // tile rows (pixel pl, frame f) of 16-pixel group mt -> x row (clip, frame, pixel)
              const int ngrp = p.ta_hw >> 4, mt = m >> 8, r = m & 255;
              const int bb = mt / ngrp, pgg = mt - bb * ngrp;
              src = ((bb << 4) + (r & 15)) * p.ta_hw + (pgg << 4) + (r >> 4);
            }
            base1[s][pc] = m < p.M ? (uint32_t)(src * p.lda1 + c * 8) * 2u : (uint32_t)kOOB;
            base2[s][pc] = m < p.M ? (uint32_t)(src * p.lda2 + c * 8) * 2u : (uint32_t)kOOB;
          }
        } else {
          const int rb = s == 2 ? 32 : RB1;
          const int n = n0 + (r / rb) * Cfg::WN + (s - 2) * 32 + (r % rb);
          base1[s][pc] = (n < p.N && (s == 2 ? pc < 2 : pc < NPB1)) ? (uint32_t)(n * p.ldw + c * 8) * 2u : (uint32_t)kOOB;
        }
      }
  };
  // CONV: A slot s's pieces for its next k-tile (the slot's cursor); live = false issues zeros (counts stay uniform)
  auto conv_rebase = [&](int s) {
    const int ky = cv_tap[s] / 3, kx = cv_tap[s] - 3 * (cv_tap[s] / 3);
    cv_second[s] = cv_ci[s] >= p.C1;
    const int cs = cv_second[s] ? p.C2 : p.C1;
    cv_ci0[s] = cv_second[s] ? p.C1 : 0;
#pragma unroll
    for (int pc = 0; pc < NPA; ++pc) {
      int iy, ix;
      bool ok = cv_img[s][pc] >= 0;
      if (p.up) {
        const int uy = cv_oy[s][pc] + ky - 1, ux = cv_ox[s][pc] + kx - 1;
        ok = ok && uy >= 0 && uy < 2 * p.H && ux >= 0 && ux < 2 * p.W;
        iy = uy >> 1; ix = ux >> 1;
      } else {
        iy = cv_oy[s][pc] * p.stride + ky - 1 + p.pad0; ix = cv_ox[s][pc] * p.stride + kx - 1 + p.pad0;
        ok = ok && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      }
      base1[s][pc] = ok ? (uint32_t)(((cv_img[s][pc] * p.H + iy) * p.W + ix) * cs + c8[s][pc]) * 2u : (uint32_t)kOOB;
    }
    cv_rebase[s] = false;
  };
  auto conv_dma = [&](int s, bool live, char* dst) {
    if (cv_rebase[s]) conv_rebase(s);
    const uint32_t kc = (uint32_t)(cv_ci[s] - cv_ci0[s]) * 2u;
#pragma unroll
    for (int pc = 0; pc < NPA; ++pc)
      p8_dma16(cv_second[s] ? ra2 : ra1, dst + pc * PS * 1024, live ? (int)(base1[s][pc] + kc) : kOOB);
    cv_ci[s] += 64;
    if (cv_ci[s] == Ctot) { cv_ci[s] = 0; ++cv_tap[s]; }
    cv_rebase[s] = cv_ci[s] == 0 || (p.C2 > 0 && cv_ci[s] == p.C1);
  };
  // slot s of k-tile kt into buffer ((kbase + kt) & 1); kt >= kend: out-of-range offsets (zeros), keeps vmcnt counts
  // uniform
  auto dma_slot = [&](int s, int kt, int kend, int kbase) {
    if ((abl & 1) && kt > 1) return;
    if ((abl & 64) && s >= 2 && kt > 1) return;
    if ((abl & 128) && s < 2 && kt > 1) return;
    char* dst = smem + ((kbase + kt) & 1) * BUF + slot_off(s) + PB * 1024;
    const int k0 = kt * 64;
    const bool live = kt < kend && !((abl & 32) && kt > 1);
    if (CONV && s < 2) {
      conv_dma(s, live, dst);
    } else if (s < 2) {
      const bool second = ONE_A ? false : k0 >= p.K1;
      const uint32_t kb = (uint32_t)(second ? k0 - p.K1 : k0) * 2u;
#pragma unroll
      for (int pc = 0; pc < NPA; ++pc) {
        const bool kin = live && (!ktail || k0 + c8[s][pc] < p.K);
        const int off = kin ? (int)((second ? base2[s][pc] : base1[s][pc]) + kb) : kOOB;
        p8_dma16(second ? ra2 : ra1, dst + pc * PS * 1024, off);
      }
    } else {
      const uint32_t kb = (uint32_t)k0 * 2u;
#pragma unroll
      for (int pc = 0; pc < (s == 3 ? NPB1 : 2); ++pc) {
        const bool kin = live && (!ktail || k0 + c8[s][pc] < p.K);
        p8_dma16(rw, dst + pc * PS * 1024, kin ? (int)(base1[s][pc] + kb) : kOOB);
      }
    }
  };

  // slot s of a k-tile that is live and fully inside K (every k-tile but the last two of a segment): no checks
  auto dma_fast = [&](int s, int kt) {
    if ((abl & 1) && kt > 1) return;
    if ((abl & 64) && s >= 2 && kt > 1) return;
    if ((abl & 128) && s < 2 && kt > 1) return;
    char* dst = smem + ((kofs + kt) & 1) * BUF + slot_off(s) + PB * 1024;
    const int k0 = kt * 64;
    if (CONV && s < 2) {
      conv_dma(s, true, dst);
    } else if (s < 2) {
      const bool second = ONE_A ? false : k0 >= p.K1;
      const uint32_t kb = (uint32_t)(second ? k0 - p.K1 : k0) * 2u;
#pragma unroll
      for (int pc = 0; pc < NPA; ++pc)
        p8_dma16(second ? ra2 : ra1, dst + pc * PS * 1024, (int)((second ? base2[s][pc] : base1[s][pc]) + kb));
    } else {
#pragma unroll
      for (int pc = 0; pc < (s == 3 ? NPB1 : 2); ++pc)
        p8_dma16(rw, dst + pc * PS * 1024, (int)(base1[s][pc] + (uint32_t)k0 * 2u));
    }
  };

  // LORA: Acat columns of k-tile kt into its slot (buffer kt & 1), by waves 0-1 (the others issue nothing)
  auto dma_lora = [&](int kt, int kend, bool checked, int kbase) {
    if ((abl & 1) && kt > 1) return;
    if constexpr (LORA) {
      if (wid >= 2) return;
      char* dst = smem + Cfg::LORA_OFF + ((kbase + kt) & 1) * 2048 + wid * 1024;
      const int k0 = kt * 64;
      const bool kin = !checked || (kt < kend && k0 + lc8 < p.K);
      p8_dma16(rl, dst, kin ? (int)(lbase + (uint32_t)k0 * 2u) : kOOB);
    }
  };

  f32x4 acc[Cfg::MI][Cfg::NJ];
  f32x4 acc_u[2];   // LORA: u of row block wc of row quadrants 0 / 1 (this wave's row half)
  bf16x8 fl[2];     // LORA: Acat fragments of the current k-tile (16 u columns x 2 k-halves)
  // A fragments of the current row quadrant (mq): MQR x 16 rows x 2 k-halves.  LORA: wave column wc reads the
  // quadrant's row blocks rotated by wc (fa[i] = block (i + wc) mod MQR), so fa[0] is block wc, whose 16 u rows this
  // wave accumulates: the u MFMAs use fa[0] and no register array is indexed by the runtime wc (rounds 3-4 read block
  // wc a second time into a dedicated fu pair: 4 of the 28 ds_read_b128 per wave and k-tile).  acc[mq MQR + i] then
  // holds row block (i + wc) mod MQR of quadrant mq (p8_acc_row), which only the epilogues' row addressing sees: the
  // same operands meet in the same k order, so the bits are unchanged.
  bf16x8 fa[MQR][2];
  bf16x8 fb0[2][2], fb1[NJ1 > 2 ? NJ1 : 2][2];  // W fragments of column quadrants nq0 / nq1
#ifdef VST_P8_TRACE
  for (int i = 0; i < MQR; ++i) for (int h = 0; h < 2; ++h) fa[i][h] = bf16x8{};
  for (int j = 0; j < 2; ++j) for (int h = 0; h < 2; ++h) fb0[j][h] = bf16x8{};
  for (int j = 0; j < NJ1; ++j) for (int h = 0; h < 2; ++h) fb1[j][h] = bf16x8{};
#endif
  auto read_a = [&](int buf, int mq) {  // (buf: the LDS buffer, 0 or 1)
    if (abl & (16 | 128)) return;
    const char* S = smem + buf * BUF + slot_off(mq);
#pragma unroll
    for (int i = 0; i < MQR; ++i) {
      const int ib = LORA ? ((i + wc) & (MQR - 1)) : i;  // (MQR < 4: waves wc >= MQR repeat a block, their u unused)
#pragma unroll
      for (int h = 0; h < 2; ++h) fa[i][h] = *reinterpret_cast<const bf16x8*>(S + p8_off(wr * HALF + ib * 16 + fr, h * 4 + fq));
    }
  };
  auto read_b = [&](int buf, int nq, auto& fb) {
    if (abl & (16 | 64)) return;
    const char* S = smem + buf * BUF + slot_off(2 + nq);
    const int rb = nq == 0 ? 32 : RB1;
#pragma unroll
    for (int j = 0; j < (nq == 0 ? 2 : NJ1); ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) fb[j][h] = *reinterpret_cast<const bf16x8*>(S + p8_off(wc * rb + j * 16 + fr, h * 4 + fq));
  };
  auto read_l = [&](int buf) {
    if (abl & 16) return;
    if constexpr (LORA) {
      const char* S = smem + Cfg::LORA_OFF + buf * 2048;
#pragma unroll
      for (int h = 0; h < 2; ++h) fl[h] = *reinterpret_cast<const bf16x8*>(S + p8_off(fr, h * 4 + fq));
    }
  };
  // LORA: u rows of row block wc of the current row quadrant
  auto lora_mfma = [&](f32x4& au, int h) {
    if constexpr (LORA) if (!(abl & 2)) au = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[h], fa[0][h], au, 0, 0, 0);
  };
#define VST_P8_QUAD(MQ, NQ, FB)                                                                        \
  if (!(abl & 2)) {                                                                                  \
    _Pragma("unroll") for (int i = 0; i < MQR; ++i) _Pragma("unroll") for (int j = 0; j < ((NQ) == 0 ? 2 : NJ1); ++j) \
        _Pragma("unroll") for (int h = 0; h < 2; ++h) acc[(MQ) * MQR + i][(NQ) * 2 + j] =              \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j][h], fa[i][h], acc[(MQ) * MQR + i][(NQ) * 2 + j], 0, 0, 0); \
  }

  // k-tiles [kb, ke) of the current tile into acc (zeroed here); ends with the LDS drained and free for reuse
  auto run_segment = [&](int kb, int ke) {
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc_u[0] = acc_u[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Three barrier intervals per k-tile: I0 = {read Amq0, Bnq0} | Q(0,0) + Q(0,1) (32 MFMAs, fb1 = Bnq1(t) read in
    // I2 of t-1); I1 = {read Amq1} | Q(1,1); I2 = {read Bnq1(t+1)} | Q(1,0).  (Four phases of 16 MFMAs, one per
    // quadrant, measured 0.3 ms per step slower: 8 barriers per k-tile instead of 6, profiles/r2_ab_p8_3ph.txt.)  A slot read in interval I is refilled
    // in interval I+2 (both halves' reads retired), and waited for in the interval before its first read:
    //   I0(t): wait Amq1(t), issue Amq1(t+1);  I1(t): wait Bnq1(t+1), issue Bnq1(t+2);
    //   I2(t): wait Amq0/Bnq0(t+1), issue Amq0/Bnq0(t+2).   (2 DMAs per slot per wave)
    if constexpr (LORA) {  // V [BN][16] of this tile (older than every slot DMA: the first wait below covers it)
      const int row = wid * 32 + (lane >> 1), n = n0_tile + row;
      const bool ok = row < BN && n < p.N;
      p8_dma16(make_rsrc(p.Wt, p.wtail_bytes), smem + Cfg::V_OFF + wid * 1024,
               ok ? (int)(((uint32_t)n * p.ldw + p.K + ub0 + 8 * (lane & 1)) * 2u) : kOOB);
      if constexpr (BN > 256) {  // rows 256 .. BN - 1 (waves 0-1; older than every slot DMA like the first piece)
        const int row2 = 256 + row, n2 = n0_tile + row2;
        if (wid < 2)
          p8_dma16(make_rsrc(p.Wt, p.wtail_bytes), smem + Cfg::V_OFF + (8 + wid) * 1024,
                   row2 < BN && n2 < p.N ? (int)(((uint32_t)n2 * p.ldw + p.K + ub0 + 8 * (lane & 1)) * 2u) : kOOB);
      }
    }
    dma_slot(0, kb, ke, 0); dma_lora(kb, ke, true, 0); dma_slot(2, kb, ke, 0); dma_slot(3, kb, ke, 0);
    dma_slot(1, kb, ke, 0); dma_slot(3, kb + 1, ke, 0); dma_slot(0, kb + 1, ke, 0); dma_lora(kb + 1, ke, true, 0);
    dma_slot(2, kb + 1, ke, 0);
    VST_P8_VMWAIT_LX(2 * NPA + 2 + NPB1);  // A0, (Acat,) B0, B1 of kb landed
    p8_barrier();
    VST_P8_STAMP(1)
    read_b(kb & 1, 1, fb1);
    if (late) p8_barrier();
    if (late) __builtin_amdgcn_s_setprio(1);
    auto ktile = [&](int t, auto fast_tag) {
      constexpr bool FAST = decltype(fast_tag)::value;
      auto dma = [&](int s_, int kt) {
        if constexpr (FAST) dma_fast(s_, kt); else dma_slot(s_, kt, ke, 0);
      };
      const int buf = t & 1;
      // I0
      read_a(buf, 0);
      read_b(buf, 0, fb0);
      read_l(buf);
      if (!(abl & 4)) VST_P8_VMWAIT_LX(NPA + 2 + NPB1);  // A1(t) landed
      dma(1, t + 1);
      p8_barrier();
      lora_mfma(acc_u[0], 0);
      VST_P8_QUAD(0, 0, fb0)
      VST_P8_QUAD(0, 1, fb1)
      lora_mfma(acc_u[0], 1);
      p8_barrier();
      // I1
      read_a(buf, 1);
      if (!(abl & 4)) VST_P8_VMWAIT_LX(2 * NPA + 2);  // B1(t+1) landed
      dma(3, t + 2);
      p8_barrier();
      lora_mfma(acc_u[1], 0);
      VST_P8_QUAD(1, 1, fb1)
      lora_mfma(acc_u[1], 1);
      p8_barrier();
      // I2
      read_b(buf ^ 1, 1, fb1);
      if (!(abl & 4)) p8_vmwait<NPA + NPB1>();  // A0(t+1), B0(t+1) landed
      dma(0, t + 2);
      dma_lora(t + 2, ke, !FAST, 0);
      dma(2, t + 2);
      p8_barrier();
      VST_P8_QUAD(1, 0, fb0)
      p8_barrier();
    };
    int t = kb;
    const int ke_fast = ke - 2 - (ktail ? 1 : 0);
    for (; t < ke_fast; ++t) ktile(t, std::true_type{});
    for (; t < ke; ++t) ktile(t, std::false_type{});
    if (!late) p8_barrier();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the trailing zero DMAs land before LDS reuse
    p8_barrier();
  };
  // PH = 2: two barrier intervals of 32 MFMAs per k-tile (24 at BN = 192), so every load segment of one wave group
  // runs beside a full-length MFMA segment of the other, and each wave's DMAs split evenly over the two (the 3-interval
  // schedule pairs its 4-DMA interval with a 16-MFMA one):
  //   J0(t) = {read A0(t), B0(t), Acat(t); wait A1(t), B1(t+1); issue A1(t+1)}        | Q(0,0) + Q(0,1)
  //   J1(t) = {read A1(t); wait A0/B0(t+1); issue B1(t+2), A0(t+2) (+Acat), B0(t+2)} | Q(1,1), read B1(t+1), Q(1,0)
  // B1E (every kernel but GEGLU and the in-GEMM LoRA ones): B1's fragments are read inside J1's MFMA segment, after Q(1,1) frees fb1 (rounds
  // 2-4 read them in J0's load segment, 16 ds_reads against J1's 8; the loop ablations showed the load segments, not
  // the waits, idling the matrix core: profiles/r4_p8_loop_ablation.txt); so B1(t+1) is issued one interval earlier
  // (J1(t-1), first of that segment's DMAs) and waited with A1(t) in J0(t), before both groups' J1(t) MFMA segments.
  // GEGLU keeps   J0(t) = {read A0(t), B0(t), B1(t); wait A1(t); issue B1(t+1), A1(t+1)},  J1(t) = {read A1(t);
  // wait A0/B0/B1(t+1); issue A0(t+2), B0(t+2)}, as do the LoRA kernels: in the step GEGLU measured 0.9 % slower
  // with B1 moved and the LoRA kernels 1 %, the plain GEMMs and the convs 2-4 % faster (profiles/r4_ab_b1_j1.txt).  Every segment that reads
  // LDS ends with its reads retired (lgkmcnt(0)) before its barrier, so a slot read in interval X is refilled from
  // interval X + 1 on (WAR); a slot waited for in interval X is read in X + 1 (RAW, both groups' waits precede the
  // barrier the later reader passes).  Same k order per accumulator as PH = 3: bitwise-equal results.
  auto run_segment2 = [&](int kb, int ke, bool first) {
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc_u[0] = acc_u[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (LORA) {  // V [BN][16] of this tile (older than every slot DMA: the first wait below covers it)
      const int row = wid * 32 + (lane >> 1), n = n0_tile + row;
      const bool ok = row < BN && n < p.N;
      p8_dma16(make_rsrc(p.Wt, p.wtail_bytes), smem + Cfg::V_OFF + wid * 1024,
               ok ? (int)(((uint32_t)n * p.ldw + p.K + ub0 + 8 * (lane & 1)) * 2u) : kOOB);
      if constexpr (BN > 256) {  // rows 256 .. BN - 1 (waves 0-1; older than every slot DMA like the first piece)
        const int row2 = 256 + row, n2 = n0_tile + row2;
        if (wid < 2)
          p8_dma16(make_rsrc(p.Wt, p.wtail_bytes), smem + Cfg::V_OFF + (8 + wid) * 1024,
                   row2 < BN && n2 < p.N ? (int)(((uint32_t)n2 * p.ldw + p.K + ub0 + 8 * (lane & 1)) * 2u) : kOOB);
      }
    }
    // PERSIST, later tiles: k-tiles kb and kb + 1 were issued by the previous tile (A1 (!B1E: and B1) of kb + 1 just
    // before its epilogue) and have landed (its post-epilogue wait), so J0(kb) issues nothing and the waits of J0(kb),
    // J1(kb) (!B1E: and J0(kb + 1)) are skipped: the epilogue's stores, younger than those DMAs, stay in flight until
    // J0(kb + 1) (B1E: B1(kb + 2) is younger) / J1(kb + 1)
    const bool handed = PERSIST && !first;
    if (!PERSIST || first) {
      dma_slot(0, kb, ke, kofs); dma_lora(kb, ke, true, kofs); dma_slot(2, kb, ke, kofs); dma_slot(3, kb, ke, kofs);
      dma_slot(1, kb, ke, kofs);
      if constexpr (B1E) dma_slot(3, kb + 1, ke, kofs);
      dma_slot(0, kb + 1, ke, kofs); dma_lora(kb + 1, ke, true, kofs); dma_slot(2, kb + 1, ke, kofs);
      // A0, (Acat,) B0, B1 of kb landed; A1(kb), (B1,) A0, B0 of kb + 1 in flight
      VST_P8_VMWAIT_LX(2 * NPA + (B1E ? NPB1 : 0) + 2);
    }
    p8_barrier();
    if constexpr (B1E) read_b((kofs + kb) & 1, 1, fb1);  // B1(kb): every later B1 is read in the J1 before its k-tile
    VST_P8_STAMP(1)
    if (late) p8_barrier();
    if (late) __builtin_amdgcn_s_setprio(1);
    auto ktile2 = [&](int t, auto fast_tag) {
      constexpr bool FAST = decltype(fast_tag)::value;
      auto dma = [&](int s_, int kt) {
        if constexpr (FAST) {
          dma_fast(s_, kt);
        } else if (PERSIST && kt >= ke && has_next) {
          dma_slot(s_, kt - ke, ke, kofs + ke);  // the next tile's first k-tiles (bases switched at J1(ke - 2))
        } else {
          dma_slot(s_, kt, ke, kofs);
        }
      };
      const int buf = (kofs + t) & 1;
      // J0
      read_a(buf, 0);
      read_b(buf, 0, fb0);
      if constexpr (!B1E) read_b(buf, 1, fb1);
      read_l(buf);
      // A1(t) (B1E: and B1(t + 1)) landed
      if (!(abl & 4) && !(handed && (B1E ? t == kb : t <= kb + 1))) VST_P8_VMWAIT_LX(NPA + 2);
      // PERSIST GEGLU: the tile's 256 bias floats into the (otherwise unused) epilogue region by one LDS-DMA piece
      // of wave 0 (the other waves write a zero piece into a sink, so every wave's counts shift alike); issued before
      // A1 of ke - 1, so J0(ke - 1)'s wait keeps its count, and J1(ke - 2)'s covers it
      if constexpr (EPI == 1 && PERSIST) {
        if (!FAST && t == ke - 2) {
          const int c = bias_n0 + 4 * lane;
          p8_dma16(make_rsrc(p.bias, p.bias ? (uint32_t)p.N * 4u : 0u), smem + Cfg::EPI_OFF + (wid ? 1024 : 0),
                   wid == 0 && p.bias && c < p.N ? c * 4 : kOOB);
        }
      }
      auto dma_j0 = [&] {
        if (!(handed && t == kb)) {
          if constexpr (!B1E) dma(3, t + 1);
          dma(1, t + 1);
        }
      };
      if constexpr (!DMM) dma_j0();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      p8_barrier();
      lora_mfma(acc_u[0], 0);
      VST_P8_QUAD(0, 0, fb0)
      if constexpr (DMM) dma_j0();
      VST_P8_QUAD(0, 1, fb1)
      lora_mfma(acc_u[0], 1);
      if constexpr (DMM) p8_interleave_dma<(2 + NJ1) * MQR * 2 + (LORA ? 2 : 0), (B1E ? 0 : NPB1) + NPA>();
      p8_barrier();
      // J1
      read_a(buf, 1);
      if (!(abl & 4) && !(handed && t == kb)) p8_vmwait<NPA>();  // A0, (Acat,) B0 (!B1E: B1) of t + 1 landed
      // PERSIST: every slot has issued its last DMA of this tile (A0 / B0 (B1E: B1) at J1(ke - 3), A1 (!B1E: B1) at
      // J0(ke - 2)), so the slots' source bases switch to the next tile here
      if (PERSIST && !FAST && t == ke - 2 && has_next) setup_tile(nm0, nn0);
      // (DMM: the Acat piece, issued by waves 0-1 only, stays in the load segment, ahead of A0 / B0: a wave-dependent
      // branch inside the MFMA segment would split it; every wait that counts it counts A0 and B0 as well)
      static_assert(!(DMM && LORA && B1E), "DMM + LoRA: the Acat piece must stay younger than B1");
      // the Acat piece of k-tile t + 2: past this tile's end (PERSIST) the next tile's first two (bases switched above)
      auto dma_l = [&] {
        if (PERSIST && !FAST && t + 2 >= ke && has_next) dma_lora(t + 2 - ke, ke, true, kofs + ke);
        else dma_lora(t + 2, ke, !FAST, kofs);
      };
      auto dma_j1 = [&] {
        if constexpr (B1E) dma(3, t + 2);
        dma(0, t + 2);
        if constexpr (!DMM) dma_l();
        dma(2, t + 2);
      };
      if constexpr (DMM) dma_l();
      if constexpr (!DMM) dma_j1();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      p8_barrier();
      lora_mfma(acc_u[1], 0);
      VST_P8_QUAD(1, 1, fb1)
      if constexpr (DMM) dma_j1();
      if constexpr (B1E) {
        if (t + 1 < ke) read_b(buf ^ 1, 1, fb1);  // B1(t + 1), waited by both groups in J0(t)
      }
      VST_P8_QUAD(1, 0, fb0)
      lora_mfma(acc_u[1], 1);
      if constexpr (DMM) p8_interleave_dma<(2 + NJ1) * MQR * 2 + (LORA ? 2 : 0), (B1E ? NPB1 : 0) + NPA + 2>();
      if constexpr (B1E) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      p8_barrier();
    };
    int t = kb;
    const int ke_fast = ke - 2 - (ktail ? 1 : 0);
    for (; t < ke_fast; ++t) ktile2(t, std::true_type{});
    for (; t < ke; ++t) ktile2(t, std::false_type{});
    if (!late) p8_barrier();
    if constexpr (PERSIST) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next tile's k-tiles stay in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the trailing zero DMAs land before LDS reuse
    }
    p8_barrier();
  };
#undef VST_P8_QUAD
#undef VST_P8_VMWAIT_LX

  // LORA: u (bf16) -> LDS [BM rows][16 columns] at U, then acc += u . V^T over the 32-wide window (columns 16-31
  // zero: the [x | u] k-tile's second u half), V = W[n][K + ub0 ...]
  auto lora_post = [&](char* U) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      u32x2 v;
      v[0] = pack2bf(acc_u[q][0], acc_u[q][1]);
      v[1] = pack2bf(acc_u[q][2], acc_u[q][3]);
      if (wc < MQR) *reinterpret_cast<u32x2*>(U + (wr * Cfg::WM + q * HALF + wc * 16 + fr) * 32 + fq * 8) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bf16x8 zero8 = {};
    bf16x8 fv[Cfg::NJ];
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + Cfg::V_OFF + (wc * Cfg::WN + j * 16 + fr) * 32 + (fq & 1) * 16);
      fv[j] = fq < 2 ? v : zero8;
    }
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i) {
      bf16x8 fu = *reinterpret_cast<const bf16x8*>(U + (wr * Cfg::WM + p8_acc_row<Cfg, true>(i, wc) + fr) * 32 + (fq & 1) * 16);
      fu = fq < 2 ? fu : zero8;
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fv[j], fu, acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's u reads done before the epilogue stages the tile over them
  };
  int m0, n0;
  VST_P8_STAMP(0)
  constexpr int EREG = LORA ? Cfg::EPI_REGION_L : Cfg::EPI_REGION;  // PERSIST epilogue staging bytes
  if constexpr (PERSIST) {
    // gridDim.x (a multiple of 8) workgroups walk the tiles: the workgroups sharing an XCD (b % 8) take that XCD's
    // contiguous chunk of logical tiles in rounds, as the one-tile-per-workgroup launch places them.  Each tile's last
    // two k-tiles stream the next tile's first two into the ring, and its epilogue stages through the LDS past the ring.
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, per = gridDim.x >> 3;
    const int q = ntiles >> 3, r = ntiles & 7;
    const int beg = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    const int cnt = q + (xcd < r ? 1 : 0);
    if (loc >= cnt) return;  // (whole workgroup; the launcher keeps gridDim.x <= ntiles)
    int j = loc;
    tile_origin(beg + j, m0, n0);
    setup_tile(m0, n0);
    bool first = true;
    while (true) {
      const int jn = j + per;
      has_next = jn < cnt;
      if (has_next) tile_origin(beg + jn, nm0, nn0);
      bias_n0 = n0;
      run_segment2(0, nk, first);
#ifdef VST_ABL_NOEPI  // diagnostics build only: no epilogue (a guarded store of every accumulator's first lane
                      // element keeps all the MFMAs live)
      {
        float sink = 0.f;
        for (int i = 0; i < Cfg::MI; ++i)
          for (int jj = 0; jj < Cfg::NJ; ++jj) sink += acc[i][jj][0];
        if (sink == 1234.5f) p.C[0] = 0;
        if (has_next) {
          if constexpr (!B1E) dma_slot(3, 1, nk, kofs + nk);
          dma_slot(1, 1, nk, kofs + nk);
        }
      }
#else
      if constexpr (LORA) lora_post(smem + Cfg::U_OFF);  // (the ring holds the next tile's first k-tiles)
      p8_epilogue_passes<Cfg, EPI, EREG, LORA>(p, smem + (LORA ? Cfg::EPI_OFF_L : Cfg::EPI_OFF), m0, n0, acc, wr, wc,
                                               [&] {
        if (has_next) {  // A1 (!B1E: and B1) of the next tile's second k-tile (slots free: their last reads retired
                         // in the k-loop)
          if constexpr (!B1E) dma_slot(3, 1, nk, kofs + nk);
          dma_slot(1, 1, nk, kofs + nk);
        }
      });
#endif
      if (has_next) {  // the next tile's k-tiles landed; this wave's (exactly counted) stores may stay in flight
        p8_vmwait<p8_epi_stores<Cfg, EPI, EREG>()>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
      }
      p8_barrier();
      if (!has_next) return;
      j = jn;
      m0 = nm0;
      n0 = nn0;
      kofs += nk;
      first = false;
    }
  }
  tile_origin(xcd_remap(blockIdx.x, ntiles), m0, n0);
  setup_tile(m0, n0);
  if constexpr (PH == 2) run_segment2(0, nk, true);
  else run_segment(0, nk);
  VST_P8_STAMP(2)
  if constexpr (LORA) lora_post(smem);  // (the drained ring)
#ifdef VST_ABL_NOEPI  // diagnostics build only: no epilogue of any kind (attention epilogues included)
  {
    float sink = 0.f;
    for (int i = 0; i < Cfg::MI; ++i)
      for (int jj = 0; jj < Cfg::NJ; ++jj) sink += acc[i][jj][0];
    if (sink == 1234.5f) p.C[0] = 0;
  }
#else
  if constexpr (EPI == 4) xattn_epilogue<Cfg, LORA>(p, smem, m0, n0, acc, wr, wc);
  else if constexpr (EPI == 5) tattn_epilogue<Cfg>(p, smem, m0, n0, acc, wr, wc);
  else tile_epilogue<Cfg, EPI, LORA, CONV>(p, smem, m0, n0, acc, wr, wc);
#endif
#ifdef VST_P8_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  VST_P8_STAMP(3)
}

// The k-loop schedule: 2 (two 32-MFMA intervals per k-tile, run_segment2; default) or 3 (three intervals,
// run_segment; VST_P8_PH=3).  Measured (tools/p8_ph_ab.py, profiles/r4_p8_ph_ab.txt): 2-5 % faster in isolation on
// the step's GEMM shapes, -0.4 ms per denoise step in two alternations; outputs bit-identical.
static int p8_ph_env() {
  static const int v = [] {
    const char* e = getenv("VST_P8_PH");
    return e ? atoi(e) : 2;
  }();
  return v;
}

template <int EPI, int BN, bool LORA, int PH, int BM, bool CONV = false>
static int launch_p8_ph(const GemmArgs& a, hipStream_t s) {
  static bool attr = false;
  using Cfg = P8Cfg<BN, BM>;
  constexpr int lds = EPI == 4 ? 160 * 1024 : (LORA ? Cfg::LDS_LORA : Cfg::LDS);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_p8_kernel<EPI, BN, LORA, PH, BM, CONV>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_p8_kernel<EPI, BN, LORA, PH, BM, CONV>), dim3(nwg), dim3(512), lds, s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// Persistent tiles (default; VST_P8_PERSIST=0 restores one workgroup per tile): a grid of one workgroup per CU walks
// the tiles; each tile's last two k-tiles stream the next tile's first two into the ring, so a tile's fill overlaps
// the previous tile's epilogue.  Same bits.  Measured (tools/p8_ph_ab.py, profiles/r4_p8_persist_ab.txt): 0-15 %
// faster per launch on the step's multi-round shapes (K = 320 / 640 most), the denoise step -0.9 ms same-box; the
// convs stay on one workgroup per tile (their persistent variant spilled SGPRs and ran 2 % slower).
static int g_p8_persist = -1;  // VST_P8_PERSIST, or vst_p8_persist (tests, A/B)
static int p8_persist_env() {
  if (g_p8_persist < 0) {
    const char* e = getenv("VST_P8_PERSIST");
    g_p8_persist = e ? atoi(e) : 1;
  }
  return g_p8_persist;
}
static int p8_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8)
      n = 256;
    return n & ~7;
  }();
  return v;
}

// whether launch_gemm_p8 runs the persistent kernel for this shape: the 2-interval schedule, at least two tiles per
// workgroup, K a multiple of 64 and >= 128 (the stream hands over two whole k-tiles), whole 8-column output chunks
// (and one A source: launch_p8_epi)
bool p8_persist_applies(int M, int N, int K, int epi, int bn) {
  if (!p8_persist_env() || p8_ph_env() != 2 || (epi != 0 && epi != 1 && epi != 3)) return false;
  const int bm = bn == 320 ? 128 : 256;
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  return tiles >= 2L * p8_cus() && K >= 128 && (K & 63) == 0 && (N % (epi == 1 ? 16 : 8)) == 0;
}

template <int EPI, int BN, int BM, bool LORA = false>
static int launch_p8_persist(const GemmArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_p8_kernel<EPI, BN, LORA, 2, BM, false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int grid = ntiles < p8_cus() ? (ntiles & ~7) : p8_cus();
  if (grid < 8) return VST_ERR_ARG;
  hipLaunchKernelGGL((gemm_p8_kernel<EPI, BN, LORA, 2, BM, false, true>), dim3(grid), dim3(512), 160 * 1024, s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

// The in-GEMM LoRA kernels on the persistent grid (128x320 tiles only: a pass of the staged epilogue must hold whole
// row quadrants of the rotated LoRA accumulators), wherever p8_persist_applies: the 32x32 level's q/k/v 123 -> 108 us
// and out-projection 48 -> 43 us per launch, bitwise equal (profiles/r5_ab_lora_persist.txt).  VST_P8_LORA_PERSIST=0
// restores one workgroup per tile (A/B).
static int p8_lora_persist_env() {
  static const int v = [] {
    const char* e = getenv("VST_P8_LORA_PERSIST");
    return e ? atoi(e) : 1;
  }();
  return v;
}
bool p8_lora_persist_on() { return p8_persist_env() && p8_ph_env() == 2 && p8_lora_persist_env(); }

// BN = 320 runs 128-row tiles (P8Cfg)
template <int EPI, int BN, bool LORA = false>
static int launch_p8_epi(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = BN == 320 ? 128 : 256;
  if constexpr (!LORA && EPI != 4 && EPI != 5)
    if (!a.A2 && (size_t)a.M * a.ldc * 2 < 0x7fff0000u && p8_persist_applies(a.M, a.N, a.K, EPI, BN))
      return launch_p8_persist<EPI, BN, BM>(a, s);
  if constexpr (LORA && EPI == 0 && BN == 320)
    if (p8_lora_persist_on() && !a.A2 && (size_t)a.M * a.ldc * 2 < 0x7fff0000u &&
        p8_persist_applies(a.M, a.N, a.K, EPI, BN))
      return launch_p8_persist<EPI, BN, BM, true>(a, s);
  return p8_ph_env() == 2 ? launch_p8_ph<EPI, BN, LORA, 2, BM>(a, s) : launch_p8_ph<EPI, BN, LORA, 3, BM>(a, s);
}

// in-GEMM LoRA down-projection (a.la set): epilogue 0 (bias / residual), bn 256 or 192
int launch_gemm_p8_lora(const GemmArgs& a, int bn, hipStream_t s) {
  if (!a.la) return VST_ERR_ARG;
  if (bn == 320) return launch_p8_epi<0, 320, true>(a, s);
  return bn == 192 ? launch_p8_epi<0, 192, true>(a, s) : launch_p8_epi<0, 256, true>(a, s);
}

// temporal attention epilogue (a.ta_hw set), 256x256 tiles
int launch_gemm_p8_tattn(const GemmArgs& a, hipStream_t s) {
  if (a.ta_hw <= 0 || (a.ta_hw & 15) || a.A2 || (a.M & 255)) return VST_ERR_ARG;
  return launch_p8_epi<5, 256>(a, s);
}

// cross-attention epilogue (a.xa_k set), 256x192 tiles, with or without the in-GEMM LoRA
int launch_gemm_p8_xattn(const GemmArgs& a, hipStream_t s) {
  if (!a.xa_k || !a.xa_v) return VST_ERR_ARG;
  return a.la ? launch_p8_epi<4, 192, true>(a, s) : launch_p8_epi<4, 192, false>(a, s);
}

// implicit-GEMM 3x3 conv (GemmArgs conv geometry, Ctot % 64 == 0), epilogue 0; bn: 256, 192 or 320
int launch_gemm_p8_conv(const GemmArgs& a, int bn, hipStream_t s) {
  if ((a.C1 & 63) || (a.C2 & 63) || a.K != 9 * (a.C1 + a.C2)) return VST_ERR_ARG;
  const bool ph2 = p8_ph_env() == 2;
  switch (bn) {
    case 256: return ph2 ? launch_p8_ph<0, 256, false, 2, 256, true>(a, s) : launch_p8_ph<0, 256, false, 3, 256, true>(a, s);
    case 192: return ph2 ? launch_p8_ph<0, 192, false, 2, 256, true>(a, s) : launch_p8_ph<0, 192, false, 3, 256, true>(a, s);
    case 320: return ph2 ? launch_p8_ph<0, 320, false, 2, 128, true>(a, s) : launch_p8_ph<0, 320, false, 3, 128, true>(a, s);
    default: return VST_ERR_ARG;
  }
}

// epi: 0 bias / row bias / residual, 1 GEGLU, 3 bias + GELU; bn: 256, 192 or 320 (128-row tiles; not with GEGLU)
int launch_gemm_p8(const GemmArgs& a, int epi, int bn, hipStream_t s) {
  if (a.A2 && (a.K1 & 63)) return VST_ERR_ARG;  // a 64-deep k-tile must not straddle the two A sources
  if (bn == 192 || bn == 320) {
    switch (epi) {
      case 0: return bn == 192 ? launch_p8_epi<0, 192>(a, s) : launch_p8_epi<0, 320>(a, s);
      case 3: return bn == 192 ? launch_p8_epi<3, 192>(a, s) : launch_p8_epi<3, 320>(a, s);
      default: return VST_ERR_ARG;
    }
  }
  if (bn != 256) return VST_ERR_ARG;
  switch (epi) {
    case 0: return launch_p8_epi<0, 256>(a, s);
    case 1: return launch_p8_epi<1, 256>(a, s);
    case 3: return launch_p8_epi<3, 256>(a, s);
    default: return VST_ERR_ARG;
  }
}

}  // namespace vst

extern "C" int vst_p8_persist(int on) {
  const int prev = vst::p8_persist_env() ? 1 : 0;
  vst::g_p8_persist = on ? 1 : 0;
  return prev;
}

#ifdef VST_P8_TRACE
extern "C" int vst_p8_trace_read(void* host_dst, int n_wg) {
  if (n_wg > 8192) n_wg = 8192;
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(vst::vst_p8_trace_buf), (size_t)n_wg * 64, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
#endif
