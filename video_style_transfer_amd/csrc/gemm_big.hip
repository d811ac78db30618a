// LDS-DMA ring GEMM: the main bf16 MFMA GEMM of the denoise path (projections, GEGLU FF,
// implicit-GEMM conv3x3, split-K partials).  Same contract as gemm.hip (GemmArgs, AMODE 0/1,
// EPI 0/1/2).  Tiles (template): 256x256 and 256x128 (8 waves, 1 WG/CU), 128x128 and 128x64
// (4 waves, 2-3 WG/CU).
//
// Staging: `buffer_load_dwordx4 ... lds` (__builtin_amdgcn_raw_ptr_buffer_load_lds) writes each
// wave's 1 KiB piece (16 rows x 64 B) straight into LDS; the buffer range check supplies the
// zeros for conv padding, M/N tails and the LoRA K tail.  BK = 32, 4-stage ring, ONE barrier per
// k-tile: at iteration k the DMA for tile k+3 goes into the stage read at k-1 (every wave has
// passed the barrier that ended k-1), the MFMAs of tile k run, then a counted
// `s_waitcnt vmcnt(N)` retires only tile k+1 before the barrier — two tiles (~1 us) stay in flight,
// covering the ~1.1 us issue->landed time of LDS-DMA under load (MI355X price list).
//
// LDS image per stage: [rows][32 bf16] (64-B rows), 16-B chunk c of row r stored at slot
// c ^ G[(r >> 2) & 3] with G = {2,0,1,3}: every ds_read_b128 fragment read (16 rows x one chunk
// per 16-lane block) is bank-conflict free under CDNA4's b128 lane grouping
// {0-3,12-15,20-27},{4-11,16-19,28-31},... .  Because the DMA image is lane-linear, the inverse
// permutation is applied to each lane's SOURCE address (lane l fetches chunk (l&3) ^ G[(l>>4)&3]).
#include <type_traits>

#include "gemm_common.h"
#include "gemm_epilogue.h"

namespace vst {

constexpr int RBK = 32;

__device__ __forceinline__ int gperm(int x) { return (0x3102 >> (4 * x)) & 3; }  // G = {2,0,1,3}
__device__ __forceinline__ int rswz(int row, int chunk) {
  return row * 64 + ((chunk ^ gperm((row >> 2) & 3)) << 4);
}

template <int BM_, int BN_, int WM_, int WN_, int STAGES_>
struct RingCfg {
  static constexpr int STAGES = STAGES_;
  static constexpr int BM = BM_, BN = BN_;
  static constexpr int WAVES_M = WM_, WAVES_N = WN_;
  static constexpr int NWAVES = WM_ * WN_;
  static constexpr int THREADS = 64 * NWAVES;
  static constexpr int WM = BM / WM_, WN = BN / WN_;  // wave tile
  static constexpr int MI = WM / 16, NJ = WN / 16;
  static constexpr int A_BYTES = BM * RBK * 2, B_BYTES = BN * RBK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PIECES = A_BYTES / 1024 / NWAVES;  // per wave per tile (floor)
  static constexpr int B_PIECES = B_BYTES / 1024 / NWAVES;
  // Tiles whose 1-KiB pieces do not split evenly over the waves (BN = 160: 10 B pieces, BM = 192:
  // 12 A pieces, 8 waves): waves wid < B_EXTRA (A_EXTRA) load one more B (A) piece, so a wave's DMA
  // count per tile is D_BASE + its number of extras (wait_tiles takes the wave's own count).
  static constexpr int B_EXTRA = (B_BYTES / 1024) % NWAVES;
  static constexpr int A_EXTRA = (A_BYTES / 1024) % NWAVES;
  static constexpr int D_BASE = A_PIECES + B_PIECES;
  static constexpr int DPT = D_BASE + (B_EXTRA ? 1 : 0) + (A_EXTRA ? 1 : 0);  // max DMA per thread per tile
  static constexpr int IDX_BX = D_BASE;                           // offs[] slot of the extra B piece
  static constexpr int IDX_AX = D_BASE + (B_EXTRA ? 1 : 0);       // offs[] slot of the extra A piece
  static constexpr int EPI_BYTES = BM * (BN * 2 + 16);  // bf16 tile staged for the epilogue
  static constexpr int LDS = STAGES * STAGE > EPI_BYTES ? STAGES * STAGE : EPI_BYTES;
  static_assert(A_BYTES % 1024 == 0 && B_BYTES % 1024 == 0, "piece split");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// wait until at most `tiles` tiles' DMA (D instructions each for this wave) are still outstanding
template <int D>
__device__ __forceinline__ void wait_tiles_d(int tiles) {
  switch (tiles) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * D) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * D) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * D) : "memory"); break;
  }
}

template <class Cfg>
__device__ __forceinline__ void wait_tiles(int tiles, int n_extra) {
  if constexpr (Cfg::DPT == Cfg::D_BASE) {
    wait_tiles_d<Cfg::D_BASE>(tiles);
  } else {
    if (n_extra == 0) wait_tiles_d<Cfg::D_BASE>(tiles);
    else if (Cfg::DPT == Cfg::D_BASE + 1 || n_extra == 1) wait_tiles_d<Cfg::D_BASE + 1>(tiles);
    else wait_tiles_d<Cfg::DPT>(tiles);
  }
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_piece, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)((__attribute__((address_space(3))) char*)(uintptr_t)lds_piece),
                                           16, off, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Grouped tile order: GROUP_M row panels sweep the N axis together, so the A and W panels a
// k-slice needs are shared by ~GROUP_M tiles running concurrently on one XCD (L2 hits instead of
// repeated MALL fetches).  `t` is an XCD-contiguous logical tile index.
__device__ __forceinline__ void tile_coords(int t, int nbm, int nbn, int& bm, int& bn, int group_m = 8) {
  const int GROUP_M = group_m;
  const int in_group = GROUP_M * nbn;
  const int gid = t / in_group, first_m = gid * GROUP_M;
  const int gsize = min(nbm - first_m, GROUP_M);
  bm = first_m + (t - gid * in_group) % gsize;
  bn = (t - gid * in_group) / gsize;
}

// One output tile's k-range [kt0, kt1) (the whole K, or a split-K slab with EPI 2): ring pipeline + epilogue.
template <class Cfg, int AMODE, int EPI>
__device__ __forceinline__ void ring_tile(const GemmArgs& p, char* smem, const int m0, const int n0, const int kt0,
                                          const int kt1) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / Cfg::WAVES_N, wc = wid - wr * Cfg::WAVES_N;

  const auto ra1 = make_rsrc(p.A1, p.a1_bytes);
  const auto ra2 = make_rsrc(p.A2 ? p.A2 : p.A1, p.A2 ? p.a2_bytes : 0u);
  const auto rw = make_rsrc(p.Wt, p.w_bytes);

  // piece q (of this wave) = tile rows 16*(q*NWAVES + wid) .. +15; lane -> row +(lane>>2), slot lane&3
  const int prow = lane >> 2;
  const int lchunk = (lane & 3) ^ gperm((lane >> 4) & 3);

  constexpr int AQ = Cfg::A_PIECES + (Cfg::A_EXTRA ? 1 : 0);  // q == A_PIECES: the extra piece
  int rowA[AQ], oyv[AQ], oxv[AQ];
#pragma unroll
  for (int q = 0; q < AQ; ++q) {
    const int m = m0 + 16 * (q * Cfg::NWAVES + wid) + prow;
    if (AMODE == 0) {
      rowA[q] = m < p.M ? m : -1;
      oyv[q] = oxv[q] = 0;
    } else if (m < p.M) {
      const int hw = p.OH * p.OW;
      const int img = m / hw, rem = m - img * hw;
      rowA[q] = img;
      oyv[q] = rem / p.OW;
      oxv[q] = rem - oyv[q] * p.OW;
    } else {
      rowA[q] = -1; oyv[q] = oxv[q] = 0;
    }
  }
  int rowB[Cfg::B_PIECES + 1];
#pragma unroll
  for (int q = 0; q <= Cfg::B_PIECES; ++q) {
    const int n = n0 + 16 * (q * Cfg::NWAVES + wid) + prow;  // q == B_PIECES: the extra piece
    rowB[q] = n < p.N ? n : -1;
  }
  const bool has_bx = wid < Cfg::B_EXTRA, has_ax = wid < Cfg::A_EXTRA;  // wave-uniform
  const int n_extra = (has_bx ? 1 : 0) + (has_ax ? 1 : 0);
  const int Ctot = p.C1 + p.C2;
  const int nk = kt1 - kt0;

  // ---- incremental DMA addressing (keeps the load segment of each k-tile short) ----
  // A piece's byte offset for k-tile kt is base + (k offset inside the current source run) * 2.
  // Rows past M / N carry base kOOB: unsigned adds keep it beyond every buffer, so the hardware
  // range check returns zeros.  Per-lane K checks are only needed when K is not a multiple of 32.
  // Convs walk a (tap, channel) cursor one k-tile at a time (issue() is called for consecutive
  // tiles) and recompute bases only when the tap or the concat source changes.
  const bool ktail = (p.K & (RBK - 1)) != 0;
  uint32_t bB[Cfg::B_PIECES + 1];
#pragma unroll
  for (int q = 0; q <= Cfg::B_PIECES; ++q)
    bB[q] = rowB[q] >= 0 ? (uint32_t)(rowB[q] * p.ldw + lchunk * 8) * 2u : (uint32_t)kOOB;
  uint32_t bA[AQ], bA2[AQ];
  if (AMODE == 0) {
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      bA[q] = rowA[q] >= 0 ? (uint32_t)(rowA[q] * p.lda1 + lchunk * 8) * 2u : (uint32_t)kOOB;
      bA2[q] = rowA[q] >= 0 ? (uint32_t)(rowA[q] * p.lda2 + lchunk * 8) * 2u : (uint32_t)kOOB;
    }
  }
  int c_tap = 0, c_ci = 0, run_ci0 = 0;  // conv cursor: next tile's tap and channel (of C1 + C2)
  bool rebase_due = true;
  if (AMODE == 1) {
    const int k00 = kt0 * RBK;
    c_tap = k00 / Ctot;
    c_ci = k00 - c_tap * Ctot;
  }
  auto rebase = [&]() {
    const int ky = c_tap / 3, kx = c_tap - 3 * (c_tap / 3);
    const bool second = c_ci >= p.C1;
    const int cs = second ? p.C2 : p.C1;
    run_ci0 = second ? p.C1 : 0;
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      int iy, ix;
      bool ok = rowA[q] >= 0;
      if (p.up) {
        const int uy = oyv[q] + ky - 1, ux = oxv[q] + kx - 1;
        ok = ok && uy >= 0 && uy < 2 * p.H && ux >= 0 && ux < 2 * p.W;
        iy = uy >> 1; ix = ux >> 1;
      } else {
        iy = oyv[q] * p.stride + ky - 1 + p.pad0; ix = oxv[q] * p.stride + kx - 1 + p.pad0;
        ok = ok && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      }
      bA[q] = ok ? (uint32_t)(((rowA[q] * p.H + iy) * p.W + ix) * cs + lchunk * 8) * 2u : (uint32_t)kOOB;
    }
  };
  int offs[Cfg::DPT];
  bool a_second = false;
  auto prep = [&](int kt, auto fast_tag) {  // fast: the k-tile lies fully inside K (no per-lane tail check)
    const int k0 = kt * RBK;
    const uint32_t kb = (uint32_t)k0 * 2u;
    const bool kin = decltype(fast_tag)::value || !ktail || (k0 + lchunk * 8 < p.K);
#pragma unroll
    for (int q = 0; q < Cfg::B_PIECES; ++q) offs[q] = kin ? (int)(bB[q] + kb) : kOOB;
    if constexpr (Cfg::B_EXTRA != 0) offs[Cfg::IDX_BX] = kin ? (int)(bB[Cfg::B_PIECES] + kb) : kOOB;
    if (AMODE == 0) {
      a_second = k0 >= p.K1;  // K1 is a multiple of 64: a k-tile never straddles the sources
      const uint32_t ka = a_second ? (uint32_t)(k0 - p.K1) * 2u : kb;
#pragma unroll
      for (int q = 0; q < Cfg::A_PIECES; ++q)
        offs[Cfg::B_PIECES + q] = kin ? (int)((a_second ? bA2[q] : bA[q]) + ka) : kOOB;
      if constexpr (Cfg::A_EXTRA != 0)
        offs[Cfg::IDX_AX] = kin ? (int)((a_second ? bA2[Cfg::A_PIECES] : bA[Cfg::A_PIECES]) + ka) : kOOB;
    } else {
      if (rebase_due) rebase();
      a_second = run_ci0 != 0;
      const uint32_t kc = (uint32_t)(c_ci - run_ci0) * 2u;
#pragma unroll
      for (int q = 0; q < Cfg::A_PIECES; ++q) offs[Cfg::B_PIECES + q] = (int)(bA[q] + kc);
      if constexpr (Cfg::A_EXTRA != 0) offs[Cfg::IDX_AX] = (int)(bA[Cfg::A_PIECES] + kc);
      c_ci += RBK;
      if (c_ci == Ctot) { c_ci = 0; ++c_tap; }
      rebase_due = c_ci == 0 || (p.C2 > 0 && c_ci == p.C1);
    }
  };
  auto dma_piece = [&](int stage, int idx) {  // idx: compile-time after unrolling
    char* As = smem + stage * Cfg::STAGE;
    if (Cfg::A_EXTRA != 0 && idx == Cfg::IDX_AX) {
      if (has_ax) dma16(a_second ? ra2 : ra1, As + (Cfg::A_PIECES * Cfg::NWAVES + wid) * 1024, offs[idx]);
    } else if (Cfg::B_EXTRA != 0 && idx == Cfg::IDX_BX) {
      if (has_bx) dma16(rw, As + Cfg::A_BYTES + (Cfg::B_PIECES * Cfg::NWAVES + wid) * 1024, offs[idx]);
    } else if (idx < Cfg::B_PIECES) {
      dma16(rw, As + Cfg::A_BYTES + (idx * Cfg::NWAVES + wid) * 1024, offs[idx]);
    } else {
      const int q = idx - Cfg::B_PIECES;
      dma16(a_second ? ra2 : ra1, As + (q * Cfg::NWAVES + wid) * 1024, offs[idx]);
    }
  };
  auto issue = [&](int kt, int stage, auto fast_tag) {
    prep(kt, fast_tag);
#pragma unroll
    for (int d = 0; d < Cfg::DPT; ++d) dma_piece(stage, d);
  };

  f32x4 acc[Cfg::MI][Cfg::NJ];
#pragma unroll
  for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int S = Cfg::STAGES;
  const int fr = lane & 15, fq = lane >> 4;
#ifdef VST_GEMM_DIAG
  const int abl = p.ablate;  // VST_GEMM_ABLATE (diagnostics build only, tools/p8_variants.sh)
#else
  constexpr int abl = 0;
#endif
  const bool no_dma = abl & 1, no_mfma = abl & 2, no_lds = abl & 16;
  typedef bf16x8 FragA[Cfg::MI];
  typedef bf16x8 FragB[Cfg::NJ];
  FragA fa0, fa1;
  FragB fb0, fb1;
  auto load_into = [&](FragA& fa, FragB& fb, int stage) {
    if (no_lds) return;  // diagnostics: no fragment reads (wrong results)
    const char* As = smem + stage * Cfg::STAGE;
    const char* Bs = As + Cfg::A_BYTES;
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(Bs + rswz(wc * Cfg::WN + j * 16 + fr, fq));
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(As + rswz(wr * Cfg::WM + i * 16 + fr, fq));
  };
  auto mfmas = [&](FragA& ca, FragB& cb, auto flip_tag) {  // flip: s_setprio 1/0 around the chain
    if constexpr (decltype(flip_tag)::value) __builtin_amdgcn_s_setprio(1);
    if (!no_mfma) {
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::NJ; ++j)
          // W fragment as the MFMA's A operand: acc[i][j][r] = C[m = i*16 + (lane&15)][n = j*16 +
          // 4*(lane>>4) + r] — four consecutive output columns per lane (vector epilogue).
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i) asm volatile("" ::"v"(ca[i]));
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) asm volatile("" ::"v"(cb[j]));
    }
    if constexpr (decltype(flip_tag)::value) __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (Cfg::NWAVES == 8) {
    // ---- ping-pong schedule (8 waves; waves w and w+4 share a SIMD) ----
    // Each k-tile is two barrier intervals: L = {LDS-DMA issue of tile it+S-1, ds_reads of tile it's
    // fragments, counted wait for this wave's DMA of tile it+1} and C = {the MFMA chain of tile it}.
    // Waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier up front, which waves 0-3 pay
    // back after the loop), so in every interval one wave of each SIMD issues MFMAs while its
    // partner issues loads: the load work AND its LDS latency hide under the partner's matrix
    // work, so one register set of fragments suffices (48 VGPRs instead of 96).
    // Hazards (intervals counted globally, group g's L(it) at 2it+g, C(it) at 2it+1+g):
    //  RAW: tile it is read in L(it) (interval >= 2it); each group waited for its own DMA of tile it
    //       in L(it-1) (interval <= 2it-1), before the barrier that ends it.
    //  WAR: L(it) refills the stage of tile it-1, whose fragments every group read in L(it-1) and
    //       retired (lgkmcnt(0)) before the barrier that ended that interval (<= 2it-1).
    const bool late = wid >= 4;
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) issue(kt0 + s, s, std::false_type{});
    wait_tiles<Cfg>(min(nk, S - 1) - 1, n_extra);  // own DMA of tile 0 landed
    __builtin_amdgcn_s_barrier();
    if (late) __builtin_amdgcn_s_barrier();
#ifdef VST_RING_LATEPRIO
    if (late) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half
    using flip_t = std::false_type;
#else
    using flip_t = std::true_type;
#endif
    int wrs = S - 1, rd = 0;
    auto ktile = [&](int it, auto fast_tag) {
      constexpr bool FAST = decltype(fast_tag)::value;  // tile it+S-1 exists and is not the last of K
      const bool steady = FAST || it + S - 1 < nk;  // tile it+S-1 exists: issue it, keep S-2 tiles in flight
      if (steady && !no_dma) issue(kt0 + it + S - 1, wrs, fast_tag);
      wrs = wrs + 1 == S ? 0 : wrs + 1;
      load_into(fa0, fb0, rd);
      rd = rd + 1 == S ? 0 : rd + 1;
      if (steady && !no_dma) wait_tiles<Cfg>(S - 2, n_extra);
      else if (it + 1 < nk) wait_tiles<Cfg>(0, n_extra);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      mfmas(fa0, fb0, flip_t{});
      __builtin_amdgcn_s_barrier();
    };
    int it = 0;
    // fast iterations: tile it+S-1 < nk - 1 (and, with a K tail, never the last k-tile of K)
    const int it_fast = ktail && kt1 == (p.K + RBK - 1) / RBK ? nk - S : nk - S + 1;
#ifndef VST_RING_NOFAST
    for (; it < it_fast; ++it) ktile(it, std::true_type{});
#endif
    for (; it < nk; ++it) ktile(it, std::false_type{});
    if (!late) __builtin_amdgcn_s_barrier();
  } else {
  // ---- prologue: tiles 0..S-2 in flight, retire tile 0 ----
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(kt0 + s, s, std::false_type{});
  wait_tiles<Cfg>(min(nk, S - 1) - 1, n_extra);
  __builtin_amdgcn_s_barrier();

  // fragments of the current k-tile live in registers: all MI + NJ ds_read_b128 are issued
  // right after the barrier that publishes the stage, so the MFMA chain below runs back to
  // back (the compiler's lgkmcnt ladder exposes only the first read's latency).
  // Fragments are double-buffered in registers: iteration `it` publishes tile it+1 (counted
  // vmcnt + barrier), refills the stage tile it-1 used, issues the ds_reads of tile it+1 into
  // the spare register set, and only then runs tile it's MFMA chain — the LDS read latency of
  // the next tile hides under the current MFMAs instead of opening a bubble after every barrier.
  int wrs = S - 1, nrd = 1 % S;  // next stage to fill / stage holding tile it+1
  // FAST: tile it+S-1 exists and is not the last k-tile of K (no per-lane tail checks, no end-of-range tests)
  auto step = [&](int it, FragA& ca, FragB& cb, FragA& na, FragB& nb, auto fast_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
    if (FAST || it + 1 < nk) {
      // tile it+1 must have landed: steady state leaves S-3 younger tiles in flight, the tail drains
      if (FAST || (it + S - 2 < nk && !no_dma)) wait_tiles<Cfg>(S - 3, n_extra);
      else wait_tiles<Cfg>(0, n_extra);
      __builtin_amdgcn_s_barrier();
    }
    if (FAST || (it + S - 1 < nk && !no_dma)) issue(kt0 + it + S - 1, wrs, fast_tag);
    wrs = wrs + 1 == S ? 0 : wrs + 1;
    if (FAST || it + 1 < nk) load_into(na, nb, nrd);
    nrd = nrd + 1 == S ? 0 : nrd + 1;
    mfmas(ca, cb, std::true_type{});
  };
  if (nk > 0) load_into(fa0, fb0, 0);
  const int it_fast = no_dma ? 0 : (ktail && kt1 == (p.K + RBK - 1) / RBK ? nk - S : nk - S + 1);
  int it = 0;
  for (; it + 1 < it_fast; it += 2) {
    step(it, fa0, fb0, fa1, fb1, std::true_type{});
    step(it + 1, fa1, fb1, fa0, fb0, std::true_type{});
  }
  for (; it < nk; it += 2) {
    step(it, fa0, fb0, fa1, fb1, std::false_type{});
    if (it + 1 < nk) step(it + 1, fa1, fb1, fa0, fb0, std::false_type{});
  }
  }
  __builtin_amdgcn_s_barrier();  // all waves done with the ring before the epilogue reuses LDS
  if (abl & 8) {  // diagnostics: no epilogue (keep the accumulators alive)
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }

  // ---------------- epilogue ----------------
  // Split-K partials go straight from registers to the fp32 slab (16 B per lane).  Otherwise
  // bias (and GELU for EPI 3) is applied in registers, the whole BMxBN tile is staged ONCE in LDS as bf16 (the rounding
  // point of the reference's bf16 linear/conv output), and a vectorized pass applies the per-frame
  // row bias / residual add (after that rounding, as the reference's separate add does) or GEGLU
  // and writes full 16-B chunks.  All residual loads of a thread are issued before any use.
  const int lrow0 = wr * Cfg::WM + fr;          // + i*16
  const int lcol0 = wc * Cfg::WN + 4 * fq;      // + j*16
  if constexpr (EPI == 2) {
    float* slab = p.ws + (size_t)blockIdx.z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i) {
      const int m = m0 + lrow0 + i * 16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < Cfg::NJ; ++j) {
        const int n = n0 + lcol0 + j * 16;
        float* dst = slab + (size_t)m * p.N + n;
        if (n + 4 <= p.N) {
          *reinterpret_cast<f32x4*>(dst) = acc[i][j];
        } else {
          for (int e = 0; e < p.N - n; ++e) dst[e] = acc[i][j][e];
        }
      }
    }
    return;
  } else {
    tile_epilogue<Cfg, EPI>(p, smem, m0, n0, acc, wr, wc);
  }
}

// Data-parallel launch: one tile per workgroup (split-K: blockIdx.z selects the k-range).
template <class Cfg, int AMODE, int EPI>
__global__ __launch_bounds__(Cfg::THREADS, 1) void gemm_ring_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = Cfg::BM, BN = Cfg::BN;
  const int nbn = (p.N + BN - 1) / BN, nbm = (p.M + BM - 1) / BM;
  const int nk_all = (p.K + RBK - 1) / RBK;
  if (EPI != 2 && p.persist) {
    // Persistent: gridDim.x workgroups (one per resident slot) walk the tiles.  Workgroup b runs on XCD
    // b % 8 and takes that XCD's contiguous chunk of logical tiles in rounds, so co-resident tiles share
    // L2 panels as in the one-tile-per-workgroup launch; the next tile's ring prologue follows the
    // previous tile's epilogue stores without a workgroup relaunch (the stores drain under its DMA).
    const int T = nbm * nbn, G = gridDim.x;
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int per_xcd = (G - xcd + 7) / 8;
    const int q = T >> 3, r = T & 7;
    const int beg = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    const int cnt = q + (xcd < r ? 1 : 0);
    for (int j = loc; j < cnt; j += per_xcd) {
      int bm, bn;
      tile_coords(beg + j, nbm, nbn, bm, bn, p.group_m > 0 ? p.group_m : 8);
      ring_tile<Cfg, AMODE, EPI>(p, smem, bm * BM, bn * BN, 0, nk_all);
      __syncthreads();  // the staged epilogue tile / ring LDS is reused by the next tile
    }
    return;
  }
  int bm, bn;
  tile_coords(xcd_remap(blockIdx.x, nbn * nbm), nbm, nbn, bm, bn, p.group_m > 0 ? p.group_m : 8);
  int kt0 = 0, kt1 = nk_all;
  if (EPI == 2) {
    kt0 = (int)((long long)nk_all * blockIdx.z / p.splits);
    kt1 = (int)((long long)nk_all * (blockIdx.z + 1) / p.splits);
  }
  ring_tile<Cfg, AMODE, EPI>(p, smem, bm * BM, bn * BN, kt0, kt1);
}

// stages: as many as the LDS budget allows at the intended residency (lookahead S-2 tiles)
using Cfg256x256 = RingCfg<256, 256, 2, 4, 5>;  // 160 KiB, 1 WG/CU
using Cfg256x128 = RingCfg<256, 128, 4, 2, 6>;  // 144 KiB, 1 WG/CU
using Cfg128x128 = RingCfg<128, 128, 2, 2, 5>;  //  80 KiB, 2 WG/CU
using Cfg128x64 = RingCfg<128, 64, 2, 2, 6>;    //  72 KiB, 2 WG/CU
using Cfg256x160 = RingCfg<256, 160, 4, 2, 5>;  // 130 KiB, 1 WG/CU: N = 320/640/960/1280/1920/3840 without waste
using Cfg192x256 = RingCfg<192, 256, 2, 4, 5>;  // 140 KiB, 1 WG/CU: 215 tiles at M = 8192, N = 1280

template <class Cfg, int AMODE, int EPI>
static int launch_ring_k(const GemmArgs& a, hipStream_t s, dim3 grid) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_ring_kernel<Cfg, AMODE, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_ring_kernel<Cfg, AMODE, EPI>), grid, dim3(Cfg::THREADS), Cfg::LDS, s, a);
  return hipGetLastError() == hipSuccess ? VST_OK : VST_ERR_LAUNCH;
}

template <class Cfg, int AMODE, int EPI>
static int launch_ring_t(const GemmArgs& a, hipStream_t s, int splits) {
  const int nwg = ((a.M + Cfg::BM - 1) / Cfg::BM) * ((a.N + Cfg::BN - 1) / Cfg::BN);
  if (EPI != 2 && a.persist > 0) {
    const int per_cu = Cfg::NWAVES == 8 ? 1 : 2;
    const int slots = a.persist * per_cu;
    if (nwg > slots) return launch_ring_k<Cfg, AMODE, EPI>(a, s, dim3(slots, 1, 1));
  }
  return launch_ring_k<Cfg, AMODE, EPI>(a, s, dim3(nwg, 1, splits));
}

template <class Cfg>
static int dispatch_cfg(const GemmArgs& a, int amode, int epi, hipStream_t s, int splits) {
  if (amode == 0) {
    if (epi == 0) return launch_ring_t<Cfg, 0, 0>(a, s, splits);
    if (epi == 3) return launch_ring_t<Cfg, 0, 3>(a, s, splits);
    if (epi == 1) {
      if constexpr (Cfg::NJ % 4 == 0) return launch_ring_t<Cfg, 0, 1>(a, s, splits);
      return VST_ERR_ARG;  // GEGLU pairs 32 hidden + 32 gate columns inside one wave's 64
    }
    return launch_ring_t<Cfg, 0, 2>(a, s, splits);
  }
  if (epi == 0) return launch_ring_t<Cfg, 1, 0>(a, s, splits);
  if (epi == 2) return launch_ring_t<Cfg, 1, 2>(a, s, splits);
  return VST_ERR_ARG;
}

// tile: 1 = 128x128, 2 = 128x64, 3 = 256x256, 4 = 256x128, 6 = 256x160, 7 = 192x256.  epi: 0 plain, 1 GEGLU,
// 2 split-K partial, 3 bias + GELU
int launch_gemm_ring(const GemmArgs& a, int amode, int epi, int tile, int splits, hipStream_t s) {
  switch (tile) {
    case 1: return dispatch_cfg<Cfg128x128>(a, amode, epi, s, splits);
    case 2: return epi == 1 ? VST_ERR_ARG : dispatch_cfg<Cfg128x64>(a, amode, epi, s, splits);
    case 3: return dispatch_cfg<Cfg256x256>(a, amode, epi, s, splits);
    case 4: return dispatch_cfg<Cfg256x128>(a, amode, epi, s, splits);
    case 6: return epi == 1 ? VST_ERR_ARG : dispatch_cfg<Cfg256x160>(a, amode, epi, s, splits);
    case 7: return dispatch_cfg<Cfg192x256>(a, amode, epi, s, splits);
    default: return VST_ERR_ARG;
  }
}

}  // namespace vst
