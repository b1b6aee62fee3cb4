// 16-bit (fp16 / bf16) k x k stride-1 convolution on big maps, round 5 ("conv16").
//
// One workgroup (8 waves, two per SIMD) owns a 16 x 32-pixel tile of one image and BN output
// channels.  The GEMM is computed TRANSPOSED: MFMA A = the packed weights (rows = output
// channels), B = the input halo (columns = pixels), so a lane's accumulator holds runs of 4
// consecutive channels of one pixel and the epilogue stores them straight from registers (no
// LDS round trip).  Wave layout: WN channel columns x (8 / WN) pixel rows; every wave owns
// 96 channels (3 accumulator tiles) x PJ tile rows of 32 pixels (PJ = 4 at WN = 2, 2 at WN = 1).
//
// The reduction runs over stages (16-channel chunk k, tap group g of G taps).  Stage s+1's data
// -- the G taps' weights [G][BN][32 B] and, at g = 0, chunk k+1's input halo
// [(16+KH-1) x (32+KW-1) px][32 B] -- is moved by LDS-DMA (buffer_load ... lds) into the other half
// of two double buffers while stage s computes; every wave issues its share of the 1-KB pieces
// spread over the stage's first taps.  Out-of-image halo pixels are out-of-range buffer offsets
// (the hardware returns zeros), so no load is conditional and no lane computes a pixel test per
// chunk: each piece's per-lane offset is fixed for the whole launch, the chunk advances the
// scalar soffset.  16-B halves of a halo pixel are XOR-swizzled by bit 3 of its halo COLUMN (and a
// weight row by bit 3 of its channel), so the ds_read_b128 fragment reads of 32 consecutive
// pixels / channels are conflict-free at every tap shift, and every fragment address is a
// per-lane base (one per tap column) plus a compile-time immediate: no VALU in the loop.
// One barrier per stage.  v_mfma_f32_32x32x16_{f16,bf16}, fp32 accumulation.
#pragma once
#include <type_traits>
#include "lic_common.h"

namespace lic {

int wd_env(const char* name, int def);   // conv_split_wd.hip

typedef __attribute__((address_space(3))) void c16_lds_void;

// diagnostic build only (-DC16_STAMP=1, tools/conv16_stamps.py): per-workgroup phase cycle sums
// (s_memtime) written past the end of the output (the caller allocates room); outputs stay valid
#ifndef C16_STAMP
#define C16_STAMP 0
#endif
// diagnostic ablations (-DC16_ABL=bits, timing only, outputs wrong): 1 no stores in the register epilogue,
// 2 every chunk's halo read from chunk 0 (L2-resident after the first stage), 4 no weight DMA after the
// prologue, 8 no halo DMA after the prologue
#ifndef C16_ABL
#define C16_ABL 0
#endif
// a stage's LDS-DMA pieces are issued over its first C16_ISSUE taps
#ifndef C16_ISSUE
#define C16_ISSUE 6
#endif
#if C16_STAMP
#define C16T(v)                                                                          \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#else
#define C16T(v)
#endif

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): compile-time loop indices where an
// unroll pragma is not binding (an index that stays a runtime value would move a register array --
// the accumulators -- to scratch)
template <int I, int N, typename F>
__device__ __forceinline__ void c16_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    c16_static_for<I + 1, N>(f);
  }
}

// The epilogue variants the conv16 / gemm16 launches take (lic_common.h epilogue_run on NQ staged
// 32 x 32 tiles, ct + q * 32 * 33): plain, + r1, gate (g, r1, r2), GDN (g; + r1: ResidualBlockWithStride's
// GDN + skip), and the scalar path (unaligned views, pixel shuffle).  Fewer compiled variants than
// epilogue_all's seven.
inline int c16_epi_mask_host(const lic_conv_args& a) {
  const bool gdn = a.epi == LIC_EPI_GDN_DIV || a.epi == LIC_EPI_GDN_RSQRT || a.epi == LIC_EPI_GDN_SQRT;
  return ((gdn || a.epi == LIC_EPI_GATE) ? EPI_G : 0) | ((a.r1 != nullptr && a.epi != LIC_EPI_HALF_TANH) ? EPI_R1 : 0) |
         ((a.epi == LIC_EPI_HALF_TANH || a.epi == LIC_EPI_GATE) ? EPI_R2 : 0);   // = epi_mask()
}
inline bool c16_epi_supported(const lic_conv_args& a) {
  const int m = c16_epi_mask_host(a);
  return m == 0 || m == EPI_R1 || m == EPI_G || m == (EPI_G | EPI_R1) || m == (EPI_G | EPI_R1 | EPI_R2);
}
// VMASKS: the operand sets that get a vector variant (bit 0: none, 1: r1, 2: g, 3: g + r1, 4: g + r1 + r2);
// any other set, and unaligned views, take the scalar path (each variant is a copy of the epilogue
// loop: conv16's 12-tile kernels spill with more than two of them)
template <typename T, int NQ, int TN, int CT_STRIDE, int VMASKS, typename Stage>
__device__ __forceinline__ void c16_epilogue(const lic_conv_args& a, float* ct, const int* rowpix, int n0,
                                             const float* sbias, int lane, Stage& stage) {
  const int m = epi_vec_ok<T>(a) ? epi_mask(a) : -1;
  if constexpr ((VMASKS & 1) != 0) {
    if (m == 0) return epilogue_run<T, NQ, TN, 0, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
  }
  if constexpr ((VMASKS & 2) != 0) {
    if (m == EPI_R1) return epilogue_run<T, NQ, TN, EPI_R1, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
  }
  if constexpr ((VMASKS & 4) != 0) {
    if (m == EPI_G) return epilogue_run<T, NQ, TN, EPI_G, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
  }
  if constexpr ((VMASKS & 8) != 0) {
    if (m == (EPI_G | EPI_R1))
      return epilogue_run<T, NQ, TN, EPI_G | EPI_R1, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
  }
  if constexpr ((VMASKS & 16) != 0) {
    if (m == (EPI_G | EPI_R1 | EPI_R2))
      return epilogue_run<T, NQ, TN, EPI_G | EPI_R1 | EPI_R2, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
  }
  epilogue_run<T, NQ, TN, -1, Stage, CT_STRIDE>(a, ct, rowpix, n0, sbias, lane, stage);
}

// One LDS-DMA piece: 64 lanes x 16 B from rsrc + voffset + soffset to lds + 16 * lane.  (In a
// __device__ helper: used directly in the kernel body, the builtin makes the host pass drop the
// kernel's launch stub.)
__device__ __forceinline__ void c16_dma(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (c16_lds_void*)lds, 16, voff, soff, 0, 0);
}

struct C16Plan {
  int tiles_x, tiles_y;
  int dymin, dxmin;
  int nchunks;        // cpad / 16
  unsigned xrec;      // bytes addressable from a.x (buffer range; past it loads read zeros)
  unsigned wrec;      // bytes of the packed weights
  int nst;            // stages = nchunks * ngroups
  int fast_epi;       // the register epilogue variant (c16_fast_epi): 0 none, 1 plain / + r1, 2 gate
  int frag;           // 1: the weights come from a.wgt_split in MFMA-fragment order (c16_frag_ok)
  // byte strides of the weight source (either layout, c16_wstrides): 32-row block, 16-channel chunk, tap;
  // and per lane: row, 16-B channel half
  int ws_co, ws_k, ws_tap, wl_row, wl_half;
};

// 16-bit weights in MFMA-fragment order (lic_conv_args.wgt_split for LIC_F16 / LIC_BF16, include/lic.h):
// [copad/32][cpad/16][ntaps][64 lanes][16 B], lane = 32 * (channel half) + (row % 32) -- one fragment is
// one contiguous 1 KB (8 cache lines) instead of 32 rows x 32 B on 32 lines
inline bool c16_frag_ok(const lic_conv_args& a) {
  return a.wgt_split != nullptr && a.mfma_mode == 0 && (a.dtype == LIC_F16 || a.dtype == LIC_BF16) &&
         ((uintptr_t)a.wgt_split % 16) == 0 && a.copad % 32 == 0 && a.cpad % 16 == 0 && wd_env("LIC_W16_FRAG", 1);
}
// the weight source strides of both layouts: [copad][ntaps][cpad] rows, or fragment order
template <typename Plan>
inline void c16_wstrides(const lic_conv_args& a, Plan& p) {
  const int nch = a.cpad / 16;
  if (p.frag) {
    p.ws_co = nch * a.ntaps * 1024;
    p.ws_k = a.ntaps * 1024;
    p.ws_tap = 1024;
    p.wl_row = 16;
    p.wl_half = 512;
  } else {
    p.ws_co = 32 * a.ntaps * a.cpad * 2;
    p.ws_k = 32;
    p.ws_tap = a.cpad * 2;
    p.wl_row = a.ntaps * a.cpad * 2;
    p.wl_half = 16;
  }
}

// S = 1: stages are (chunk, group of G taps = G/KW tap rows).  S = 2: stages are (chunk, input-parity
// phase (py, px)): phase taps (2a+py, 2b+px) form a stride-1 grid of ceil((KH-py)/2) x ceil((KW-px)/2)
// taps over the input sampled at (2r+py, 2c+px), so each phase is a stride-1 conv on its own halo.
template <int KH, int KW, int S, int G, int BN, int WN>
struct C16Geo {
  static constexpr int TH = 16, TW = 32, NW = 8, NT = NW * 64;
  static constexpr int WM = NW / WN;           // wave rows (pixel direction)
  static constexpr int PJ = TH / WM;           // tile rows (32-px fragments) per wave
  static constexpr int WCH = BN / WN;          // channels per wave
  static constexpr int CT = WCH / 32;          // channel tiles per wave
  static constexpr int KHE = S == 1 ? KH : (KH + 1) / 2, KWE = S == 1 ? KW : (KW + 1) / 2;   // halo tap grid
  static constexpr int HH = TH + KHE - 1, HWD = TW + KWE - 1;
  static constexpr int HPIX = HH * HWD;
  static constexpr int HPIECES = (HPIX * 2 + 63) / 64;
  static constexpr int HBYTES = HPIECES * 1024;
  static constexpr int NTAPS = KH * KW;
  static constexpr int NG = S == 1 ? NTAPS / G : 4;           // stages per chunk
  static constexpr int GMAX = S == 1 ? G : KHE * KWE;         // taps of the largest stage
  static constexpr int WPIECES = GMAX * BN / 32;
  static constexpr int WBYTES = WPIECES * 1024;
  static constexpr int HPW = (HPIECES + NW - 1) / NW;   // halo pieces per wave (max)
  static constexpr int WPW = (WPIECES + NW - 1) / NW;   // weight pieces per wave (max)
  static constexpr int LDS_PIPE = 2 * HBYTES + 2 * WBYTES;          // the main loop's double buffers
  static constexpr int LDS_EPI = NW * 32 * 33 * 4;                    // the epilogue's per-wave slots (>= 32 x 80 B)
  static constexpr int LDS_MAIN = LDS_PIPE > LDS_EPI ? LDS_PIPE : LDS_EPI;
  static constexpr int SMEM = LDS_MAIN + BN * 4 + TH * TW * 4;     // + bias + destination pixels
  static_assert(S == 2 || (NTAPS % G == 0 && G % KW == 0), "a tap group is whole tap rows");
  static_assert(WCH % 32 == 0 && TH % WM == 0, "wave tile");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

// FAST: 0 = the shared epilogue (c16_epilogue), 1 = the register epilogue (plain / + r1), 2 = the
// register epilogue of the Win_noShift_Attention gate g * sigmoid(act(acc + b) + r1) + r2
template <typename T, int KH, int KW, int S, int G, int BN, int WN, int FAST>
__global__ __launch_bounds__(512, 1) void conv16_kernel(const lic_conv_args a, const C16Plan p) {
  using Geo = C16Geo<KH, KW, S, G, BN, WN>;
  constexpr int NW = Geo::NW, PJ = Geo::PJ, CT = Geo::CT, HWD = Geo::HWD;
  constexpr int TH = Geo::TH, TW = Geo::TW;
  constexpr int HBYTES = Geo::HBYTES, WBYTES = Geo::WBYTES;
  constexpr int HPW = Geo::HPW, WPW = Geo::WPW;
  constexpr int NPW = HPW + WPW;

  extern __shared__ __attribute__((aligned(1024))) char smem[];
  float* sbias = (float*)(smem + Geo::LDS_MAIN);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WN, wr = wave / WN;
  const int l32 = lane & 31, lh = lane >> 5;

  int bid = blockIdx.x;
  const int tx_t = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty_t = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int n0 = blockIdx.y * BN;
  const int i0 = ty_t * TH, j0 = tx_t * TW;
  const int iy0 = i0 * S + p.dymin, ix0 = j0 * S + p.dxmin;

  for (int n = tid; n < BN; n += Geo::NT) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
  // destination pixel of every tile pixel (row-major 16 x 32; -1 = outside the output lattice)
  int* rowpix = (int*)(sbias + BN);
  for (int m = tid; m < TH * TW; m += Geo::NT) {
    const int i = i0 + m / TW, j = j0 + m % TW;
    int base = -1;
    if (i < a.mi && j < a.mj) {
      int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
      if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
      base = (b * a.ho + oy) * a.wo + ox;
    }
    rowpix[m] = base;
  }

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)p.xrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.frag ? a.wgt_split : a.wgt), (short)0, (int)p.wrec, 0x00020000);

  // ---- per-lane source offsets of this wave's pieces (fixed for the launch) ----
  // halo piece P = wave + NW*m: slot q = 64P + lane -> halo pixel q>>1, stored half q&1 holds
  // channel half (q&1) ^ bit3(column)
  // (S = 2: phase (py, px) samples input pixel (iy0 + py + 2r, ix0 + px + 2c); computed per stage)
  auto halo_off = [&](int m, int py, int px) -> unsigned {
    const int P = wave + NW * m;
    const int q = P * 64 + lane;
    const int hp = q >> 1;
    const int r = hp / HWD, cc = hp - r * HWD;
    const int c = (q & 1) ^ ((cc >> 3) & 1);
    const int iy = iy0 + py + S * r, ix = ix0 + px + S * cc;
    const bool ok = hp < Geo::HPIX && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    return ok ? (unsigned)((((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + c * 8) * 2) : 0x80000000u;
  };
  unsigned hoff[S == 1 ? HPW : 1];
  if constexpr (S == 1) {
#pragma unroll
    for (int m = 0; m < HPW; ++m) hoff[m] = halo_off(m, 0, 0);
  }
  // weight piece Q (rotated by 4 waves to balance the per-wave piece counts): tap Q / (BN/32),
  // channels (Q % (BN/32))*32 + lane/2, stored half lane&1 holds channel half (lane&1) ^ bit3(n)
  const int wq0 = (wave + 4) % NW;
  const unsigned woff_lane = (unsigned)((lane >> 1) * p.wl_row + ((lane & 1) ^ ((lane >> 4) & 1)) * p.wl_half);

  // (a chunk order rotated per workgroup, so that the workgroups sharing an L2 stream different weight
  // lines, measured 0.3-2 % slower: r05w)
  auto issue_piece = [&](int m, int k, int g, int hb, int wb, bool with_halo) {
    // m < HPW: halo piece m; else weight piece m - HPW
    if (m < HPW) {
      if (!with_halo || ((C16_ABL & 8) && (k | g) != 0)) return;
      const int P = wave + NW * m;
      if (P >= Geo::HPIECES) return;
      const unsigned ho = S == 1 ? hoff[S == 1 ? m : 0] : halo_off(m, g >> 1, g & 1);
      c16_dma(xrs, smem + hb * HBYTES + P * 1024, ho, (C16_ABL & 2) ? 0 : k * 32);
    } else {
      const int Q = wq0 + NW * (m - HPW);
      if (Q >= Geo::WPIECES || ((C16_ABL & 4) && (k | g) != 0)) return;
      const int tt = Q / (BN / 32), nq = Q - tt * (BN / 32);
      int tap;
      if constexpr (S == 1) {
        tap = g * G + tt;
      } else {   // tap tt of phase g = (py, px): grid (tt / kwp, tt % kwp)
        const int py = g >> 1, px = g & 1, khp = (KH - py + 1) / 2, kwp = (KW - px + 1) / 2;
        if (tt >= khp * kwp) return;
        const int ta = tt / kwp, tb = tt - ta * kwp;
        tap = (2 * ta + py) * KW + 2 * tb + px;
      }
      const int soff = ((n0 >> 5) + nq) * p.ws_co + tap * p.ws_tap + k * p.ws_k;
      c16_dma(wrs, smem + 2 * HBYTES + wb * WBYTES + Q * 1024, woff_lane, soff);
    }
  };

  // ---- fragment addressing: per-lane bases + compile-time immediates ----
  // weights: row n = wc*WCH + i*32 + l32, logical half lh -> stored half lh ^ bit3(l32)
  const int wlane = l32 * 32 + ((lh ^ ((l32 >> 3) & 1)) << 4) + wc * Geo::WCH * 32;
  // halo: pixel (row wr*PJ + j + ty, column l32 + tx); one base per tap column tx
  int hlane[Geo::KWE];
#pragma unroll
  for (int tx = 0; tx < Geo::KWE; ++tx) {
    const int col = l32 + tx;
    hlane[tx] = (wr * PJ * HWD + col) * 32 + ((lh ^ ((col >> 3) & 1)) << 4);
  }

  floatx16 acc[CT][PJ];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int j = 0; j < PJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#if C16_STAMP
  unsigned long long t_begin = 0, t_loop = 0, t_a = 0, t_b = 0, t_c = 0, t_end = 0, sum_comp = 0, sum_wait = 0;
#endif
  C16T(t_begin);
  // prologue: stage 0 (halo of chunk 0 + the first tap group's weights)
#pragma unroll
  for (int m = 0; m < NPW; ++m) issue_piece(m, 0, 0, 0, 0, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  C16T(t_loop);

  const int nst = p.nst;
  // one stage: s = k * NG + g; PH >= 0 is the stride-2 phase of the stage (compile time)
  auto stage = [&](int s, auto ph_c) {
    constexpr int PH = decltype(ph_c)::value;
    C16T(t_a);
    const int k = s / Geo::NG, g = S == 1 ? s - k * Geo::NG : PH;
    const int s1 = s + 1;
    const int k1 = s1 / Geo::NG, g1 = S == 1 ? s1 - k1 * Geo::NG : (PH + 1) & 3;
    const bool more = s1 < nst;
    // S = 1: one halo per chunk (buffer k & 1, loaded with the chunk's first stage); S = 2: one per stage
    const bool with_halo = S == 2 || g1 == 0;
    const int hb1 = S == 1 ? (k1 & 1) : (s1 & 1);
    const char* hbuf = smem + (S == 1 ? (k & 1) : (s & 1)) * HBYTES;
    const char* wbuf = smem + 2 * HBYTES + (s & 1) * WBYTES;
    // the stage's taps: an NTY x NTX stride-1 grid starting at halo row ty0 (S = 2, phase (py, px):
    // ceil((KH-py)/2) x ceil((KW-px)/2) taps)
    constexpr int NTY = S == 1 ? G / KW : (PH >> 1 ? KH / 2 : (KH + 1) / 2);
    constexpr int NTX = S == 1 ? KW : (PH & 1 ? KW / 2 : (KW + 1) / 2);
    constexpr int NTP = NTY * NTX;
    // pieces are issued during the first ISSUE taps of a stage (the rest of the stage hides them)
    constexpr int ISSUE = NTP < C16_ISSUE ? NTP : C16_ISSUE;
    const char* hrow = hbuf + (S == 1 ? (g * G) / KW : 0) * HWD * 32;
    auto load_a = [&](int tt, u32x4(&fa)[CT]) {
#pragma unroll
      for (int i = 0; i < CT; ++i) fa[i] = *(const u32x4*)(wbuf + wlane + (tt * BN + i * 32) * 32);
    };
    auto load_b = [&](int tt, int j) -> u32x4 {
      const int ty = tt / NTX, tx = tt - (tt / NTX) * NTX;
      return *(const u32x4*)(hrow + hlane[tx] + (j + ty) * HWD * 32);
    };
    u32x4 fa[2][CT], fb[PJ];
    load_a(0, fa[0]);
#pragma unroll
    for (int j = 0; j < PJ; ++j) fb[j] = load_b(0, j);
#pragma unroll
    for (int tt = 0; tt < NTP; ++tt) {
      const int cur = tt & 1;
      if (tt + 1 < NTP) load_a(tt + 1, fa[cur ^ 1]);
      // this tap's share of the next stage's pieces
      if (tt < ISSUE && more) {
#pragma unroll
        for (int m = (tt * NPW) / ISSUE; m < ((tt + 1) * NPW) / ISSUE; ++m)
          issue_piece(m, k1, g1, hb1, s1 & 1, with_halo);
      }
#pragma unroll
      for (int j = 0; j < PJ; ++j) {
#pragma unroll
        for (int i = 0; i < CT; ++i) acc[i][j] = mfma_k16<T>(fa[cur][i], fb[j], acc[i][j]);
        if (tt + 1 < NTP) fb[j] = load_b(tt + 1, j);
      }
    }
    C16T(t_b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    C16T(t_c);
#if C16_STAMP
    sum_comp += t_b - t_a;
    sum_wait += t_c - t_b;
#endif
  };
  using std::integral_constant;
  if constexpr (S == 1) {
    for (int s = 0; s < nst; ++s) stage(s, integral_constant<int, 0>{});
  } else {   // the four phases of a chunk as straight-line code
    for (int s = 0; s < nst; s += 4) {
      stage(s, integral_constant<int, 0>{});
      stage(s + 1, integral_constant<int, 1>{});
      stage(s + 2, integral_constant<int, 2>{});
      stage(s + 3, integral_constant<int, 3>{});
    }
  }

  // ---- epilogue (lic_common.h epilogue_all): each wave stages one 32 x 32 fp32 tile at a time in a
  // private LDS slot (over the now idle halo buffers) as [pixel][channel], then finishes it in the
  // store layout -- 16 B of one pixel per lane, consecutive lanes on consecutive channels -- with the
  // fused bias / activation / residual / gate / GDN operands loaded the same way (the transposed
  // accumulators hold 4-channel runs; stored as they are, every store would touch 32 cache lines) ----
  // one pass per tile row: its CT tiles are staged first (their accumulators die before the operand
  // loads of the pass), then finished
  float* ct = (float*)smem + wave * (32 * 33);
  // All CT * PJ tiles go through ONE runtime loop (epilogue_run, two tiles per iteration, operands one
  // tile ahead) that stages tile q in the wave's slot by compile-time indices under a uniform test: the
  // loop body runs from the instruction cache.  Unrolled per tile, the epilogue was ~250 k instructions
  // of straight-line code, each executed once: 45 % of the kernel's cycles (stamps, profiles/r05).
  auto stage_tile = [&](int q) {
    c16_static_for<0, CT * PJ>([&](auto qc) {
      constexpr int qq = decltype(qc)::value;
      if (q == qq) {
#pragma unroll
        for (int r = 0; r < 16; ++r) ct[l32 * 33 + 8 * (r >> 2) + 4 * lh + (r & 3)] = acc[qq % CT][qq / CT][r];
      }
    });
  };
  if constexpr (FAST) {
    // Register epilogue (plain / + residual with a cheap activation, 16-B aligned views, whole
    // channel tiles): bias + activation (+ r1) on the accumulators as they stand (4-channel runs of
    // one pixel per lane), rounded, staged as 16-bit [pixel][channel] rows in the wave's slot, read
    // back as 16 B of consecutive channels per lane and stored.  Unrolled per tile with compile-time
    // accumulator indices and ~50 instructions a tile (the general epilogue spends ~250 a tile).
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    // one tile row (CT tiles = the wave's 96 channels) at a time: staged as [32 px][CT*32 ch] 16-bit rows
    // (208-B pitch), ONE LDS round trip per row, then each pixel's CT*64 contiguous bytes stored as 16-B
    // chunks (a round trip per tile made the epilogue 16 % of the kernel: profiles/r05 stamps)
    constexpr int SP = 208;   // >= CT*64 + 16
    static_assert(CT * 64 + 16 <= SP && NW * 32 * SP <= Geo::LDS_MAIN, "epilogue staging");
    char* stg = smem + wave * (32 * SP);
    T* __restrict__ yg = (T*)a.y;
    T* __restrict__ y2g = (T*)a.y2;
    const T* __restrict__ r1g = (const T*)a.r1;
    const T* __restrict__ gg = (const T*)a.g;
    const T* __restrict__ r2g = (const T*)a.r2;
    const int act = a.act;
    const float slope = a.slope;
    c16_static_for<0, PJ>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const int row = i0 + wr * PJ + j;
      c16_static_for<0, CT>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int nloc = wc * Geo::WCH + i * 32;       // channel of the tile's first column, in the block
        // residual / gate operands, in the accumulator layout (8 B = 4 channels per lane and run)
        u32x2 rr[4], rg[4], r2v[4];
        if (FAST == 2 || r1g) {
          const int col = j0 + l32;
          const bool ok = row < a.mi && col < a.mj;
          const int64_t pix = ok ? ((int64_t)b * a.ho + a.oy0 + a.osy * row) * a.wo + a.ox0 + a.osx * col : 0;
          const int nb = n0 + nloc + 4 * lh;
          if (r1g) {
#pragma unroll
            for (int k = 0; k < 4; ++k) rr[k] = *(const u32x2*)(r1g + pix * a.ldr1 + nb + 8 * k);
          }
          if constexpr (FAST == 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              rg[k] = *(const u32x2*)(gg + pix * a.ldg + nb + 8 * k);
              r2v[k] = *(const u32x2*)(r2g + pix * a.ldr2 + nb + 8 * k);
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const floatx4 bv = *(const floatx4*)(sbias + nloc + 8 * k + 4 * lh);
          float w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = acc[i][j][4 * k + e] + bv[e];
          if (act == LIC_ACT_LRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : w[e] * slope;
          } else if (act == LIC_ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : 0.f;
          } else if (BN == 96 && act == LIC_ACT_GELU) {   // (ResidualBottleneck's 3x3; 4 tiles a wave)
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = gelu_f(w[e]);
          }
          if (r1g) {
            const T* re = (const T*)&rr[k];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] += to_f(re[e]);
          }
          if constexpr (FAST == 2) {   // gate: g * sigmoid(.) + r2
            const T* ge = (const T*)&rg[k];
            const T* r2e = (const T*)&r2v[k];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = to_f(ge[e]) * sigmoid_f(w[e]) + to_f(r2e[e]);
          }
          u32x2 raw;
          T* o = (T*)&raw;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = from_f<T>(w[e]);
          *(u32x2*)(stg + l32 * SP + (i * 32 + 8 * k + 4 * lh) * 2) = raw;
        }
      });
      wave_lds_sync();
      constexpr int NCH = CT * 4;   // 16-B chunks of a pixel's CT*32 channels
#pragma unroll
      for (int h = 0; h < (32 * NCH) / 64; ++h) {
        const int idx = lane + 64 * h, pr = idx / NCH, c = idx - pr * NCH;
        const u32x4 val = *(const u32x4*)(stg + pr * SP + c * 16);
        const int col = j0 + pr;
        if (row < a.mi && col < a.mj && !(C16_ABL & 1)) {
          const int64_t pix = ((int64_t)b * a.ho + a.oy0 + a.osy * row) * a.wo + a.ox0 + a.osx * col;
          const int n = n0 + wc * Geo::WCH + c * 8;
          *(u32x4*)(yg + pix * a.ldy + n) = val;
          if (y2g) *(u32x4*)(y2g + pix * a.ldy2 + n) = val;
        }
      }
      wave_lds_sync();
    });
  } else {
    // (plain and + r1 only: the gate has its register variant, the rest is rare -- scalar)
    c16_epilogue<T, CT * PJ, CT, 0, 3>(a, ct, rowpix + wr * PJ * 32, n0 + wc * Geo::WCH, sbias + wc * Geo::WCH, lane,
                                       stage_tile);
  }
#if C16_STAMP
  C16T(t_end);
  if (tid == 0) {
    unsigned long long* o = (unsigned long long*)((T*)a.y + (size_t)a.n * a.ho * a.wo * a.ldy) +
                             ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
    o[0] = t_loop - t_begin;
    o[1] = sum_comp;
    o[2] = sum_wait;
    o[3] = t_end - t_loop - sum_comp - sum_wait;   // epilogue (+ stage bookkeeping)
    o[4] = t_end - t_begin;
    o[5] = __smid();
  }
#endif
}

// The register epilogue: 1 = plain or + r1 (PLAIN), 2 = the gate (GATE with g, r1, r2); activation none /
// relu / lrelu, and GELU on the 96-channel blocks (its erf would bloat the 12-tile variants), outputs 16-B aligned with rows of whole 16-B chunks, operands
// 8-B aligned, whole 32-channel tiles, no pixel shuffle.  0: the shared epilogue.
inline int c16_fast_epi(const lic_conv_args& a, int esz, bool gelu_ok) {
  auto al = [&](const void* ptr, int ld) { return ptr == nullptr || (((uintptr_t)ptr & 15) == 0 && (ld * esz) % 16 == 0); };
  auto al8 = [&](const void* ptr, int ld) { return ptr == nullptr || (((uintptr_t)ptr & 7) == 0 && (ld * esz) % 8 == 0); };
  const int m = c16_epi_mask_host(a);
  if (!(a.out_shuffle == 0 && a.co == a.copad &&
        (a.act == LIC_ACT_NONE || a.act == LIC_ACT_RELU || a.act == LIC_ACT_LRELU || (gelu_ok && a.act == LIC_ACT_GELU)) &&
        al(a.y, a.ldy) && al(a.y2, a.ldy2) && al8(a.r1, a.ldr1) && al8(a.g, a.ldg) && al8(a.r2, a.ldr2)))
    return 0;
  if ((m == 0 || m == EPI_R1) && a.epi == LIC_EPI_PLAIN) return 1;
  if (m == (EPI_G | EPI_R1 | EPI_R2) && a.epi == LIC_EPI_GATE) return 2;
  return 0;
}

// Returns 1 and launches when the conv16 kernel applies; 0 to let the caller fall back.
template <typename T, int KH, int KW, int S, int G, int BN, int WN>
int try_conv16(const lic_conv_args& a, hipStream_t s, int& status) {
  using Geo = C16Geo<KH, KW, S, G, BN, WN>;
  if (a.ntaps != KH * KW || a.copad % BN || a.isy != S || a.isx != S) return 0;
  if (a.prologue != LIC_PRO_NONE || a.groups != 1 || !c16_epi_supported(a)) return 0;
  if (a.ci != a.cpad || a.cpad % 16 || a.ldx % 8 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt % 16)) return 0;
  // unit-spaced tap grid KH x KW in row-major order
  for (int t = 0; t < a.ntaps; ++t)
    if (a.dy[t] != a.dy[0] + t / KW || a.dx[t] != a.dx[0] + t % KW) return 0;
  const int64_t xbytes = ((int64_t)a.n * a.h * a.w - 1) * a.ldx * 2 + (int64_t)a.ci * 2;
  const int64_t wbytes = (int64_t)a.copad * a.ntaps * a.cpad * 2;
  if (xbytes >= (1LL << 31) || wbytes >= (1LL << 31) || (int64_t)a.n * a.ho * a.wo >= (1LL << 31)) return 0;
  C16Plan p;
  p.dymin = a.dy[0];
  p.dxmin = a.dx[0];
  p.tiles_y = (a.mi + Geo::TH - 1) / Geo::TH;
  p.tiles_x = (a.mj + Geo::TW - 1) / Geo::TW;
  p.nchunks = a.cpad / 16;
  p.xrec = (unsigned)xbytes;
  p.wrec = (unsigned)wbytes;
  p.nst = p.nchunks * Geo::NG;
  p.fast_epi = wd_env("LIC_C16_FAST_EPI", 1) ? c16_fast_epi(a, 2, BN == 96) : 0;
  p.frag = c16_frag_ok(a) ? 1 : 0;
  c16_wstrides(a, p);
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / BN);
  auto kern = p.fast_epi == 1 ? conv16_kernel<T, KH, KW, S, G, BN, WN, 1> : conv16_kernel<T, KH, KW, S, G, BN, WN, 0>;
  if (p.fast_epi == 2) kern = conv16_kernel<T, KH, KW, S, G, BN, WN, 2>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, Geo::SMEM);
  if (ea != hipSuccess) {
    status = fail(std::string("conv16: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return 1;
  }
  hipLaunchKernelGGL(kern, grid, dim3(Geo::NT), Geo::SMEM, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("conv16 launch: ") + hipGetErrorString(e));
  return 1;
}

}  // namespace lic

#include "conv16s.h"

namespace lic {

// Tile choice of the conv16 kernels (16-bit): conv16 for stride-1 3x3 and stride-2 5x5 on output maps
// with >= 16 x 32 pixels and enough tiles to fill the chip; conv16s for stride-1 3x3 / 7x7 on the
// maps conv16 does not fill (the 16 x 16 latents).  LIC_CONV16=0 restores the halo kernel (A/B);
// LIC_CONV16S=0 keeps small maps on it, =2 takes conv16s wherever it applies (A/B).
template <typename T>
int conv16_dispatch_impl(const lic_conv_args& a, hipStream_t s, int& status) {
  static const int on = wd_env("LIC_CONV16", 1);
  static const int small_on = wd_env("LIC_CONV16S", 1);
  if (!on || a.force_mfma_generic || a.force_direct) return 0;
  auto blocks = [&](int bn) { return (int64_t)a.n * ((a.mi + 15) / 16) * ((a.mj + 31) / 32) * (a.copad / bn); };
  const bool big = a.mi >= 16 && a.mj >= 32 && small_on != 2;
  // 1x1 on small maps (after gemm16 declined: K not 96 / 192 or < 4 K pixels), e.g. the slice loop's
  // 128-channel Linears at 16x16: 4 x 16-pixel tiles x 32 channels, K split over the 4 waves, instead of
  // the generic kernel's 64-pixel x 128-channel tiles (32 workgroups at 2 K pixels).  A/B: LIC_CONV16S_1X1=0
  if (a.ntaps == 1) {
    static const int on1 = wd_env("LIC_CONV16S_1X1", 1);
    if (!on1 || !small_on || a.isy != 1 || a.isx != 1 || a.dy[0] != 0 || a.dx[0] != 0 || a.copad % 32 ||
        (int64_t)a.n * a.mi * a.mj > 8192)
      return 0;
    const int64_t sb1 = (int64_t)a.n * ((a.mi + 3) / 4) * ((a.mj + 15) / 16) * (a.copad / 32);
    if (sb1 > 2048 && a.copad % 64 == 0 && try_conv16s<T, 1, 1, 2>(a, s, status)) return 1;
    return try_conv16s<T, 1, 1, 1>(a, s, status);
  }
  if (a.isy == 1 && a.isx == 1) {
    if (a.ntaps == 9 && big) {
      if (a.copad % 192 == 0 && blocks(192) >= 128) return try_conv16<T, 3, 3, 1, 9, 192, 2>(a, s, status);
      if (a.copad % 96 == 0 && blocks(96) >= 128) return try_conv16<T, 3, 3, 1, 9, 96, 1>(a, s, status);
    }
    // 7x7: one tap row per stage (7 stages per chunk).  With the unrolled epilogue of round 5's first
    // version the 7 tap-column bases next to 12 accumulator tiles spilled 536 VGPRs (1.9 ms against the
    // halo kernel's 0.40); with the compact epilogues 18.  A/B: LIC_CONV16_7X7=0 (halo kernel)
    if (a.ntaps == 49 && big && a.copad % 192 == 0 && blocks(192) >= 128 && wd_env("LIC_CONV16_7X7", 1))
      return try_conv16<T, 7, 7, 1, 7, 192, 2>(a, s, status);
    const bool small_map = !(a.mi >= 16 && a.mj >= 32 && blocks(96) >= 128);
    if (small_on && (small_map || small_on == 2) && (a.ntaps == 9 || (a.ntaps == 49 && small_map))) {
      auto sblocks = [&](int ct) { return (int64_t)a.n * ((a.mi + 3) / 4) * ((a.mj + 15) / 16) * (a.copad / (32 * ct)); };
      if (a.ntaps == 49) return a.copad % 96 == 0 && try_conv16s<T, 7, 7, 3>(a, s, status);
      // 32-channel blocks (more, smaller workgroups: up to three per CU) unless that re-reads the halo of a
      // big grid too often: 3x3 192->192 @16^2 B=32 19.2 -> 17.4 us, 224->128 13.3 -> 12.3 (r05za).
      // A/B: LIC_C16S_CT=1/2/3 forces the channel tiles per workgroup
      // a candidate that declines (LDS or alignment) falls through to the next one
      static const int force_ct = wd_env("LIC_C16S_CT", 0);
      if ((force_ct == 1 || (force_ct == 0 && sblocks(1) <= 2048)) && a.copad % 32 == 0 &&
          try_conv16s<T, 3, 3, 1>(a, s, status)) return 1;
      if (force_ct == 2 && a.copad % 64 == 0 && try_conv16s<T, 3, 3, 2>(a, s, status)) return 1;
      if (a.copad % 96 == 0 && sblocks(3) >= 128 && try_conv16s<T, 3, 3, 3>(a, s, status)) return 1;
      if (a.copad % 64 == 0 && sblocks(2) >= 128 && try_conv16s<T, 3, 3, 2>(a, s, status)) return 1;
      if (a.copad % 32 == 0 && try_conv16s<T, 3, 3, 1>(a, s, status)) return 1;
    }
  }
  if (a.mi < 16 || a.mj < 32) return 0;
  // ResidualBlockWithStride's conv3x3 s2 (64^2 -> 32^2 in the a_model): four input-parity phases
  // (2x2 / 2x1 / 1x2 / 1x1 taps); 96-channel blocks where 192 leave the chip half empty
  if (a.isy == 2 && a.isx == 2 && a.ntaps == 9 && wd_env("LIC_CONV16_S2", 1)) {
    if (a.copad % 192 == 0 && blocks(192) >= 128) return try_conv16<T, 3, 3, 2, 0, 192, 2>(a, s, status);
    if (a.copad % 96 == 0 && blocks(96) >= 128) return try_conv16<T, 3, 3, 2, 0, 96, 1>(a, s, status);
  }
  // ZeroPad2d((1,2,1,2)) + conv5x5 s2 (the a_model's downsampling convs): four input-parity phases
  if (a.isy == 2 && a.isx == 2 && a.ntaps == 25 && a.copad % 192 == 0 && blocks(192) >= 128 &&
      wd_env("LIC_CONV16_S2", 1))
    return try_conv16<T, 5, 5, 2, 0, 192, 2>(a, s, status);
  return 0;
}

}  // namespace lic
