// fp32 convolutions on the 16-bit matrix cores, "weights-direct" form (lic_conv_args.mfma_mode 2
// fp32x6 / 1 fp32x3; split arithmetic and packed-weight layout: conv_split.h).
//
// Why a second split kernel.  conv_halo_split.hip stages everything through LDS behind one
// workgroup-wide barrier per weight stage (LDS-DMA of the fp32 halo and of [G taps][BN][parts]
// weight stages, a split pass between barriers, one 160 KB workgroup per CU): on gfx950 the
// fp32x6 3x3 192->192 conv at 64^2 spent 495 us against 300 us for its bare MFMA stream
// (ablations, profiles/r03/split_ablation.txt: DMA 75 us, split 42, fragment reads 27, epilogue 25,
// none of it overlapped with MFMAs).  Here:
//   * weights never touch LDS: they are packed in MFMA-fragment order, so each wave loads its B
//     fragments for the next (chunk, tap) step straight from L2 into VGPRs (one contiguous 1 KB
//     global_load_dwordx4 per fragment) while the current step's MFMAs run -- no weight barrier;
//   * the fp32 halo of the NEXT chunk is prefetched into registers (16 B per thread and quad) a
//     whole chunk ahead, split in registers and written to the other of two LDS plane sets
//     after the current chunk's taps: ONE barrier per 16-channel chunk;
//   * the LDS footprint (two plane sets of the halo, 16 bits x parts) fits two workgroups per CU,
//     so one workgroup's split / barrier / epilogue overlaps the other's MFMAs.
// Per wave and step: TM x NPA fragment reads from LDS (ds_read_b128) and TN x NPB 1 KB weight
// loads for NPROD x TM x TN MFMAs (fp32x6, TM = 4, TN = 1: 12 reads + 3 loads per 24 MFMAs).
#pragma once
#include "conv_halo.h"
#include "conv_split.h"
#include <type_traits>

// odd channel chunks are split from -x and the running sum flips sign at every chunk start: the
// 16-bit MFMA's accumulation rounding is biased toward -inf and the two halves cancel
// diagnostic ablations (-DWD_ABL=bits, timing only; outputs are wrong): 1 no in-loop split / halo
// prefetch, 2 no in-loop B loads, 4 no in-loop A reads, 8 no epilogue, 16 no MFMA
#ifndef WD_ABL
#define WD_ABL 0
#endif
#ifndef WD_SB
#define WD_SB 0
#endif
// cache policy of the halo loads (2 = nt: the activations are streamed once, the weight fragments
// that every workgroup re-reads should stay in L2)
#ifndef WD_HALO_AUX
#define WD_HALO_AUX 0
#endif
#ifndef WD_ALT
#define WD_ALT 1
#endif
// two-slot B rings (R = 2): each weight part of step s + 2 is loaded right after this step's last product
// that reads the part (w2 after the 3rd product, w1 after the 5th, w0 after the 6th) into the slot it
// frees, instead of all parts of step s + 1 at the top of the step: the same registers, up to two steps
// of latency (0: the old order, A/B)
#ifndef WD_LATE_B
#define WD_LATE_B 1
#endif
// with WD_LATE_B: part 0 (read first in a step, last used by its final product) gets a third slot and is
// loaded two steps ahead at the top of each step, where the step count per loop trip allows a static slot
// (measured neutral, r06u: 3x3 @64^2 353.5 -> 355.3 us, off)
#ifndef WD_W0R3
#define WD_W0R3 0
#endif

namespace lic {

struct WdPlan {
  int hh, hw, hpix;          // halo rows, cols, pixels
  int plane_bytes, set_bytes;// one 16-bit plane (32 B per halo pixel), NPA planes
  int dbuf;                  // two plane sets (always: the next chunk is split during this one)
  int tiles_y, tiles_x;
  int toff0, nx, ystep, xstep;  // tap grid: tap t at halo offset toff0 + (t/nx)*ystep + (t%nx)*xstep
  int dymin, dxmin;
  int hsy, hsx;              // halo sampling stride: 2 when the launch's taps share one parity at
                             // input stride 2 (a stride-2 conv's phase, conv.hip), else 1
  int rp_off;                // byte offset of rowpix[BM] + bias[BN]
  int nchunks;
  int ncb;                   // > 0: XCD-aware 1-D grid of (tile, channel block) pairs, ncb channel blocks
};

// VT > 0: a 1x1 convolution whose NTAPS = VT "virtual taps" are VT consecutive 16-channel chunks
// staged together (one barrier per VT chunks; the halo is the tile itself, VT blocks of BM pixels).
// Occupancy: two waves per SIMD, four for the one-tile-per-wave small-map configurations (TM = TN = 1).
// GEO 1: a plain K x K launch on a unit tap grid in halo coordinates (K = 3 or 7 at stride 1, or a
// stride-2 input-parity phase whose halo samples every other row / column; KXT: rectangular grids;
// halo (TH+KY-1) x (TW+KX-1), ci a multiple of 16, no prologue), or a virtual-tap 1x1 (VT > 0, ci a multiple of the chunk).  Its addressing is compile-time: the halo's LDS swizzle flips the 16-B half by halo ROW
// parity (conflict-free for 16-wide tiles: a wave's 32 rows are two tile rows, and ds_read_b128's lane
// groups then take complementary halves), so a tap's A-fragment address is a per-lane base chosen by
// the tap row's parity (compile-time) plus a compile-time immediate, and every halo quad's global and
// LDS offsets are computed once per workgroup (the chunk advances a scalar offset): the per-read
// address VALU of the general path (~5 per ds_read, half of the kernel's vector instructions,
// profiles/r03/wd_ablation_pmc.txt) is gone.
// OCC: waves per SIMD the registers are budgeted for (0: four for the one-tile-per-wave small-map
// configurations, else two); RF: B-ring slots (0: by the tap count, below).
// KS = 2: two tap groups ("tap split").  The workgroup has 2 x WM x WN waves; group g runs taps
// [T0, TE) (the first / second half of the tap grid) of every chunk on its own accumulators, both
// groups share the chunk's halo planes, its split work and its barrier, and group 1 hands its sums
// to group 0 through LDS at the end (one add per accumulator).  Each wave's dependent MFMA chain is
// half as long and the launch has twice the waves: for latency-bound grids (the 16x16 latents of the
// slice loop, fewer workgroups than the GPU holds) that is what bounds the step.
template <int MODE, int NTAPS, int TH, int TW, int BN, int WM, int WN, int NQ, int VT = 0, int GEO = 0, int KXT = 0,
          int OCC = 0, int RF = 0, int KS = 1>
__global__ __launch_bounds__(KS * WM * WN * 64, OCC > 0 ? OCC : ((TH * TW / WM == 32 && BN / WN == 32) ? 4 : 2)) void conv_split_wd_kernel(
    const lic_conv_args a, const WdPlan p) {
  using SM = SplitMode<MODE>;
  using T = typename SM::T;
  constexpr int NPA = SM::NPA, NPB = SM::NPB, NPROD = SM::NPROD;
  constexpr int NT = KS * WM * WN * 64;
  constexpr int BM = TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(KS == 1 || (KS == 2 && GEO == 1 && VT == 0 && NTAPS >= 2 && TM * TN <= 4),
                "tap groups: compile-time tap grids, accumulators staged whole");
  constexpr int CSTEP = 16 * (VT > 0 ? VT : 1);   // input channels per chunk
  static_assert(WTM % 32 == 0 && WTN % 32 == 0 && NT % 4 == 0, "tile");
  static_assert(VT == 0 || VT == NTAPS, "virtual taps");
  // every accumulator tile staged before the epilogue when that fits the plane sets (TM*TN <= 4)
  constexpr bool EPI_ALL = TM * TN <= 4;
  // LDS plane geometry is compile-time (every quad's pixel has a slot): the part offsets fold into
  // the ds_read / ds_write immediate offsets
  constexpr int PLANE = NQ * (NT / 4) * 32, SET = NPA * PLANE;
  constexpr bool FIX = GEO == 1;
  // FIX: LDS row stride of the halo in pixel slots; 8-wide tiles pad the 10-px rows to 12 so that the
  // four tile rows a wave's 32 lanes span land on complementary bank halves (row parity swizzle)
  // (16-wide tiles: any row stride; a row's 16 lanes cover 8 consecutive columns -> all 8 bank groups)
  // tap grid KY x KX (KXT > 0: KX = KXT, the rectangular transposed-conv phases; else square)
  constexpr int KK = KXT > 0 ? KXT : (NTAPS == 49 ? 7 : (NTAPS == 4 ? 2 : 3));
  constexpr int KY = NTAPS / KK;
  constexpr bool FIXK = FIX && VT == 0;   // KY x KX grid; FIX && VT > 0: virtual-tap 1x1
  constexpr int RS = TW == 8 ? 12 : TW + KK - 1;
  static_assert(!FIXK || (KY * KK == NTAPS && (TW == 16 || (TW == 8 && KK <= 3))), "GEO 1: tap grid");
  static_assert(!FIXK || (TH + KY - 1) * RS <= NQ * (NT / 4), "GEO 1: halo slots");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* rowpix = (int*)(smem + p.rp_off);
  float* sbias = (float*)(rowpix + BM);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
  const int kg = KS > 1 ? wave / (WM * WN) : 0;           // tap group
  const int wl = KS > 1 ? wave - kg * (WM * WN) : wave;   // wave within the group
  const int wm = wl / WN, wn = wl % WN;
  const int lrow = lane & 31, lhalf = lane >> 5;

  // XCD-aware order (p.ncb > 0): workgroups are dealt round-robin to the 8 XCDs, so id, id + 8, ...
  // share an L2; they take the ncb channel blocks of one tile in turn, and the halo each block
  // re-reads is then an L2 hit instead of a second trip to HBM
  int bid = blockIdx.x, cb = blockIdx.y;
  if (p.ncb > 0) {
    const int q = (int)blockIdx.x >> 3, t8 = q / p.ncb;
    cb = q - t8 * p.ncb;
    bid = t8 * 8 + ((int)blockIdx.x & 7);
  }
  const int tx_t = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty_t = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int n0 = cb * BN;
  const int i0 = ty_t * TH, j0 = tx_t * TW;
  const int iy0 = i0 * a.isy + p.dymin, ix0 = j0 * a.isx + p.dxmin;

  for (int n = tid; n < BN; n += NT) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
  for (int m = tid; m < BM; m += NT) {
    const int i = i0 + m / TW, j = j0 + m % TW;
    int base = -1;
    if (i < a.mi && j < a.mj) {
      int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
      if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
      base = (b * a.ho + oy) * a.wo + ox;
    }
    rowpix[m] = base;
  }

  const float* __restrict__ xg = (const float*)a.x;
  const int nchunks = p.nchunks;
  const int nsteps = nchunks * NTAPS;
  const int pro = a.prologue;

  // Every load below is unconditional (clamped indices, zero-selects): a load under a branch makes
  // the compiler's wait-count merge assume it was skipped, and the next wait then drains the whole
  // in-order vmcnt queue -- each step would wait for its own prefetch.
  // halo quads of this thread: pixel hp = (tid >> 2) + i * NT/4, channels 4c4 .. 4c4+3 of the chunk
  const int c4 = tid & 3;
  // halo pixel -> (row, col) by a float reciprocal (exact for hp < 2^16 and hw < 2^10)
  const float inv_hw = 1.0f / (float)p.hw;
  // element offset of quad i's pixel at channel 4c4 (+ its virtual tap's 16-channel block), -1 = zero;
  // cq = the quad's channel within the chunk
  auto quad_off = [&](int i, int& cq) -> int {
    int tv = tid;
    asm volatile("" : "+v"(tv));   // opaque: recomputed per chunk, not hoisted out of the loop and spilled
    const int hp = (tv >> 2) + i * (NT / 4);
    int iy, ix;
    if constexpr (VT > 0) {
      const int sub = hp / BM, m = hp - sub * BM;
      iy = iy0 + (m / TW) * a.isy;
      ix = ix0 + (m % TW) * a.isx;
      cq = sub * 16 + c4 * 4;
    } else {
      const int r = (int)(((float)hp + 0.5f) * inv_hw), cc = hp - r * p.hw;
      iy = iy0 + r * p.hsy;
      ix = ix0 + cc * p.hsx;
      cq = c4 * 4;
    }
    const bool ok = hp < p.hpix && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    return ok ? ((b * a.h + iy) * a.w + ix) * a.ldx + cq : -1;
  };
  // raw buffer loads: an out-of-range offset reads zeros (padding / out-of-image pixels) with no
  // branch and no select the compiler could turn back into a conditional load
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xg, (short)0, (int)((int64_t)a.n * a.h * a.w * a.ldx * 4), 0x00020000);
  u32x4 hreg[NQ];
  // FIX: per-quad byte offsets, once per workgroup (global: -> 0x80000000 = reads zeros; LDS: row-parity swizzle)
  unsigned qv[FIX ? NQ : 1];
  int ql[FIX ? NQ : 1];
  if constexpr (FIX) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int hp = (tid >> 2) + i * (NT / 4);   // LDS slot
      if constexpr (FIXK) {
        const int r = hp / RS, cc = hp - r * RS;
        const int iy = iy0 + r * p.hsy, ix = ix0 + cc * p.hsx;   // (a stride-2 phase samples every other row / column)
        const bool ok = r < TH + KY - 1 && cc < TW + KK - 1 && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
        qv[i] = ok ? (unsigned)((((b * a.h + iy) * a.w + ix) * a.ldx + c4 * 4) * 4) : 0x80000000u;
        ql[i] = hp * 32 + (((c4 >> 1) ^ (r & 1)) << 4) + (c4 & 1) * 8;
      } else {   // virtual taps: block `sub` of BM tile pixels carries channels 16 sub .. of the chunk
        const int sub = hp / BM, m = hp - sub * BM;
        const int iy = iy0 + (m / TW) * a.isy, ix = ix0 + (m % TW) * a.isx;
        const bool ok = hp < p.hpix && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
        qv[i] = ok ? (unsigned)((((b * a.h + iy) * a.w + ix) * a.ldx + sub * 16 + c4 * 4) * 4) : 0x80000000u;
        ql[i] = hp * 32 + (((c4 >> 1) ^ ((hp >> 3) & 1)) << 4) + (c4 & 1) * 8;
      }
    }
  }
  auto load_quad = [&](int i, int k) {
    if constexpr (FIX) {
      hreg[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, qv[i], k * CSTEP * 4, WD_HALO_AUX);
      return;
    }
    int cq;
    const int q = quad_off(i, cq);
    const unsigned off = (q >= 0 && k * CSTEP + cq < a.ci) ? (unsigned)(q + k * CSTEP) * 4u : 0x80000000u;
    hreg[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, WD_HALO_AUX);
  };
  // every quad stores (plane_bytes covers NQ * NT/4 pixels): no per-lane branch around the stores
  // sg: the chunk's sign (odd chunks are split from -x); compile-time where the chunk parity is
  auto split_quad = [&](int i, float sg, char* set) {
    const int hp = (tid >> 2) + i * (NT / 4);
    uint2 parts[NPA];
    const u32x4 h = hreg[i];
    split4<MODE>(make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z), __uint_as_float(h.w)),
                 FIXK ? (int)LIC_PRO_NONE : pro, sg, parts);
    const int off = FIX ? ql[i] : hp * 32 + (((c4 >> 1) ^ ((hp >> 3) & 1)) << 4) + (c4 & 1) * 8;
#pragma unroll
    for (int pl = 0; pl < NPA; ++pl) *(uint2*)(set + pl * PLANE + off) = parts[pl];
  };

  int hbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mm = wm * WTM + i * 32 + lrow;
    const int ty = mm / TW, tx = mm % TW;
    hbase[i] = VT > 0 ? mm : ty * (a.isy / p.hsy) * p.hw + tx * (a.isx / p.hsx);
  }
  // per-chunk opaque copy of hbase: the per-tap fragment addresses are then computed in the chunk,
  // not hoisted out of the chunk loop as NTAPS x TM live registers (which spilled)
  int hb[TM];
  // FIX: per-lane A bases by tap-row parity s (lane's halo pixel of tap (0,0), half lhalf ^ row parity)
  int abase[FIX ? 2 : 1][TM], ab[FIX ? 2 : 1][TM];
  if constexpr (FIX) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mm = wm * WTM + i * 32 + lrow, ty = mm / TW, tx = mm % TW;
      if constexpr (FIXK) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) abase[sp][i] = (ty * RS + tx) * 32 + ((lhalf ^ ((ty + sp) & 1)) << 4);
      } else {   // virtual tap t at slot t * BM + mm: the bit-3 swizzle of mm (BM is a multiple of 16)
        abase[0][i] = abase[1][i] = mm * 32 + ((lhalf ^ ((mm >> 3) & 1)) << 4);
      }
    }
  }
  // part pl of the A fragments of the tap at halo offset `toff` (scalar tap cursor, see chunk);
  // FIX: `toff` is the compile-time tap index
  auto load_a_part = [&](const char* set, int toff, int pl, u32x4(&fa)[NPA][TM]) {
    if constexpr (FIXK) {
      const int ty = toff / KK, tx = toff - ty * KK;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[pl][i] = *(const u32x4*)(smem + ab[ty & 1][i] + ((ty * RS + tx) * 32 + pl * PLANE));
      return;
    } else if constexpr (FIX) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[pl][i] = *(const u32x4*)(smem + ab[0][i] + (toff * BM * 32 + pl * PLANE));
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int hp = hb[i] + toff;
      const int o = hp * 32 + ((lhalf ^ ((hp >> 3) & 1)) << 4);
      fa[pl][i] = *(const u32x4*)(set + pl * PLANE + o);
    }
  };
  // B fragments of step s = chunk * NTAPS + tap (clamped): n-tile (n0/32 + wn*TN + j), 1 KB per part,
  // by raw buffer loads whose only vector offset is the lane's 16 B (fragment offsets are scalar);
  // n-tiles past the pack (copad not a multiple of BN) are clamped, their outputs masked
  const int ntiles = a.copad / 32;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wgt_split, (short)0, (int)((int64_t)ntiles * nsteps * NPB * 1024), 0x00020000);
  auto load_b = [&](int s, u32x4(&fb)[NPB][TN]) {
    s = s < nsteps ? s : nsteps - 1;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int jt = n0 / 32 + wn * TN + j;
      jt = jt < ntiles ? jt : ntiles - 1;
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        fb[pl][j] = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, ((jt * nsteps + s) * NPB + pl) * 1024, 0);
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // A: ONE register set; each part is re-read for the next tap right after this tap's last product
  // that reads it (products run smallest first, pr = NPROD-1 .. 0, so part NPA-1 is free after the
  // first group and part 0 is needed first only by the third), so the reads have most of a step
  // to land.  B: a ring of R slots by step, B(s+2) issued at step s (below, per tap group).
  u32x4 fa[NPA][TM];
  // one tap's products; the running sum is the MFMA's C operand.  `mid` runs after the first product
  // group: the next chunk's split work of this step, interleaved with the MFMAs by the scheduler
  // fb0c: part 0's slot when it has its own ring (w0r3), else unused (fbc[0] holds part 0)
  auto step = [&](const char* set, int toff_next, bool has_next, u32x4(&fbc)[NPB][TN], const u32x4(&fb0c)[TN],
                  auto w0r3, auto&& mid, auto&& after_b) {
    constexpr bool W0 = decltype(w0r3)::value;
#pragma unroll
    for (int pr = NPROD - 1; pr >= 0; --pr) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const u32x4& bop = (W0 && SM::PB[pr] == 0) ? fb0c[j] : fbc[SM::PB[pr]][j];
#if WD_ABL & 16
          acc[i][j][0] += __uint_as_float(fa[SM::PA[pr]][i][0] ^ bop[0]);
#else
          acc[i][j] = mfma_k16<T>(fa[SM::PA[pr]][i], bop, acc[i][j]);
#endif
        }
      bool last = true;   // the last product of this tap reading part PA[pr] (folded at compile time)
#pragma unroll
      for (int q = 0; q < pr; ++q) last = last && SM::PA[q] != SM::PA[pr];
#if !(WD_ABL & 4)
      if (has_next && last) load_a_part(set, toff_next, SM::PA[pr], fa);
#endif
      bool last_b = true;   // the last product of this tap reading weight part PB[pr] (compile-time)
#pragma unroll
      for (int q = 0; q < pr; ++q) last_b = last_b && SM::PB[q] != SM::PB[pr];
      if (last_b) after_b(SM::PB[pr]);
      if (pr == NPROD - 1) mid();
#if WD_SB
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
  };
  // chunk 0 split up front; chunk 1 in the prefetch registers
#pragma unroll
  for (int i = 0; i < NQ; ++i) load_quad(i, 0);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    split_quad(i, 1.f, smem);
    load_quad(i, 1 < nchunks ? 1 : 0);
  }

  // the chunk loop of tap group G (taps [T0, TE) of every chunk; KS = 1: all taps)
  auto run_group = [&](auto gi) {
    constexpr int G = decltype(gi)::value;
    constexpr int T1 = KS > 1 ? (NTAPS + 1) / 2 : NTAPS;
    constexpr int T0 = G == 0 ? 0 : T1, TE = G == 0 ? T1 : NTAPS;
    constexpr int NTG = TE - T0;   // taps per chunk of this group = its steps per chunk
    // B ring: R slots, B(l+PD) issued at the group's step l into slot (l+PD) % R.  R divides NTG
    // where it can (3 or 4), so every chunk starts at slot 0; else the chunk loop is unrolled by KU
    // (chunk k starts at slot (k*NTG) % R); an even count that 3 and 4 do not divide: two slots at
    // prefetch distance one
    constexpr int R = (KS == 1 && RF > 0) ? RF : ((NTG % 3 == 0) ? 3 : ((NTG % 4 == 0) ? 4 : ((NTG % 2 == 0) ? 2 : 3)));
    constexpr int PD = R == 2 ? 1 : 2;   // B prefetch distance in steps
    // chunks per loop trip: the smallest KU with KU * NTG a multiple of R
    constexpr int KU = (NTG % R == 0) ? 1 : ((2 * NTG) % R == 0 ? 2 : ((3 * NTG) % R == 0 ? 3 : 4));
    static_assert((KU * NTG) % R == 0, "B ring");
    u32x4 fb[R][NPB][TN];
    // the pack's step index of the group's step tl (compile-time) of chunk k (tl may run past the chunk)
    auto gstep = [&](int k, int tl) { return (k + tl / NTG) * NTAPS + T0 + tl % NTG; };
    constexpr bool LATE = WD_LATE_B && R == 2 && !(WD_ABL & 2);   // (R = 2: PD = 1)
    // one weight part of step s (clamped) into slot fb_s: n-tiles as load_b
    auto load_b_part = [&](int s, int pl, u32x4(&fbs)[NPB][TN]) {
      s = s < nsteps ? s : nsteps - 1;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int jt = n0 / 32 + wn * TN + j;
        jt = jt < ntiles ? jt : ntiles - 1;
        fbs[pl][j] = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, ((jt * nsteps + s) * NPB + pl) * 1024, 0);
      }
    };
    constexpr bool W0R3 = LATE && WD_W0R3 && (KU * NTG) % 3 == 0 && NQ <= 4;   // (NQ 6: 12 more registers spill)
    u32x4 fb0[W0R3 ? 3 : 1][TN];
    if constexpr (W0R3) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        load_b_part(gstep(0, q), 0, fb[q]);   // (slot's part 0 unused; only fills the registers' shape)
#pragma unroll
        for (int j = 0; j < TN; ++j) fb0[q][j] = fb[q][0][j];
        load_b_part(gstep(0, q), 1, fb[q]);
        load_b_part(gstep(0, q), 2, fb[q]);
      }
    } else if constexpr (LATE) {
      load_b(gstep(0, 0), fb[0]);
      load_b(gstep(0, 1), fb[1]);
    } else {
#pragma unroll
      for (int q = 0; q < PD; ++q) load_b(gstep(0, q), fb[q]);
    }
    __syncthreads();

    // one chunk; KSI = chunk index mod KU (compile-time), so the group's step (k, tl) sits in ring slot
    // (KSI*NTG + tl) % R.  During chunk k, step tl also splits halo quads [tl*QPS, (tl+1)*QPS) of chunk
    // k+1 (in the registers since chunk k-1) into the other plane set -- free since the barrier that
    // ended chunk k-1 -- and refills those registers with chunk k+2: the split's VALU work and its LDS
    // stores sit between this wave's MFMAs instead of in a serial phase before the barrier.
    constexpr int QPS = (NQ + NTG - 1) / NTG;
    // PAR: chunks unrolled in pairs so that a chunk's parity (its plane set, the next chunk's sign) is
    // a compile-time constant: the sign folds into the split's instructions, the set into LDS offsets
    constexpr bool PAR = FIX && KU == 1 && NTG <= 9 && TW == 8;   // (16-wide: the pair spills)
    auto chunk = [&](int k, auto ks, auto kpar) {
      constexpr int KSI = decltype(ks)::value;
      constexpr int KP = decltype(kpar)::value;   // k & 1 when >= 0
      const int kodd = KP >= 0 ? KP : (k & 1);
      const char* set = smem + kodd * SET;
      char* nset = smem + (kodd ^ 1) * SET;
      const float nsg = WD_ALT ? (kodd ? 1.f : -1.f) : 1.f;   // sign of chunk k + 1
      const int kn = k + 2 < nchunks ? k + 2 : nchunks - 1;
#if WD_ALT
      if (k > 0)   // exact sign flip: the running sum changes sign with the chunk's parts
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = -acc[i][j];
#endif
      int toff = FIX ? T0 : p.toff0, cx = 0;   // tap grid cursor (scalar; FIX: the tap index)
      if constexpr (FIX) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int i = 0; i < TM; ++i) ab[sp][i] = abase[sp][i] + kodd * SET;
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          hb[i] = hbase[i];
          asm volatile("" : "+v"(hb[i]));
        }
      }
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl) load_a_part(set, toff, pl, fa);
#pragma unroll
      for (int tl = 0; tl < NTG; ++tl) {
        const int sr = KSI * NTG + tl;
        // kept in this order by the scheduling barriers: the prefetches are issued before this
        // step's MFMAs (left to itself the scheduler sinks them next to their consumers)
#if !(WD_ABL & 2)
        if constexpr (!LATE) load_b(gstep(k, tl + PD), fb[(sr + PD) % R]);
        if constexpr (W0R3) {   // part 0 of step + 2 into the slot step - 1 freed
          u32x4(&d0)[TN] = fb0[(sr + 2) % 3];
          const int s2 = gstep(k, tl + 2) < nsteps ? gstep(k, tl + 2) : nsteps - 1;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            int jt = n0 / 32 + wn * TN + j;
            jt = jt < ntiles ? jt : ntiles - 1;
            d0[j] = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, ((jt * nsteps + s2) * NPB + 0) * 1024, 0);
          }
        }
#endif
        if constexpr (FIX) {
          toff = T0 + tl + 1;
        } else if (tl + 1 < NTG) {
          toff += p.xstep;
          if (++cx == p.nx) {
            cx = 0;
            toff += p.ystep - p.nx * p.xstep;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        auto& fbs = fb[sr % R];
        step(set, toff, tl + 1 < NTG, fbs, fb0[W0R3 ? sr % 3 : 0], std::integral_constant<bool, W0R3>{}, [&]() {
#if !(WD_ABL & 1)
#pragma unroll
          for (int i = tl * QPS; i < (tl + 1) * QPS && i < NQ; ++i) {
            split_quad(i, nsg, nset);
#if WD_ABL & 32   // diagnostic: always chunk 0 (L2-resident): separates HBM latency from the split work
            load_quad(i, 0);
#else
            load_quad(i, kn);
#endif
          }
#endif
        }, [&](int pl) {
          // slot sr % 2 held this step's part pl; step sr + 2 uses the same slot
          if constexpr (LATE) {
            if (!(W0R3 && pl == 0)) load_b_part(gstep(k, tl + 2), pl, fbs);
          }
        });
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
    };
    using NOPAR = std::integral_constant<int, -1>;
    if constexpr (PAR) {
      for (int k = 0; k < nchunks; k += 2) {
        chunk(k, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        if (k + 1 >= nchunks) break;
        chunk(k + 1, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
      }
    } else {
      for (int k = 0; k < nchunks; k += KU) {
        chunk(k, std::integral_constant<int, 0>{}, NOPAR{});
        if constexpr (KU >= 2) {
          if (k + 1 >= nchunks) break;
          chunk(k + 1, std::integral_constant<int, 1>{}, NOPAR{});
        }
        if constexpr (KU >= 3) {
          if (k + 2 >= nchunks) break;
          chunk(k + 2, std::integral_constant<int, 2>{}, NOPAR{});
        }
        if constexpr (KU >= 4) {
          if (k + 3 >= nchunks) break;
          chunk(k + 3, std::integral_constant<int, 3>{}, NOPAR{});
        }
      }
    }
  };
  if constexpr (KS == 1) {
    run_group(std::integral_constant<int, 0>{});
  } else {
    // (both groups pass the same barriers: one before the loop, one per chunk)
    if (kg == 0) run_group(std::integral_constant<int, 0>{});
    else run_group(std::integral_constant<int, 1>{});
  }

  // with WD_ALT an even chunk count leaves the running sum negated
  const float oscale = (WD_ALT && nchunks > 0 && !(nchunks & 1)) ? -SM::scale : SM::scale;
  constexpr int CTS = 32 * 33;
  if constexpr (KS > 1) {
    // tap group 1 hands its sums to group 0 (the plane sets are free after the last chunk's barrier;
    // the hand-over area lies past group 0's epilogue staging)
    float* red = (float*)smem + (WM * WN) * (EPI_ALL ? TM * TN : 1) * CTS + wl * (TM * TN * 16 * 64);
    if (kg == 1) {
#pragma unroll
      for (int qq = 0; qq < TM * TN; ++qq)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(qq * 16 + r) * 64 + lane] = acc[qq / TN][qq % TN][r];
    }
    __syncthreads();
    if (kg == 1) return;
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[qq / TN][qq % TN][r] += red[(qq * 16 + r) * 64 + lane];
  }
  if constexpr (EPI_ALL) {
    // every accumulator tile of the wave is staged in LDS first (the plane sets are free after the
    // last barrier): the accumulators are dead before the epilogue loads its operands
    float* ct = (float*)smem + wl * (TM * TN * CTS);
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ct[qq * CTS + ((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r] * oscale;
    auto stage = [&](int) {};
#if WD_ABL & 8
    if (ct[0] != 1234.5f) return;
#endif
    epilogue_all<float, TM * TN, TN, decltype(stage), CTS>(a, ct, rowpix + wm * WTM, n0 + wn * WTN, sbias + wn * WTN,
                                                            lane, stage);
  } else {
    float* ct = (float*)smem + wl * CTS;
    epilogue_all<float, TM * TN, TN>(a, ct, rowpix + wm * WTM, n0 + wn * WTN, sbias + wn * WTN, lane, [&](int q) {
#pragma unroll
      for (int qq = 0; qq < TM * TN; ++qq)
        if (qq == q) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ct[((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r] * oscale;
        }
    });
  }
}

template <int MODE, int NTAPS, int TH, int TW, int BN, int WM, int WN, int NQ, int VT = 0, int GEO = 0, int KXT = 0,
          int OCC = 0, int RF = 0, int KS = 1>
static int try_split_wd(const lic_conv_args& a, hipStream_t s, int& status) {
  constexpr int NT = KS * WM * WN * 64;
  constexpr int NPA = SplitMode<MODE>::NPA;
  if (a.ntaps != (VT > 0 ? 1 : NTAPS) || a.copad % 32 || a.cpad % (16 * (VT > 0 ? VT : 1)) || a.ci % 4 || a.ldx % 4 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt_split % 16))
    return 0;
  if ((int64_t)a.n * a.h * a.w * a.ldx >= (1LL << 31)) return 0;
  WdPlan p;
  int dymin = 1 << 20, dymax = -(1 << 20), dxmin = 1 << 20, dxmax = -(1 << 20);
  for (int t = 0; t < a.ntaps; ++t) {
    dymin = dymin < a.dy[t] ? dymin : a.dy[t];
    dymax = dymax > a.dy[t] ? dymax : a.dy[t];
    dxmin = dxmin < a.dx[t] ? dxmin : a.dx[t];
    dxmax = dxmax > a.dx[t] ? dxmax : a.dx[t];
  }
  p.dymin = dymin;
  p.dxmin = dxmin;
  // stride-2 input whose taps all share one row (column) parity: the halo samples every other row
  // (column) -- the rows of the other parity are never read
  bool ypar = a.isy == 2, xpar = a.isx == 2;
  for (int t = 0; t < a.ntaps; ++t) {
    ypar = ypar && ((a.dy[t] - dymin) & 1) == 0;
    xpar = xpar && ((a.dx[t] - dxmin) & 1) == 0;
  }
  p.hsy = ypar ? 2 : 1;
  p.hsx = xpar ? 2 : 1;
  p.hh = ((TH - 1) * a.isy + (dymax - dymin)) / p.hsy + 1;
  p.hw = ((TW - 1) * a.isx + (dxmax - dxmin)) / p.hsx + 1;
  p.hpix = p.hh * p.hw;
  if (((VT > 0 ? VT * TH * TW : p.hpix) + NT / 4 - 1) / (NT / 4) > NQ) return 0;   // more quads than NQ
  if ((int64_t)a.n * a.h * a.w * a.ldx * 4 >= (1LL << 31)) return 0;   // buffer-load byte offsets
  p.plane_bytes = NQ * (NT / 4) * 32;   // every quad's pixel, valid or not (unconditional stores)
  p.set_bytes = NPA * p.plane_bytes;
  int nx = 1;
  while (nx < a.ntaps && a.dy[nx] == a.dy[0]) ++nx;
  if (a.ntaps % nx) return 0;
  const int sy = a.ntaps > nx ? a.dy[nx] - a.dy[0] : 0;
  const int sx = nx > 1 ? a.dx[1] - a.dx[0] : 0;
  for (int t = 0; t < a.ntaps; ++t)
    if (a.dy[t] != a.dy[0] + (t / nx) * sy || a.dx[t] != a.dx[0] + (t % nx) * sx) return 0;
  p.toff0 = ((a.dy[0] - dymin) / p.hsy) * p.hw + (a.dx[0] - dxmin) / p.hsx;
  p.nx = nx;
  p.ystep = (sy / p.hsy) * p.hw;
  p.xstep = sx / p.hsx;
  if (VT > 0) {   // 1x1: VT blocks of the tile's BM pixels, virtual tap t = block t
    p.hpix = VT * TH * TW;
    p.toff0 = 0;
    p.nx = VT;
    p.xstep = TH * TW;
    p.ystep = 0;
  }
  static const bool geo_on = [] {
    const char* e = getenv("LIC_WD_GEO");
    return !(e && e[0] == '0');
  }();
  if (GEO == 1 && VT == 0) {
    constexpr int K = KXT > 0 ? KXT : (NTAPS == 49 ? 7 : (NTAPS == 4 ? 2 : 3));
    if (!geo_on || !(a.ntaps == NTAPS && nx == K && p.xstep == (K > 1 ? 1 : 0) && (NTAPS == K || p.ystep == p.hw) &&
                     p.hw == TW + K - 1 && p.hh == TH + NTAPS / K - 1 &&
                     p.hsy == a.isy && p.hsx == a.isx && p.toff0 == 0 && a.ci % 16 == 0 &&
                     a.prologue == LIC_PRO_NONE))
      return 0;
  }
  if (GEO == 1 && VT > 0 && (!geo_on || a.ci % (16 * VT) != 0)) return 0;
  p.tiles_y = (a.mi + TH - 1) / TH;
  p.tiles_x = (a.mj + TW - 1) / TW;
  p.nchunks = a.cpad / (16 * (VT > 0 ? VT : 1));
  const int tail = TH * TW * 4 + BN * 4;
  constexpr int TQ = (TH * TW / WM / 32) * (BN / WN / 32);   // accumulator tiles per wave
  // epilogue staging of the (group-0) waves, plus the tap groups' hand-over area
  const int epi_bytes = (WM * WN) * (TQ <= 4 ? TQ : 1) * 32 * 33 * 4 + (KS > 1 ? WM * WN * TQ * 16 * 64 * 4 : 0);
  // LDS plan: two plane sets when two workgroups still fit a CU, else one set at two per CU,
  // else the single-workgroup plans
  auto need = [&](int sets) { return (sets * p.set_bytes > epi_bytes ? sets * p.set_bytes : epi_bytes) + tail; };
  p.dbuf = 1;   // the next chunk is split during this one: always two plane sets
  if (need(2) > 160 * 1024) return 0;
  const int sets_bytes = (p.dbuf ? 2 : 1) * p.set_bytes;
  p.rp_off = sets_bytes > epi_bytes ? sets_bytes : epi_bytes;
  const int smem = p.rp_off + tail;
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  if ((int64_t)(a.copad / 32) * p.nchunks * NTAPS * SplitMode<MODE>::NPB * 1024 >= (1LL << 31)) return 0;
  const int ncb = (a.copad + BN - 1) / BN;
  static const bool remap_on = [] {
    const char* e = getenv("LIC_WD_XCD");
    return !(e && e[0] == '0');
  }();
  p.ncb = (remap_on && ncb > 1 && blocks % 8 == 0) ? ncb : 0;
  dim3 grid = p.ncb ? dim3((unsigned)(blocks * ncb), 1) : dim3((unsigned)blocks, ncb);
  auto kern = conv_split_wd_kernel<MODE, NTAPS, TH, TW, BN, WM, WN, NQ, VT, GEO, KXT, OCC, RF, KS>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, 160 * 1024);
  if (ea != hipSuccess) {
    status = fail(std::string("split wd conv: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return 1;
  }
  hipLaunchKernelGGL(kern, grid, dim3(NT), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("split wd conv launch: ") + hipGetErrorString(e));
  return 1;
}

// configuration groups, one translation unit each (conv_split_wd_{vt,small,big,7x7}.hip): each
// returns 1 and launches when one of its tiles applies
int wd_dispatch_vt(const lic_conv_args& a, hipStream_t s, int& status);      // 1x1 on big maps
int wd_dispatch_small(const lic_conv_args& a, hipStream_t s, int& status);   // 8x8-px tiles
int wd_dispatch_big(const lic_conv_args& a, hipStream_t s, int& status);     // 16x16-px tiles (not 7x7)
int wd_dispatch_7x7(const lic_conv_args& a, hipStream_t s, int& status);     // 7x7, 16x16-px tiles
int wd_env(const char* name, int def);   // integer environment switch (A/B and experiments), read once per name

}  // namespace lic
