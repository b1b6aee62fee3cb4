// fp32 convolutions on the 16-bit matrix cores ("split" MFMA modes, lic_conv_args.mfma_mode).
//
// The spatial-tile conv of conv_halo.h for fp32 activations, with every product formed from
// 16-bit parts on v_mfma_f32_32x32x16_{f16,bf16} instead of the 16x slower fp32-input MFMA.
//
// Split modes and the packed-weight layout: conv_split.h.
//
// Per 16-channel chunk the fp32 halo of the tile arrives by LDS-DMA in a staging buffer
// (double-buffered, the next chunk's DMA overlaps this chunk's MFMAs); all threads then
// split it once into NPA 16-bit planes laid out as the fp16 kernel's halo (32 B per pixel,
// halves XOR-swizzled), and every tap reads its shifted windows from the planes.  Weights
// stream as [G taps][BN][NPB planes x 32 B] stages by LDS-DMA (double buffer).
#include "conv_halo.h"
#include "conv_split.h"

namespace lic {

// SPLIT_PARTIAL: chain the products of one tap from zero and add the partial to the running sum
// with an fp32 VALU add (else the running sum is the MFMA's C operand).  SPLIT_ALT: odd channel
// chunks are split from -x and subtracted (see split_chunk).
#ifndef SPLIT_PARTIAL
#define SPLIT_PARTIAL 0
#endif
#ifndef SPLIT_ALT
#define SPLIT_ALT 1
#endif
#ifndef SPLIT_SMALL_2WG
#define SPLIT_SMALL_2WG 1
#endif
// diagnostic ablations (-DSPLIT_ABL=bits, timing only; outputs are wrong): 1 no in-loop LDS-DMA,
// 2 no epilogue, 4 no split pass, 8 no MFMA (one VALU op per product group), 16 no fragment reads
#ifndef SPLIT_ABL
#define SPLIT_ABL 0
#endif
// diagnostic builds: only the fp32x6 16x16x128 / 8x8x64 tiles (fast compile)
#ifndef SPLIT_DIAG_ONLY
#define SPLIT_DIAG_ONLY 0
#endif

template <int MODE, int TH, int TW, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void conv_halo_split_kernel(const lic_conv_args a, const HaloPlan p) {
  using SM = SplitMode<MODE>;
  using T = typename SM::T;
  constexpr int NPA = SM::NPA, NPB = SM::NPB;
  constexpr int NT = WM * WN * 64;
  constexpr int BM = TH * TW;
  constexpr int CK = 16;  // fp32 channels per chunk (64 B per pixel)
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int sbytes = p.hpix_pad * 64;   // fp32 staging of one chunk
  const int pbytes = p.hpix_pad * 32;   // one 16-bit plane
  const int wbytes = p.G * BN * NPB * 32;
  char* stg0 = smem;
  char* pl0 = smem + 2 * sbytes;        // NPA planes, pbytes apart
  char* wbuf0 = pl0 + NPA * pbytes;
  int* rowpix = (int*)(smem + p.rp_off);
  float* sbias = (float*)(rowpix + BM);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
  const int wm = wave / WN, wn = wave % WN;
  const int lrow = lane & 31, lhalf = lane >> 5;

  int bid = blockIdx.x;
  const int tx_t = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty_t = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int n0 = blockIdx.y * BN;
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
  const T* __restrict__ wg = (const T*)a.wgt_split;
  const int nchunks = a.cpad / CK;
  const int nst = nchunks * p.ngroups;
  const int hq_total = p.hpix_pad * 4;
  const int hpix = p.hh * p.hw;

  // fp32 halo of chunk k -> staging buffer `buf` (linear: pixel hp, 16-B piece c at hp*64 + c*16)
  auto issue_halo = [&](int k, int buf, int nw_ld) {
    const int c0 = k * CK;
    char* dst = stg0 + buf * sbytes;
    for (int q0 = wave * 64; q0 < hq_total; q0 += nw_ld * 64) {
      const int q = q0 + lane;
      const int hp = q >> 2, c = q & 3;
      const int r = hp / p.hw, cc = hp - r * p.hw;
      const int iy = iy0 + r, ix = ix0 + cc;
      const int ch = c0 + c * 4;
      const bool ok = hp < hpix && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w && ch < a.ci;
      const void* src = ok ? (const void*)(xg + ((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + ch)
                           : (const void*)g_lic_zero_page;
      glds16(src, dst + q0 * 16);
    }
  };
  // weights of stage s: 16-B slot (tt, n, sl) holds plane sl>>1, swizzled half sl&1
  auto issue_w = [&](int s, int buf, int nw_ld) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    const int total = gcur * BN * 2 * NPB;
    char* dst = wbuf0 + buf * wbytes;
    for (int q0 = wave * 64; q0 < total; q0 += nw_ld * 64) {
      const int q = q0 + lane;
      const int row = q / (2 * NPB), slot = q - row * (2 * NPB);
      const int tt = row / BN, n = row - tt * BN;
      const int piece = (slot & ~1) | ((slot & 1) ^ ((n >> 3) & 1));
      const int ng = n0 + n;   // fragment-order pack (conv_split.h): part piece>>1, lane (ng&31) + 32*(piece&1)
      const T* src = wg + split_frag_off(ng >> 5, k, t0 + tt, piece >> 1, nchunks, a.ntaps, NPB) +
                     ((ng & 31) + 32 * (piece & 1)) * 8;
      glds16(src, dst + q0 * 16);
    }
  };
  // staging -> NPA planes (32 B per pixel each, halves swizzled as the fp16 kernel).  The
  // 16-bit MFMA's internal rounding is biased toward -inf (tools/split_accuracy.py: mean error
  // -1.5e-8 of the output scale, exact-fp32 MFMA: 2e-10); with SPLIT_ALT the odd chunks are split
  // from -x and their partials subtracted, so the bias of the two halves cancels.
  auto split_chunk = [&](int buf, bool neg) {
    const char* src = stg0 + buf * sbytes;
    const float sg = neg ? -1.f : 1.f;
    for (int q = tid; q < hq_total; q += NT) {
      const int hp = q >> 2, c = q & 3;
      uint2 parts[NPA];
      split4<MODE>(*(const float4*)(src + q * 16), a.prologue, sg, parts);
      const int off = hp * 32 + (((c >> 1) ^ ((hp >> 3) & 1)) << 4) + (c & 1) * 8;
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl) *(uint2*)(pl0 + pl * pbytes + off) = parts[pl];
    }
  };

  int hbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mm = wm * WTM + i * 32 + lrow;
    const int ty = mm / TW, tx = mm % TW;
    hbase[i] = ty * a.isy * p.hw + tx * a.isx;
  }

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  if (nst > 0) {
    issue_halo(0, 0, NT / 64);
    issue_w(0, 0, NT / 64);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int s = 0; s < nst; ++s) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    if (g == 0) {  // a new chunk landed in staging[k & 1]: split it (all waves are past the last tap reads)
#if SPLIT_ALT && !SPLIT_PARTIAL
      if (k > 0)   // exact sign flip: the running sum changes sign with the chunk's planes
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = -acc[i][j];
#endif
#if !(SPLIT_ABL & 4)
      split_chunk(k & 1, SPLIT_ALT && (k & 1));
#endif
      __syncthreads();
    }
    constexpr int NL = HALO_LOADERS < NT / 64 ? HALO_LOADERS : NT / 64;
#if !(SPLIT_ABL & 1)
    if (wave < NL) {
      if (s + 1 < nst) issue_w(s + 1, (s + 1) & 1, NL);
      if (g == 0 && k + 1 < nchunks) issue_halo(k + 1, (k + 1) & 1, NL);
    }
#endif
    const char* wb = wbuf0 + (s & 1) * wbytes;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    int cy = t0 / p.nx, cx = t0 - cy * p.nx;
    auto load_frags = [&](int tt, u32x4(&fa)[NPA][TM], u32x4(&fb)[NPB][TN]) {
#if SPLIT_ABL & 16
      if (tt > 0) return;
#endif
      const int toff = p.toff0 + cy * p.ystep + cx * p.xstep;
      if (++cx == p.nx) {
        cx = 0;
        ++cy;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hp = hbase[i] + toff;
        const int o = hp * 32 + ((lhalf ^ ((hp >> 3) & 1)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) fa[pl][i] = *(const u32x4*)(pl0 + pl * pbytes + o);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WTN + j * 32 + lrow;
        const char* wr = wb + (tt * BN + n) * (NPB * 32) + ((lhalf ^ ((n >> 3) & 1)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl) fb[pl][j] = *(const u32x4*)(wr + pl * 32);
      }
    };
    // Per fragment and tap the NPROD products of 16 channels are chained from zero and added to
    // the running sum by one fp32 VALU add (round to nearest even): the 16-bit MFMA's own
    // accumulation rounding is biased (measured: mean error -7e-9 of the output scale when the
    // running sum is its C operand, tools/split_accuracy.py), and chaining it only over a partial
    // of 16 x NPROD terms shrinks that bias with the partial's magnitude.
    const bool negk = SPLIT_ALT && (k & 1);
    auto mfmas = [&](const u32x4(&fa)[NPA][TM], const u32x4(&fb)[NPB][TN]) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#if SPLIT_ABL & 8
          acc[i][j][0] += __int_as_float(fa[0][i][0] ^ fa[NPA - 1][i][1] ^ fb[0][j][0] ^ fb[NPB - 1][j][1]);
#elif SPLIT_PARTIAL
          floatx16 t = mfma_k16<T>(fa[SM::PA[SM::NPROD - 1]][i], fb[SM::PB[SM::NPROD - 1]][j], floatx16{});
#pragma unroll
          for (int pr = SM::NPROD - 2; pr >= 0; --pr)   // smallest terms first
            t = mfma_k16<T>(fa[SM::PA[pr]][i], fb[SM::PB[pr]][j], t);
          if (negk) acc[i][j] -= t;
          else acc[i][j] += t;
#else
          // running sum as C; it holds -sum through the odd chunks (flipped at chunk starts)
#pragma unroll
          for (int pr = SM::NPROD - 1; pr >= 0; --pr)
            acc[i][j] = mfma_k16<T>(fa[SM::PA[pr]][i], fb[SM::PB[pr]][j], acc[i][j]);
#endif
        }
    };
    u32x4 fa[2][NPA][TM], fb[2][NPB][TN];
    load_frags(0, fa[0], fb[0]);
    int tt = 0;
    for (; tt + 2 <= gcur; tt += 2) {
      load_frags(tt + 1, fa[1], fb[1]);
      mfmas(fa[0], fb[0]);
      load_frags(tt + 2, fa[0], fb[0]);   // past the group's last tap: discarded
      mfmas(fa[1], fb[1]);
    }
    if (tt < gcur) mfmas(fa[0], fb[0]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // with SPLIT_ALT and the running sum as C, an even chunk count leaves it negated
#if SPLIT_ABL & 2
  {
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) z += acc[i][j][r];
    if (z == 1234.5f) ((float*)a.y)[tid] = z;
    return;
  }
#endif
  const float oscale = (!SPLIT_PARTIAL && SPLIT_ALT && nchunks > 0 && !(nchunks & 1)) ? -SM::scale : SM::scale;
  float* ct = (float*)smem + wave * (32 * 33);
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

template <int MODE, int TH, int TW, int BN, int WM, int WN>
static int try_halo_split(const lic_conv_args& a, hipStream_t s, int& status) {
  constexpr int NT = WM * WN * 64;
  if (a.copad % BN || a.cpad % 16 || a.ci % 4 || a.ldx % 4 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt_split % 16))
    return 0;
  HaloPlan p;
  int dymin = 1 << 20, dymax = -(1 << 20), dxmin = 1 << 20, dxmax = -(1 << 20);
  for (int t = 0; t < a.ntaps; ++t) {
    dymin = dymin < a.dy[t] ? dymin : a.dy[t];
    dymax = dymax > a.dy[t] ? dymax : a.dy[t];
    dxmin = dxmin < a.dx[t] ? dxmin : a.dx[t];
    dxmax = dxmax > a.dx[t] ? dxmax : a.dx[t];
  }
  p.dymin = dymin;
  p.dxmin = dxmin;
  p.hh = (TH - 1) * a.isy + (dymax - dymin) + 1;
  p.hw = (TW - 1) * a.isx + (dxmax - dxmin) + 1;
  const int hpix = p.hh * p.hw;
  if (hpix > 32767) return 0;
  p.hpix_pad = (hpix + 31) / 32 * 32;
  constexpr int NPA = SplitMode<MODE>::NPA, NPB = SplitMode<MODE>::NPB;
  const int fixed = 2 * p.hpix_pad * 64 + NPA * p.hpix_pad * 32;
  const int budget = 160 * 1024 - fixed - TH * TW * 4 - BN * 4;
  int G = budget / (2 * BN * NPB * 32);
  if (G < 1) return 0;
  // 8x8 x 64 (the 16x16 latents: a few hundred workgroups): fewer taps per weight stage so that two
  // workgroups fit a CU's LDS and the whole grid is resident at once
  if (SPLIT_SMALL_2WG && TH * TW == 64 && BN == 64) {
    const int g2 = (80 * 1024 - fixed - TH * TW * 4 - BN * 4) / (2 * BN * NPB * 32);
    if (g2 >= 1 && g2 < G) G = g2;
  }
  if (G > a.ntaps) G = a.ntaps;
  p.G = G;
  p.ngroups = (a.ntaps + G - 1) / G;
  p.tiles_y = (a.mi + TH - 1) / TH;
  p.tiles_x = (a.mj + TW - 1) / TW;
  int nx = 1;
  while (nx < a.ntaps && a.dy[nx] == a.dy[0]) ++nx;
  if (a.ntaps % nx) return 0;
  const int sy = a.ntaps > nx ? a.dy[nx] - a.dy[0] : 0;
  const int sx = nx > 1 ? a.dx[1] - a.dx[0] : 0;
  for (int t = 0; t < a.ntaps; ++t)
    if (a.dy[t] != a.dy[0] + (t / nx) * sy || a.dx[t] != a.dx[0] + (t % nx) * sx) return 0;
  p.toff0 = (a.dy[0] - dymin) * p.hw + (a.dx[0] - dxmin);
  p.nx = nx;
  p.ystep = sy * p.hw;
  p.xstep = sx;
  const int epi_bytes = (NT / 64) * 32 * 33 * 4;
  p.rp_off = fixed + 2 * G * BN * NPB * 32;
  if (p.rp_off < epi_bytes) p.rp_off = epi_bytes;
  const int smem = p.rp_off + TH * TW * 4 + BN * 4;
  p.smem = smem;
  if (smem > 160 * 1024) return 0;
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / BN);
  auto kern = conv_halo_split_kernel<MODE, TH, TW, BN, WM, WN>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, 160 * 1024);
  if (ea != hipSuccess) {
    status = fail(std::string("halo split conv: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return 1;
  }
  hipLaunchKernelGGL(kern, grid, dim3(NT), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("halo split conv launch: ") + hipGetErrorString(e));
  return 1;
}

template <int MODE>
static int split_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  auto blocks = [&](int th, int tw, int bn) {
    return (int64_t)a.n * ((a.mi + th - 1) / th) * ((a.mj + tw - 1) / tw) * (a.copad / bn);
  };
  // each try returns 0 without launching when its LDS plan does not fit (e.g. stride-2 halos)
#if SPLIT_DIAG_ONLY
  if (MODE == 2 && a.copad % 64 == 0 && a.mi > 8 && try_halo_split<2, 16, 16, 64, 4, 2>(a, s, status)) return 1;
  if (MODE == 2 && a.copad % 64 == 0 && try_halo_split<2, 8, 8, 64, 2, 2>(a, s, status)) return 1;
  return 0;
#else
  if (a.mi > 8 && a.mj > 8) {
    // 16x16 x 192 (8 waves of 64 px x 96 ch) fits the fp32x3 fragments in 256 VGPRs; a 4-wave
    // 128 px x 96 ch variant (acc in AGPRs, 1 wave per SIMD) measured 23 % slower
    if (MODE == 1 && a.copad % 192 == 0 && blocks(16, 16, 192) >= 200 &&
        try_halo_split<MODE, 16, 16, 192, 4, 2>(a, s, status))
      return 1;
    if (a.copad % 128 == 0 && blocks(16, 16, 128) >= 200 && try_halo_split<MODE, 16, 16, 128, 4, 2>(a, s, status))
      return 1;
    if (a.copad % 64 == 0 && blocks(16, 16, 64) >= 200 && try_halo_split<MODE, 16, 16, 64, 4, 2>(a, s, status))
      return 1;
  }
  // stride-2 5x5 (ZeroPad + conv5x5 s2 at 128^2 -> 64^2) and other halos too large for a 16x16 tile:
  // 8x8 x 192 stages each halo once for all 192 output channels instead of three times
  if (MODE == 1 && a.copad % 192 == 0 && blocks(8, 8, 192) >= 512 &&
      try_halo_split<MODE, 8, 8, 192, 2, 2>(a, s, status))
    return 1;
  if (a.copad % 64 == 0 && blocks(8, 8, 64) >= 128 && try_halo_split<MODE, 8, 8, 64, 2, 2>(a, s, status)) return 1;
  return 0;
#endif
}

// Returns 1 and launches when a split tile config applies (fp32, mfma_mode 1 / 2, k x k taps incl. 1x1),
// 0 to let the caller run the exact-fp32 kernels.
int conv_halo_split_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if ((a.mfma_mode != 1 && a.mfma_mode != 2) || !a.wgt_split || a.dtype != LIC_F32) return 0;
  // one 16-channel chunk (the image-side 3x3 s2 of a 4-channel input): the exact-fp32 kernels are
  // faster than a split pass whose cost is not amortised over any channel reduction
  if (a.cpad <= 16) return 0;
  if (a.groups != 1 || a.ntaps < 1 || a.force_direct || a.force_mfma_generic) return 0;
  if (a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE && a.prologue != LIC_PRO_ABS) return 0;
  return a.mfma_mode == 1 ? split_dispatch<1>(a, s, status) : split_dispatch<2>(a, s, status);
}

}  // namespace lic
