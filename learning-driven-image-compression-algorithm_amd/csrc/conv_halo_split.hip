// fp32 convolutions on the fp16 matrix cores ("split" MFMA mode, lic_conv_args.mfma_mode = 1).
//
// The spatial-tile conv of conv_halo.h for fp32 activations, with every product formed from
// fp16 parts on v_mfma_f32_32x32x16_f16 instead of the 16x slower fp32-input MFMA:
//   x: x_hi = fp16(x),  x_lo = fp16(x - x_hi)                             (split in LDS)
//   w: W1 = fp16(w) * 2^11 (exact),  W2 = fp16((w - fp16(w)) * 2^11)     (packed on the host)
//   2^11 * x * w ~= x_hi*W1 + x_hi*W2 + x_lo*W1                          (one fp32 accumulator)
// The dropped term (x - x_hi)(w - fp16(w)) is <= 2^-22 |x w| and each part carries 11 bits, so
// a product is within ~3e-7 of its fp32 value (fp32 itself: 6e-8).  x_lo is an fp16 subnormal
// for |x| < 2^-3; its absolute error stays <= 2^-25, ~2^-25 sum|w| on an output.  The fp32
// accumulator (fp32 adds) is scaled back by 2^-11 in the epilogue.
//
// Per 16-channel chunk the fp32 halo of the tile arrives by LDS-DMA in a staging buffer
// (double-buffered, the next chunk's DMA overlaps this chunk's MFMAs); all threads then
// split it once into an x_hi and an x_lo plane laid out as the fp16 kernel's halo (32 B per
// pixel, halves XOR-swizzled), and every tap reads its shifted windows from the planes.
// Weights stream as [G taps][BN][W1 32 B | W2 32 B] stages by LDS-DMA (double buffer).
#include "conv_halo.h"

namespace lic {

constexpr float kSplitScale = 2048.0f;  // 2^11

template <int TH, int TW, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void conv_halo_split_kernel(const lic_conv_args a, const HaloPlan p) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = TH * TW;
  constexpr int CK = 16;  // fp32 channels per chunk (64 B per pixel)
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int sbytes = p.hpix_pad * 64;   // fp32 staging of one chunk
  const int pbytes = p.hpix_pad * 32;   // one fp16 plane
  const int wbytes = p.G * BN * 64;
  char* stg0 = smem;
  char* phi = smem + 2 * sbytes;
  char* plo = phi + pbytes;
  char* wbuf0 = plo + pbytes;
  int* rowpix = (int*)(smem + p.rp_off);
  float* sbias = (float*)(rowpix + BM);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  const half_t* __restrict__ wg = (const half_t*)a.wgt_split;
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
  // weights of stage s: slot (tt, n, s4) holds plane s4>>1 (W1 / W2), swizzled half s4&1
  auto issue_w = [&](int s, int buf, int nw_ld) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    const int total = gcur * BN * 4;
    char* dst = wbuf0 + buf * wbytes;
    for (int q0 = wave * 64; q0 < total; q0 += nw_ld * 64) {
      const int q = q0 + lane;
      const int tt = q / (BN * 4);
      const int n = (q >> 2) - tt * BN;
      const int slot = q & 3;
      const int piece = (slot & 2) | ((slot & 1) ^ ((n >> 3) & 1));
      const half_t* src = wg + ((int64_t)(n0 + n) * a.ntaps + t0 + tt) * (2 * a.cpad) + k * 32 + piece * 8;
      glds16(src, dst + q0 * 16);
    }
  };
  // staging -> x_hi / x_lo planes (32 B per pixel each, halves swizzled as the fp16 kernel)
  auto split_chunk = [&](int buf) {
    const char* src = stg0 + buf * sbytes;
    for (int q = tid; q < hq_total; q += NT) {
      const int hp = q >> 2, c = q & 3;
      const float4 v = *(const float4*)(src + q * 16);
      const float f[4] = {v.x, v.y, v.z, v.w};
      half_t hi[4], lo[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (half_t)f[e];
        lo[e] = (half_t)(f[e] - (float)hi[e]);
      }
      const int off = hp * 32 + (((c >> 1) ^ ((hp >> 3) & 1)) << 4) + (c & 1) * 8;
      *(uint2*)(phi + off) = *(const uint2*)hi;
      *(uint2*)(plo + off) = *(const uint2*)lo;
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
      split_chunk(k & 1);
      __syncthreads();
    }
    constexpr int NL = HALO_LOADERS < NT / 64 ? HALO_LOADERS : NT / 64;
    if (wave < NL) {
      if (s + 1 < nst) issue_w(s + 1, (s + 1) & 1, NL);
      if (g == 0 && k + 1 < nchunks) issue_halo(k + 1, (k + 1) & 1, NL);
    }
    const char* wb = wbuf0 + (s & 1) * wbytes;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    int cy = t0 / p.nx, cx = t0 - cy * p.nx;
    auto load_frags = [&](int tt, u32x4(&fh)[TM], u32x4(&fl)[TM], u32x4(&f1)[TN], u32x4(&f2)[TN]) {
      const int toff = p.toff0 + cy * p.ystep + cx * p.xstep;
      if (++cx == p.nx) {
        cx = 0;
        ++cy;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hp = hbase[i] + toff;
        const int o = hp * 32 + ((lhalf ^ ((hp >> 3) & 1)) << 4);
        fh[i] = *(const u32x4*)(phi + o);
        fl[i] = *(const u32x4*)(plo + o);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WTN + j * 32 + lrow;
        const char* wr = wb + (tt * BN + n) * 64 + ((lhalf ^ ((n >> 3) & 1)) << 4);
        f1[j] = *(const u32x4*)wr;
        f2[j] = *(const u32x4*)(wr + 32);
      }
    };
    auto mfmas = [&](const u32x4(&fh)[TM], const u32x4(&fl)[TM], const u32x4(&f1)[TN], const u32x4(&f2)[TN]) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = mfma_k16<half_t>(fh[i], f1[j], acc[i][j]);
          acc[i][j] = mfma_k16<half_t>(fh[i], f2[j], acc[i][j]);
          acc[i][j] = mfma_k16<half_t>(fl[i], f1[j], acc[i][j]);
        }
    };
    u32x4 fh[2][TM], fl[2][TM], f1[2][TN], f2[2][TN];
    load_frags(0, fh[0], fl[0], f1[0], f2[0]);
    int tt = 0;
    for (; tt + 2 <= gcur; tt += 2) {
      load_frags(tt + 1, fh[1], fl[1], f1[1], f2[1]);
      mfmas(fh[0], fl[0], f1[0], f2[0]);
      load_frags(tt + 2, fh[0], fl[0], f1[0], f2[0]);   // past the group's last tap: discarded
      mfmas(fh[1], fl[1], f1[1], f2[1]);
    }
    if (tt < gcur) mfmas(fh[0], fl[0], f1[0], f2[0]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  float* ct = (float*)smem + wave * (32 * 33);
  epilogue_all<float, TM * TN, TN>(a, ct, rowpix + wm * WTM, n0 + wn * WTN, sbias + wn * WTN, lane, [&](int q) {
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
      if (qq == q) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ct[((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r] * (1.0f / kSplitScale);
      }
  });
}

template <int TH, int TW, int BN, int WM, int WN>
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
  const int fixed = 2 * p.hpix_pad * 64 + 2 * p.hpix_pad * 32;
  const int budget = 160 * 1024 - fixed - TH * TW * 4 - BN * 4;
  int G = budget / (2 * BN * 64);
  if (G < 1) return 0;
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
  p.rp_off = fixed + 2 * G * BN * 64;
  if (p.rp_off < epi_bytes) p.rp_off = epi_bytes;
  const int smem = p.rp_off + TH * TW * 4 + BN * 4;
  p.smem = smem;
  if (smem > 160 * 1024) return 0;
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / BN);
  auto kern = conv_halo_split_kernel<TH, TW, BN, WM, WN>;
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

// Returns 1 and launches when a split tile config applies (fp32, mfma_mode 1, k x k taps),
// 0 to let the caller run the exact-fp32 kernels.
int conv_halo_split_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.mfma_mode != 1 || !a.wgt_split || a.dtype != LIC_F32) return 0;
  if (a.groups != 1 || a.ntaps < 2 || a.prologue != LIC_PRO_NONE || a.force_direct || a.force_mfma_generic) return 0;
  auto blocks = [&](int th, int tw, int bn) {
    return (int64_t)a.n * ((a.mi + th - 1) / th) * ((a.mj + tw - 1) / tw) * (a.copad / bn);
  };
  if (a.mi > 8 && a.mj > 8) {
    if (a.copad % 192 == 0 && blocks(16, 16, 192) >= 200) return try_halo_split<16, 16, 192, 4, 2>(a, s, status);
    if (a.copad % 128 == 0 && blocks(16, 16, 128) >= 200) return try_halo_split<16, 16, 128, 4, 2>(a, s, status);
    if (a.copad % 64 == 0 && blocks(16, 16, 64) >= 200) return try_halo_split<16, 16, 64, 4, 2>(a, s, status);
  }
  if (a.copad % 64 == 0 && blocks(8, 8, 64) >= 128) return try_halo_split<8, 8, 64, 2, 2>(a, s, status);
  return 0;
}

}  // namespace lic
