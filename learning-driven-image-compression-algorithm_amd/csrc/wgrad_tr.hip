// Tiled weight gradient for 16-bit training (fp16 / bf16): all taps of a tap group per
// work-group, operands staged untransposed and read with the LDS transpose read.
//
//   dW[co][tap][ci] = sum over lattice pixels (b, i, j) of dz[b, oy0+osy*i, ox0+osx*j][co]
//                                                      * pro(x[b, S*i + dy_t, S*j + dx_t][ci])
// (conv2d wgrad, autograd.py _Conv2dFn.backward; the transposed-conv wgrad with the roles of
// x and dz exchanged, _ConvT2dFn.backward; GDN dGamma' with PRO_SQUARE).
//
// A work-group owns 64 output channels x 64 input channels x one tap group (all 9 taps of a
// 3x3 window, one 5- or 7-tap row of a 5x5 / 7x7 window, or a single 1x1 tap) and walks a contiguous run
// of spatial tiles (8 x 8 lattice pixels, 16 x 8 for 1x1) — the split-K dimension.  Per tile it
// stages, with plain coalesced 16-byte loads (raw buffer loads: out-of-image rows and the ragged
// lattice edge read as zeros):
//   dz tile  [2 planes of 32 channels][TI*8 pixels][64 B]          (pixels x co, untransposed)
//   x  halo  [2 planes of 32 channels][HR*HC halo pixels][64 B]    (covers every tap of the group)
// and each wave (32 co x 32 ci of the 64 x 64 block) builds its MFMA operands with
// ds_read_b64_tr_b16: K is the pixel axis, which is the ROW axis of both images, so the
// transpose read delivers 4 consecutive pixels of one channel per lane; a tap is a constant
// row offset into the halo image, so the dz fragment is read once per K step and reused by all
// G taps (G MFMAs per 2 + 2G transpose reads).  64-byte plane rows make each 32-lane half's
// 4 rows x 64 B one conflict-free 256-byte span.  Partials go to ws[split][tap][co][ci] and
// the deterministic wgrad_reduce_kernel (train.hip) sums the splits.  With a bias gradient requested,
// the waves of the first ci block / tap group also sum their dz fragments (8 values per lane and K
// step, VALU) into per-split column sums that the same reduce finishes: db costs no extra pass over dz.
#include "lic_common.h"

namespace lic {

typedef short v4s16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s16 lds_v4s16;

struct WtrPlan {
  int tiles_i, tiles_j, ntile, per, nsplit, tiles_n, ngroups, nv;
  int zbytes, xbytes;
  int8_t gy[LIC_MAX_TAPS], gx[LIC_MAX_TAPS];  // halo origin (dymin, dxmin) of each tap group
  int8_t ty[LIC_MAX_TAPS], tx[LIC_MAX_TAPS];  // tap offset inside its group's halo
};

// NV > 1 (1x1 only): the work-group takes NV 64-channel blocks of ci and each wave treats them as
// NV "virtual taps" (x plane pairs), so the dz fragment is again reused by NV MFMAs
template <int S, int G, int NV = 1> struct WtrCfg {
  static constexpr int SPY = G == 9 ? 2 : 0;               // tap-window spans the halo covers
  static constexpr int SPX = G == 9 ? 2 : (G == 1 ? 0 : G - 1);
  static constexpr int TI = (G == 1 && NV == 1) ? 16 : 8, TJ = 8;   // lattice tile (K per stage = TI*TJ)
  static constexpr int HR = (TI - 1) * S + SPY + 1, HC = (TJ - 1) * S + SPX + 1;
  static constexpr int HPIX = HR * HC, ZPIX = TI * TJ;
  static constexpr int NA = G * NV;                         // accumulator tiles per wave
  static constexpr int ZB = 2 * ZPIX * 64, XB = 2 * NV * HPIX * 64, BUF = ZB + XB;
  static constexpr int LDS = 2 * BUF;
};

__device__ __forceinline__ u32x4 tr_frag(const char* p, int d) {
  const v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)p);
  const v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(p + d));
  u32x4 r;
  __builtin_memcpy((char*)&r, &lo, 8);
  __builtin_memcpy((char*)&r + 8, &hi, 8);
  return r;
}

template <typename T, int S, int G, int PRO, int NV = 1>
__global__ __launch_bounds__(256, 2) void wgrad_tr_kernel(const lic_wgrad_args a, const WtrPlan p,
                                                          float* __restrict__ ws, float* __restrict__ wsb) {
  static_assert(NV == 1 || G == 1, "virtual ci taps are for 1x1 windows");
  using C = WtrCfg<S, G, NV>;
  constexpr int TI = C::TI, TJ = C::TJ, HC = C::HC, HPIX = C::HPIX, ZPIX = C::ZPIX, NA = C::NA;
  constexpr int XCH = 8 * NV;   // 16-byte chunks per halo pixel
  constexpr int ZU = ZPIX * 8 / 256, XU = (HPIX * XCH + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
  const int wm = wave >> 1, wn = wave & 1;
  int bx = blockIdx.x;
  const int grp = bx % p.ngroups;
  bx /= p.ngroups;
  const int tn = bx % p.tiles_n, tm = bx / p.tiles_n;
  const int n0 = tm * 64, c0 = tn * 64 * NV;
  const int kbeg = blockIdx.y * p.per, kend = min(p.ntile, kbeg + p.per);
  const int gdy = p.gy[grp], gdx = p.gx[grp];
  const int tpi = p.tiles_i * p.tiles_j;

  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.dz, (short)0, p.zbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, p.xbytes, 0x00020000);
  constexpr int OOB = (int)0x80000000;

  u32x4 zr[ZU], xr[XU];
  auto gload = [&](int k) {
    const int b = k / tpi, rem = k - b * tpi;
    const int ti0 = (rem / p.tiles_j) * TI, tj0 = (rem % p.tiles_j) * TJ;
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      const int c = tid + 256 * u, px = c >> 3, ch = n0 + (c & 7) * 8;
      const int i = ti0 + px / TJ, j = tj0 + px % TJ;
      const bool ok = i < a.mi && j < a.mj && ch < a.co;
      const int off = ok ? (((b * a.ho + a.oy0 + a.osy * i) * a.wo + a.ox0 + a.osx * j) * a.ldz + ch) * 2 : OOB;
      zr[u] = __builtin_amdgcn_raw_buffer_load_b128(zrs, off, 0, 0);
    }
    const int y0 = ti0 * S + gdy, x0 = tj0 * S + gdx;
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int c = tid + 256 * u, hp = c / XCH, ch = c0 + (c - hp * XCH) * 8;
      const int hr = hp / HC, hc = hp - hr * HC;
      const int y = y0 + hr, x = x0 + hc;
      const bool ok = c < HPIX * XCH && (unsigned)y < (unsigned)a.h && (unsigned)x < (unsigned)a.w && ch < a.ci;
      const int off = ok ? (((b * a.h + y) * a.w + x) * a.ldx + ch) * 2 : OOB;
      xr[u] = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
    char* zb = smem + buf * C::BUF;
    char* xb = zb + C::ZB;
#pragma unroll
    for (int u = 0; u < ZU; ++u) {
      const int c = tid + 256 * u, px = c >> 3, cc = c & 7;
      *(u32x4*)(zb + (cc >> 2) * (ZPIX * 64) + px * 64 + (cc & 3) * 16) = zr[u];
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int c = tid + 256 * u, hp = c / XCH, cc = c - hp * XCH;
      if (XU * 256 > HPIX * XCH && c >= HPIX * XCH) continue;
      u32x4 v = xr[u];
      if constexpr (PRO == LIC_PRO_SQUARE) {
        T* e = (T*)&v;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float f = to_f(e[q]);
          e[q] = from_f<T>(f * f);
        }
      }
      *(u32x4*)(xb + (cc >> 2) * (HPIX * 64) + hp * 64 + (cc & 3) * 16) = v;
    }
  };

  floatx16 acc[NA];
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // lane (hi, g1, q, p): transpose-read address of row q (pixel), columns 16*g1 + 4p .. +3
  const int hi = lane >> 5, g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  const int col_b = (16 * g1 + 4 * pp) * 2;
  const int a_lane = wm * (ZPIX * 64) + (8 * hi + q) * 64 + col_b;
  const int b_lane = C::ZB + wn * (HPIX * 64) + (hi * S * HC + q * S) * 64 + col_b;
  int toff[NA];   // a tap's (or virtual tap's x plane pair's) byte offset into the halo image
#pragma unroll
  for (int t = 0; t < NA; ++t) toff[t] = NV > 1 ? t * 2 * HPIX * 64 : (p.ty[grp * G + t] * HC + p.tx[grp * G + t]) * 64;

  // bias partial: lane l sums dz[k][co = n0 + 32 wm + (l & 31)] over its K half (wave-uniform branch)
  const bool do_bias = wsb != nullptr && tn == 0 && grp == 0 && wn == 0;
  float bsum = 0.f;
  auto compute = [&](int buf) {
    const char* za = smem + buf * C::BUF + a_lane;
    const char* xbb = smem + buf * C::BUF + b_lane;
#pragma unroll
    for (int s = 0; s < TI / 2; ++s) {
      const u32x4 fa = tr_frag(za + 16 * s * 64, 4 * 64);
      if (do_bias) {
        const T* e = (const T*)&fa;
#pragma unroll
        for (int q = 0; q < 8; ++q) bsum += to_f(e[q]);
      }
#pragma unroll
      for (int t = 0; t < NA; ++t) {
        const u32x4 fb = tr_frag(xbb + toff[t] + 2 * s * S * HC * 64, 4 * S * 64);
        acc[t] = mfma_k16<T>(fa, fb, acc[t]);
      }
    }
  };

  const int n = kend - kbeg;
  if (n > 0) {
    gload(kbeg);
    sstore(0);
    __syncthreads();
    for (int it = 0; it < n; ++it) {
      const int cur = it & 1;
      if (it + 1 < n) gload(kbeg + it + 1);
      compute(cur);
      if (it + 1 < n) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  if (do_bias) {
    bsum += __shfl_xor(bsum, 32);
    const int co = n0 + wm * 32 + lane;
    if (lane < 32 && co < a.co) wsb[(int64_t)blockIdx.y * a.co + co] = bsum;
  }
  // partial tile -> ws[split][tap][co][ci] (lanes 0..31 write 32 consecutive ci)
#pragma unroll
  for (int t = 0; t < NA; ++t) {
    const int col = c0 + (NV > 1 ? t * 64 : 0) + wn * 32 + (lane & 31);
    float* out = ws + ((int64_t)blockIdx.y * a.ntaps + (NV > 1 ? 0 : grp * G + t)) * a.co * a.ci;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = n0 + wm * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
      if (row < a.co && col < a.ci) out[(int64_t)row * a.ci + col] = acc[t][r];
    }
  }
}

static bool wtr_enabled() {
  static const bool on = [] {
    const char* e = getenv("LIC_WGRAD_TR");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Plans the tiled kernel; returns its tap-group size G (1, 5, 7 or 9) or 0 when it does not apply
// (fp32, strides other than 1 / 2, tap sets that are not 1x1, 3x3 or rows of 5 / 7, > 2 GB views).
static int wtr_plan(const lic_wgrad_args& a, WtrPlan& p) {
  if (!wtr_enabled() || a.dtype == LIC_F32) return 0;
  if (a.isy != a.isx || (a.isy != 1 && a.isy != 2)) return 0;
  const int G = a.ntaps == 1 ? 1 : (a.ntaps == 9 ? 9 : (a.ntaps % 5 == 0 ? 5 : (a.ntaps % 7 == 0 ? 7 : 0)));
  if (!G) return 0;
  const int spy = G == 9 ? 2 : 0, spx = G == 9 ? 2 : (G == 1 ? 0 : G - 1);
  p.ngroups = a.ntaps / G;
  for (int g = 0; g < p.ngroups; ++g) {
    int ymin = 127, xmin = 127, ymax = -128, xmax = -128;
    for (int t = g * G; t < (g + 1) * G; ++t) {
      ymin = std::min(ymin, (int)a.dy[t]);
      ymax = std::max(ymax, (int)a.dy[t]);
      xmin = std::min(xmin, (int)a.dx[t]);
      xmax = std::max(xmax, (int)a.dx[t]);
    }
    if (ymax - ymin > spy || xmax - xmin > spx) return 0;
    p.gy[g] = (int8_t)ymin;
    p.gx[g] = (int8_t)xmin;
    for (int t = g * G; t < (g + 1) * G; ++t) {
      p.ty[t] = (int8_t)(a.dy[t] - ymin);
      p.tx[t] = (int8_t)(a.dx[t] - xmin);
    }
  }
  const int64_t zb = (int64_t)a.n * a.ho * a.wo * a.ldz * 2, xb = (int64_t)a.n * a.h * a.w * a.ldx * 2;
  if (zb >= ((int64_t)1 << 31) || xb >= ((int64_t)1 << 31)) return 0;
  p.zbytes = (int)zb;
  p.xbytes = (int)xb;
  // 1x1 at stride 1: NV ci blocks per work-group (NV divides the block count where it can)
  const int nb = (a.ci + 63) / 64;
  p.nv = 1;
  if (G == 1 && a.isy == 1 && nb > 1) p.nv = nb <= 4 ? nb : (nb % 4 == 0 ? 4 : (nb % 3 == 0 ? 3 : (nb % 2 == 0 ? 2 : 4)));
  const int TI = (G == 1 && p.nv == 1) ? 16 : 8;
  p.tiles_i = (a.mi + TI - 1) / TI;
  p.tiles_j = (a.mj + 7) / 8;
  p.ntile = a.n * p.tiles_i * p.tiles_j;
  p.tiles_n = (nb + p.nv - 1) / p.nv;
  const int blocks = ((a.co + 63) / 64) * p.tiles_n * p.ngroups;
  // ~512 work-groups (two per CU), at least 8 tiles each (the partials stay well below the operands)
  int ns = (512 + blocks - 1) / blocks;
  ns = std::max(1, std::min(ns, p.ntile / 8));
  p.per = (p.ntile + ns - 1) / ns;
  p.nsplit = (p.ntile + p.per - 1) / p.per;
  return G;
}

int wgrad_tr_nsplit(const lic_wgrad_args& a) {
  WtrPlan p;
  return wtr_plan(a, p) ? p.nsplit : 0;
}

template <typename T, int S, int G, int NV = 1>
static int wtr_launch(const lic_wgrad_args& a, const WtrPlan& p, hipStream_t s) {
  using C = WtrCfg<S, G, NV>;
  auto kern = a.prologue == LIC_PRO_SQUARE ? wgrad_tr_kernel<T, S, G, LIC_PRO_SQUARE, NV>
                                           : wgrad_tr_kernel<T, S, G, LIC_PRO_NONE, NV>;
  if (C::LDS > 64 * 1024) {
    const hipError_t e = ensure_dyn_lds((const void*)kern, C::LDS);
    if (e != hipSuccess) return fail(std::string("wgrad: dynamic LDS: ") + hipGetErrorString(e));
  }
  const dim3 grid(((a.co + 63) / 64) * p.tiles_n * p.ngroups, p.nsplit);
  float* wsb = a.db ? a.ws + (int64_t)p.nsplit * a.ntaps * a.co * a.ci : nullptr;
  hipLaunchKernelGGL(kern, grid, dim3(256), C::LDS, s, a, p, a.ws, wsb);
  LIC_CHECK_LAUNCH();
  return 0;
}

template <typename T>
static int wtr_launch_t(const lic_wgrad_args& a, const WtrPlan& p, int G, hipStream_t s) {
  if (a.isy == 1) {
    if (G == 9) return wtr_launch<T, 1, 9>(a, p, s);
    if (G == 5) return wtr_launch<T, 1, 5>(a, p, s);
    if (G == 7) return wtr_launch<T, 1, 7>(a, p, s);
    if (p.nv == 4) return wtr_launch<T, 1, 1, 4>(a, p, s);
    if (p.nv == 3) return wtr_launch<T, 1, 1, 3>(a, p, s);
    if (p.nv == 2) return wtr_launch<T, 1, 1, 2>(a, p, s);
    return wtr_launch<T, 1, 1>(a, p, s);
  }
  if (G == 9) return wtr_launch<T, 2, 9>(a, p, s);
  if (G == 5) return wtr_launch<T, 2, 5>(a, p, s);
  if (G == 7) return wtr_launch<T, 2, 7>(a, p, s);
  return wtr_launch<T, 2, 1>(a, p, s);
}

// Launches the partial-sum kernel into a.ws ([nsplit][tap][co][ci]); returns -1 when the tiled
// kernel does not apply (the caller then uses wgrad_kernel), else 0 / the failure code.
int wgrad_tr_launch(const lic_wgrad_args& a, hipStream_t s, int* nsplit) {
  WtrPlan p;
  const int G = wtr_plan(a, p);
  if (!G) return -1;
  *nsplit = p.nsplit;
  return a.dtype == LIC_F16 ? wtr_launch_t<half_t>(a, p, G, s) : wtr_launch_t<bf16_t>(a, p, G, s);
}

}  // namespace lic
