// Convolution entry point: kernel choice (halo / generic implicit-GEMM MFMA /
// direct VALU) and the direct kernel.  The MFMA kernels live in conv_mfma.h
// (instantiated by conv_mfma_*.hip) and conv_halo.h (conv_halo_*.hip).
#include "lic_common.h"

#ifndef HALO_BIG_TILE
#define HALO_BIG_TILE 1
#endif
// 1x1 convolutions (GEMMs) on the halo kernel: 1 = fp32, 2 = fp32 and 16-bit, 0 = never
#ifndef HALO_1X1
#define HALO_1X1 1
#endif

namespace lic {

// Generic implicit-GEMM launches, instantiated in conv_mfma_*.hip (one TU per
// dtype and row-tile so the kernels compile in parallel).
template <typename T, int BM, int BN, int WM, int WN>
int launch_mfma(const lic_conv_args& a, int M, hipStream_t s);

// Spatial-tile ("halo") launches, instantiated in conv_halo_*.hip.  Return 1 and
// launch when the tile config applies, 0 to fall back.
template <typename T, int TH, int TW, int BN, int WM, int WN>
int try_halo(const lic_conv_args& a, hipStream_t s, int& status);

// fp32 activations on the fp16 matrix cores (mfma_mode 1), conv_halo_split.hip.
int conv_halo_split_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
int conv_split_wd_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
int conv_split_1x1_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
// 16-bit stride-1 3x3 / 7x7 on big maps (conv16.h, instantiated in conv16_{f16,bf16}.hip)
template <typename T> int conv16_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
// 16-bit 1x1 convolutions on big maps (gemm16.h, gemm16_{f16,bf16}.hip)
template <typename T> int gemm16_dispatch(const lic_conv_args& a, hipStream_t s, int& status);

// Halo tile choice: the largest output-channel block whose grid still fills the
// chip (>= 200 workgroups of 16x16 pixels), then 8x8-pixel tiles for small maps
// (the 16x16 latents of the slice loop).
template <typename T>
static int conv_halo_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if constexpr (sizeof(T) == 2) {   // round-5 16-bit kernels first
    if (a.ntaps == 1 || a.ci <= 16) {
      if (int r = gemm16_dispatch<T>(a, s, status)) return r;
    }
    if (int r = conv16_dispatch<T>(a, s, status)) return r;   // (1x1: small maps only)
  }
  const bool gemm_ok = a.ntaps == 1 && (HALO_1X1 == 2 || (HALO_1X1 == 1 && sizeof(T) == 4));
  if (a.groups != 1 || (a.ntaps < 2 && !gemm_ok) || a.prologue != LIC_PRO_NONE || a.force_direct) return 0;
  auto blocks = [&](int th, int tw, int bn) {
    return (int64_t)a.n * ((a.mi + th - 1) / th) * ((a.mj + tw - 1) / tw) * (a.copad / bn);
  };
  // 16x16 tiles only where at most half of a tile row / column can fall off the map
  const bool big_map = a.mi > 8 && a.mj > 8;
  if (big_map) {
    // fp16, stride 1: 32x16-pixel tiles halve the weight bytes streamed per FLOP (the
    // LDS-DMA stream, not the MFMA, bounds the 16x16 tile) where the grid still fills
    if constexpr (sizeof(T) == 2) {
      if (HALO_BIG_TILE && a.copad % 192 == 0 && a.isy == 1 && a.isx == 1 && a.mi > 16 && blocks(32, 16, 192) >= 200)
        return try_halo<T, 32, 16, 192, 4, 2>(a, s, status);
      // 64-channel maps (HAN at full resolution): same tile, one 64-wide channel block
      if (HALO_BIG_TILE && a.copad == 64 && a.isy == 1 && a.isx == 1 && a.mi > 16 && blocks(32, 16, 64) >= 1024)
        return try_halo<T, 32, 16, 64, 8, 1>(a, s, status);
    }
    if (a.copad % 192 == 0 && blocks(16, 16, 192) >= 200) return try_halo<T, 16, 16, 192, 4, 2>(a, s, status);
    if (a.copad % 128 == 0 && blocks(16, 16, 128) >= 200) return try_halo<T, 16, 16, 128, 4, 2>(a, s, status);
    if (a.copad % 64 == 0 && blocks(16, 16, 64) >= 200) return try_halo<T, 16, 16, 64, 4, 2>(a, s, status);
    if (a.copad % 32 == 0 && blocks(16, 16, 32) >= 200) return try_halo<T, 16, 16, 32, 8, 1>(a, s, status);
  }
  if (a.copad % 64 == 0 && blocks(8, 8, 64) >= 128) return try_halo<T, 8, 8, 64, 2, 2>(a, s, status);
  if (a.copad % 32 == 0 && blocks(8, 8, 32) >= 64) return try_halo<T, 8, 8, 32, 2, 1>(a, s, status);
  return 0;
}

// Direct (VALU) convolution for tiny / misaligned channel counts (Cin = 1 or 3,
// grouped / depthwise, 1x1 layers on a handful of pixels).  One thread computes
// COG consecutive output channels of one pixel; the packed weights are staged in
// LDS as fp32 when they fit, and every input value is loaded once per thread.
template <typename T, int COG>
__global__ __launch_bounds__(256) void conv_direct_kernel(const lic_conv_args a, const int64_t M, const int ngroups,
                                                          const int wlds) {
  extern __shared__ float wsm[];
  const T* xg = (const T*)a.x;
  const T* wg = (const T*)a.wgt;
  const int wtot = a.copad * a.ntaps * a.cpad;
  if (wlds) {
    for (int k = threadIdx.x; k < wtot; k += 256) wsm[k] = to_f(wg[k]);
    __syncthreads();
  }
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * ngroups) return;
  const int g = (int)(idx % ngroups);
  const int m = (int)(idx / ngroups);
  const int mij = a.mi * a.mj;
  const int b = m / mij;
  const int rem = m - b * mij;
  const int i = rem / a.mj;
  const int j = rem - i * a.mj;
  const int cig = a.ci / a.groups;
  const int cog = a.co / a.groups;
  const int n0 = g * COG;
  const int wstride = a.ntaps * a.cpad;
  float acc[COG];
#pragma unroll
  for (int k = 0; k < COG; ++k) acc[k] = 0.f;
  for (int t = 0; t < a.ntaps; ++t) {
    const int iy = i * a.isy + a.dy[t], ix = j * a.isx + a.dx[t];
    if ((unsigned)iy >= (unsigned)a.h || (unsigned)ix >= (unsigned)a.w) continue;
    const T* px = xg + ((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx;
    if (a.groups == 1) {
      for (int c = 0; c < cig; ++c) {
        const float xv = apply_pro(to_f(px[c]), a.prologue);
        const int wo = t * a.cpad + c;
#pragma unroll
        for (int k = 0; k < COG; ++k) {
          const int n = min(n0 + k, a.copad - 1);
          const float wv = wlds ? wsm[n * wstride + wo] : to_f(wg[(int64_t)n * wstride + wo]);
          acc[k] += xv * wv;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < COG; ++k) {
        const int n = min(n0 + k, a.co - 1);
        const int cb = (n / cog) * cig;
        for (int c = 0; c < cig; ++c) {
          const float xv = apply_pro(to_f(px[cb + c]), a.prologue);
          const int wo = t * a.cpad + c;
          const float wv = wlds ? wsm[n * wstride + wo] : to_f(wg[(int64_t)n * wstride + wo]);
          acc[k] += xv * wv;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < COG; ++k) {
    const int n = n0 + k;
    if (n >= a.co) break;
    int64_t pix;
    int ch;
    out_coord(a, b, i, j, n, pix, ch);
    const float v = conv_epilogue<T>(a, acc[k], n, pix, ch);
    ((T*)a.y)[pix * a.ldy + ch] = from_f<T>(v);
    if (a.y2) ((T*)a.y2)[pix * a.ldy2 + ch] = from_f<T>(v);
  }
}

template <typename T>
static int conv_dispatch(const lic_conv_args& a, hipStream_t s) {
  const int64_t M64 = (int64_t)a.n * a.mi * a.mj;
  if (M64 <= 0 || a.co <= 0) return 0;
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = 4 * EPC;
  const int64_t out_pix = (int64_t)a.n * a.ho * a.wo;
  if (M64 >= (1LL << 31) || out_pix >= (1LL << 31)) return fail("conv: too many pixels for int32 indexing");
  const int M = (int)M64;
  // the halo kernel takes any multiple of its 32-byte chunk (2 * EPC channels: one 8-channel fp32 chunk
  // for the padded image); the split and generic MFMA kernels want 4 * EPC
  const bool tile_ok = !a.force_direct && a.groups == 1 && a.prologue != LIC_PRO_ABS && a.ci % EPC == 0 &&
                       a.cpad % (2 * EPC) == 0 && a.ldx % EPC == 0 && ((uintptr_t)a.x % 16 == 0) &&
                       ((uintptr_t)a.wgt % 16 == 0) && a.copad % 32 == 0 && a.ci >= EPC;
  bool mfma_ok = tile_ok && a.cpad % BK == 0;
  if (tile_ok && !mfma_ok && !a.force_mfma_generic) {
    int st = 0;
    if (conv_halo_dispatch<T>(a, s, st)) return st;
  }
  if (mfma_ok && !a.force_mfma_generic) {
    int st = 0;
    if constexpr (sizeof(T) == 4) {
      if (conv_split_wd_dispatch(a, s, st)) return st;
      if (conv_split_1x1_dispatch(a, s, st)) return st;
      if (conv_halo_split_dispatch(a, s, st)) return st;
    }
    if (conv_halo_dispatch<T>(a, s, st)) return st;
  }
  if (mfma_ok) {
    int BN = 0;
    const int cands[5] = {192, 128, 96, 64, 32};
    for (int k = 0; k < 5; ++k)
      if (a.copad % cands[k] == 0) { BN = cands[k]; break; }
    const int nN = a.copad / BN;
    const bool big = ((int64_t)((M + 127) / 128) * nN) >= 384;
    if (big) {
      switch (BN) {
        case 192: return launch_mfma<T, 128, 192, 2, 2>(a, M, s);
        case 128: return launch_mfma<T, 128, 128, 2, 2>(a, M, s);
        case 96: return launch_mfma<T, 128, 96, 4, 1>(a, M, s);
        case 64: return launch_mfma<T, 128, 64, 4, 1>(a, M, s);
        default: return launch_mfma<T, 128, 32, 4, 1>(a, M, s);
      }
    } else {
      switch (BN) {
        case 192: return launch_mfma<T, 64, 192, 2, 2>(a, M, s);
        case 128: return launch_mfma<T, 64, 128, 2, 2>(a, M, s);
        case 96: return launch_mfma<T, 64, 96, 2, 1>(a, M, s);
        case 64: return launch_mfma<T, 64, 64, 2, 1>(a, M, s);
        default: return launch_mfma<T, 64, 32, 2, 1>(a, M, s);
      }
    }
  }
  const int cog = a.co >= 16 && a.groups == 1 ? 16 : (a.co >= 4 && a.groups == 1 ? 4 : 1);
  const int ngroups = (a.co + cog - 1) / cog;
  const int64_t total = M64 * ngroups;
  const int64_t blocks = (total + 255) / 256;
  const size_t wbytes = (size_t)a.copad * a.ntaps * a.cpad * sizeof(float);
  const int wlds = wbytes <= 48 * 1024 ? 1 : 0;
  const size_t shm = wlds ? wbytes : 0;
  if (cog == 16)
    hipLaunchKernelGGL((conv_direct_kernel<T, 16>), dim3((unsigned)blocks), dim3(256), shm, s, a, M64, ngroups, wlds);
  else if (cog == 4)
    hipLaunchKernelGGL((conv_direct_kernel<T, 4>), dim3((unsigned)blocks), dim3(256), shm, s, a, M64, ngroups, wlds);
  else
    hipLaunchKernelGGL((conv_direct_kernel<T, 1>), dim3((unsigned)blocks), dim3(256), shm, s, a, M64, ngroups, wlds);
  LIC_CHECK_LAUNCH();
  return 0;
}

}  // namespace lic

extern "C" int lic_conv2d_fwd(const lic_conv_args* a, lic_stream_t stream) {
  using namespace lic;
  if (!a) return fail("conv: null args");
  if (a->ntaps < 1 || a->ntaps > LIC_MAX_TAPS) return fail("conv: ntaps out of range");
  if (a->groups < 1 || a->ci % a->groups || a->co % a->groups) return fail("conv: bad groups");
  if (a->copad < a->co || a->cpad < a->ci / a->groups) return fail("conv: bad padding of packed weights");
  if (a->out_shuffle != 0 && a->out_shuffle != 2 && a->out_shuffle != 3) return fail("conv: out_shuffle must be 0, 2 or 3");
  if (a->out_shuffle != 0 && (a->r1 || a->g || a->r2 || a->co % 4)) return fail("conv: shuffle with residual");
  if (a->epi < 0 || a->epi > LIC_EPI_RES_ACT) return fail("conv: bad epilogue");
  if ((a->epi == LIC_EPI_GATE || (a->epi >= LIC_EPI_GDN_DIV && a->epi <= LIC_EPI_GDN_SQRT)) && !a->g) return fail("conv: epilogue needs g");
  if ((a->epi == LIC_EPI_GATE || a->epi == LIC_EPI_HALF_TANH) && !a->r2) return fail("conv: epilogue needs r2");
  if (!a->x || !a->y || !a->wgt) return fail("conv: null tensor");
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == LIC_F32) return conv_dispatch<float>(*a, s);
  if (a->dtype == LIC_F16) return conv_dispatch<half_t>(*a, s);
  if (a->dtype == LIC_BF16) return conv_dispatch<bf16_t>(*a, s);
  return fail("conv: bad dtype");
}
