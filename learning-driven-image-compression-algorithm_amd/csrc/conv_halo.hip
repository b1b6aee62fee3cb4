// Spatial-tile ("halo") implicit-GEMM convolution for k x k kernels (gfx950).
//
// A workgroup owns a TH x TW tile of output-lattice pixels of one image and BN
// output channels.  The reduction runs over 32-byte channel chunks (16 f16 /
// 8 f32 channels).  Per chunk the input halo of the tile
//     [(TH-1)*isy + dy_max-dy_min+1] x [(TW-1)*isx + dx_max-dx_min+1] pixels x 32 B
// is staged ONCE in LDS and every tap reads its shifted window from it (a 3x3
// conv re-reads each input byte from HBM/L2 ~1.3x instead of 9x).  The packed
// weights of a group of G taps ([G][BN][32 B]) are staged per stage.  Both are
// moved by LDS-DMA (global_load_lds_dwordx4: no VGPR staging) into double
// buffers: stage s+1's weights and chunk k+1's halo are in flight while stage s
// computes; out-of-image halo pixels read a zero page.  16-B halves of every
// 32-B row are XOR-swizzled by bit 3 of the row index so the ds_read_b128
// fragment reads of 16 consecutive pixels / channels are conflict-free.
// Fragments: f16 v_mfma_f32_32x32x16_f16 (one per tap and 32x32 tile); f32
// v_mfma_f32_32x32x2_f32 x4 (exact fp32).  Epilogue as conv.hip (LDS-staged).
#include "lic_common.h"

namespace lic {

__device__ __attribute__((aligned(256))) unsigned char g_lic_zero_page[256];

struct HaloPlan {
  int hh, hw;      // halo rows / cols
  int hpix_pad;    // halo pixels rounded up to a multiple of 32
  int G;           // taps per stage group
  int ngroups;
  int tiles_y, tiles_x;
  int smem;        // dynamic LDS bytes
  int16_t toff[LIC_MAX_TAPS];  // (dy - dymin) * hw + (dx - dxmin)
  int dymin, dxmin;
};

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <typename T, int TH, int TW, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void conv_halo_kernel(const lic_conv_args a, const HaloPlan p) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = TH * TW;
  constexpr int E = 16 / (int)sizeof(T);  // elements per 16 B
  constexpr int CK = 2 * E;               // elements per 32-B chunk
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int hbytes = p.hpix_pad * 32;
  const int wbytes = p.G * BN * 32;
  char* hbuf0 = smem;
  char* wbuf0 = smem + 2 * hbytes;
  int* rowpix = (int*)(wbuf0 + 2 * wbytes);
  int16_t* stoff = (int16_t*)(rowpix + BM);

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

  for (int t = tid; t < a.ntaps; t += NT) stoff[t] = p.toff[t];
  for (int m = tid; m < BM; m += NT) {
    const int i = i0 + m / TW, j = j0 + m % TW;
    int base = -1;
    if (i < a.mi && j < a.mj) {
      int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
      if (a.out_shuffle == 2) { oy *= 2; ox *= 2; }
      base = (b * a.ho + oy) * a.wo + ox;
    }
    rowpix[m] = base;
  }

  const T* __restrict__ xg = (const T*)a.x;
  const T* __restrict__ wg = (const T*)a.wgt;
  const int nchunks = a.cpad / CK;
  const int nst = nchunks * p.ngroups;
  const int hq_total = p.hpix_pad * 2;
  const int hpix = p.hh * p.hw;

  auto issue_halo = [&](int k, int buf) {
    const int c0 = k * CK;
    char* dst = hbuf0 + buf * hbytes;
    for (int q0 = wave * 64; q0 < hq_total; q0 += NT) {
      const int q = q0 + lane;
      const int hp = q >> 1;
      const int c = (q & 1) ^ ((hp >> 3) & 1);
      const int r = hp / p.hw, cc = hp - r * p.hw;
      const int iy = iy0 + r, ix = ix0 + cc;
      const int ch = c0 + c * E;
      const bool ok = hp < hpix && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w && ch < a.ci;
      const void* src = ok ? (const void*)(xg + ((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + ch)
                           : (const void*)g_lic_zero_page;
      glds16(src, dst + q0 * 16);
    }
  };
  auto issue_w = [&](int s, int buf) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    const int c0 = k * CK;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    const int total = gcur * BN * 2;
    char* dst = wbuf0 + buf * wbytes;
    for (int q0 = wave * 64; q0 < total; q0 += NT) {
      const int q = q0 + lane;
      const int tt = q / (BN * 2);
      const int n = (q >> 1) - tt * BN;
      const int c = (q & 1) ^ ((n >> 3) & 1);
      const T* src = wg + ((int64_t)(n0 + n) * a.ntaps + t0 + tt) * a.cpad + c0 + c * E;
      glds16(src, dst + q0 * 16);
    }
  };

  // per-lane halo base pixel of each 32-row m-tile
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
    issue_halo(0, 0);
    issue_w(0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int s = 0; s < nst; ++s) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    if (s + 1 < nst) issue_w(s + 1, (s + 1) & 1);
    if (g == 0 && k + 1 < nchunks) issue_halo(k + 1, (k + 1) & 1);
    const char* hb = hbuf0 + (k & 1) * hbytes;
    const char* wb = wbuf0 + (s & 1) * wbytes;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    for (int tt = 0; tt < gcur; ++tt) {
      const int toff = stoff[t0 + tt];
      u32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hp = hbase[i] + toff;
        fa[i] = *(const u32x4*)(hb + hp * 32 + ((lhalf ^ ((hp >> 3) & 1)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WTN + j * 32 + lrow;
        fb[j] = *(const u32x4*)(wb + (tt * BN + n) * 32 + ((lhalf ^ ((n >> 3) & 1)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(half8*)&fa[i], *(half8*)&fb[j], acc[i][j], 0, 0, 0);
          } else {
            const float* af = (const float*)&fa[i];
            const float* bf = (const float*)&fb[j];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc[i][j], 0, 0, 0);
          }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue (LDS-staged, one 32x32 tile per wave at a time; see conv.hip)
  float* ct = (float*)smem + wave * (32 * 33);
  const bool vec_ok = epi_vec_ok<T>(a);
  // runtime loop over tiles (the epilogue body is emitted once); the accumulator
  // is read only through the compile-time-indexed selector below
#pragma nounroll
  for (int q = 0; q < TM * TN; ++q) {
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
      if (qq == q) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ct[((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r];
      }
    __syncthreads();
    epilogue_tile<T>(a, ct, rowpix + wm * WTM + (q / TN) * 32, n0 + wn * WTN + (q % TN) * 32, lane, vec_ok);
    __syncthreads();
  }
}

// Returns 1 and launches when the halo kernel applies; 0 to let the caller fall back.
template <typename T, int TH, int TW, int BN, int WM, int WN>
static int try_halo(const lic_conv_args& a, hipStream_t s, int& status) {
  constexpr int E = 16 / (int)sizeof(T);
  constexpr int CK = 2 * E;
  constexpr int NT = WM * WN * 64;
  if (a.copad % BN) return 0;
  if (a.cpad % CK || a.ci % E || a.ldx % E || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt % 16)) return 0;
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
  const int hbytes = p.hpix_pad * 32;
  const int budget = 160 * 1024 - 2 * hbytes - (TH * TW * 4) - 2 * LIC_MAX_TAPS - 64;
  int G = budget / (2 * BN * 32);
  if (G < 1) return 0;
  if (G > a.ntaps) G = a.ntaps;
  p.G = G;
  p.ngroups = (a.ntaps + G - 1) / G;
  p.tiles_y = (a.mi + TH - 1) / TH;
  p.tiles_x = (a.mj + TW - 1) / TW;
  for (int t = 0; t < a.ntaps; ++t) p.toff[t] = (int16_t)((a.dy[t] - dymin) * p.hw + (a.dx[t] - dxmin));
  int smem = 2 * hbytes + 2 * G * BN * 32 + TH * TW * 4 + 2 * LIC_MAX_TAPS;
  const int epi_bytes = (NT / 64) * 32 * 33 * 4;
  if (smem < epi_bytes) smem = epi_bytes;
  p.smem = smem;
  if (smem > 160 * 1024) return 0;
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / BN);
  auto kern = conv_halo_kernel<T, TH, TW, BN, WM, WN>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, grid, dim3(NT), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("halo conv launch: ") + hipGetErrorString(e));
  return 1;
}

template <typename T>
int conv_halo_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.groups != 1 || a.ntaps < 2 || a.prologue != LIC_PRO_NONE || a.force_direct) return 0;
  const int64_t tiles16 = (int64_t)a.n * ((a.mi + 15) / 16) * ((a.mj + 15) / 16);
  if (a.copad % 192 == 0) {
    if (tiles16 * (a.copad / 192) < 200) return 0;
    return try_halo<T, 16, 16, 192, 4, 2>(a, s, status);
  }
  if (a.copad % 128 == 0) {
    if (tiles16 * (a.copad / 128) < 200) return 0;
    return try_halo<T, 16, 16, 128, 4, 2>(a, s, status);
  }
  return 0;
}

template int conv_halo_dispatch<float>(const lic_conv_args&, hipStream_t, int&);
template int conv_halo_dispatch<half_t>(const lic_conv_args&, hipStream_t, int&);

}  // namespace lic
