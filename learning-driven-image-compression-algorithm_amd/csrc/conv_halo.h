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
#pragma once
#include "lic_common.h"

// diagnostic ablations (-DHALO_ABL=bits, timing only; outputs are wrong):
//   1 no in-loop loads, 2 no epilogue, 4 no weight loads, 8 no halo loads
#ifndef HALO_ABL
#define HALO_ABL 0
#endif
#ifndef HALO_LOADERS
#define HALO_LOADERS 4
#endif
#ifndef HALO_STAMP
#define HALO_STAMP 0
#endif
// diagnostic build only (-DHALO_STAMP=1, tools/halo_stamps.py): per-phase s_memtime
// sums per block, written past the end of the output (the caller allocates room)
#if HALO_STAMP
#define HSTAMP(v)                                                                        \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#else
#define HSTAMP(v)
#endif

namespace lic {

static __device__ __attribute__((aligned(256))) unsigned char g_lic_zero_page[256];

struct HaloPlan {
  int hh, hw;      // halo rows / cols
  int hpix_pad;    // halo pixels rounded up to a multiple of 32
  int G;           // taps per stage group
  int ngroups;
  int tiles_y, tiles_x;
  int smem;        // dynamic LDS bytes
  int rp_off;      // byte offset of rowpix[BM] + bias[BN] (past the epilogue slots)
  // taps form a grid in tap order: tap t sits at halo offset
  //   toff0 + (t / nx) * ystep + (t % nx) * xstep   (computed in scalar registers)
  int toff0, nx, ystep, xstep;
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

  const T* __restrict__ xg = (const T*)a.x;
  const T* __restrict__ wg = (const T*)a.wgt;
  const int nchunks = a.cpad / CK;
  const int nst = nchunks * p.ngroups;
  const int hq_total = p.hpix_pad * 2;
  const int hpix = p.hh * p.hw;

  // nw_ld waves move the data, striding by nw_ld * 64 lanes: all waves for the
  // prologue, HALO_LOADERS waves inside the stage loop (see there)
  auto issue_halo = [&](int k, int buf, int nw_ld) {
    const int c0 = k * CK;
    char* dst = hbuf0 + buf * hbytes;
    for (int q0 = wave * 64; q0 < hq_total; q0 += nw_ld * 64) {
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
  auto issue_w = [&](int s, int buf, int nw_ld) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    const int c0 = k * CK;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    const int total = gcur * BN * 2;
    char* dst = wbuf0 + buf * wbytes;
    for (int q0 = wave * 64; q0 < total; q0 += nw_ld * 64) {
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

#if HALO_STAMP
  unsigned long long st_begin = 0, st_loop = 0, st_a = 0, st_b = 0, st_c = 0, st_end = 0, rt_begin = 0, rt_end = 0;
  unsigned long long sum_issue = 0, sum_comp = 0, sum_wait = 0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt_begin)::"memory");
#endif
  HSTAMP(st_begin);
  if (nst > 0) {
    issue_halo(0, 0, NT / 64);
    issue_w(0, 0, NT / 64);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  HSTAMP(st_loop);

  for (int s = 0; s < nst; ++s) {
    const int k = s / p.ngroups, g = s - k * p.ngroups;
    HSTAMP(st_a);
    // Only the first NL waves (one per SIMD when NL = 4: a workgroup's waves are
    // spread cyclically over the 4 SIMDs) issue the next stage's LDS-DMA; an issuing
    // wave stalls while the CU's memory pipeline drains its requests, and the
    // other waves keep the matrix cores busy meanwhile.
    constexpr int NL = HALO_LOADERS < NT / 64 ? HALO_LOADERS : NT / 64;
#if !(HALO_ABL & 1)
    if (wave < NL) {
#if !(HALO_ABL & 4)
      if (s + 1 < nst) issue_w(s + 1, (s + 1) & 1, NL);
#endif
#if !(HALO_ABL & 8)
      if (g == 0 && k + 1 < nchunks) issue_halo(k + 1, (k + 1) & 1, NL);
#endif
    }
#endif
    HSTAMP(st_b);
    const char* hb = hbuf0 + (k & 1) * hbytes;
    const char* wb = wbuf0 + (s & 1) * wbytes;
    const int t0 = g * p.G;
    const int gcur = min(p.G, a.ntaps - t0);
    // fragments of tap tt+1 are read while tap tt's MFMAs run (two register sets);
    // the tap offset is a scalar grid cursor (no memory access inside the loop:
    // an SMEM load would force lgkmcnt(0) and drain the in-flight LDS reads)
    int cy = t0 / p.nx, cx = t0 - cy * p.nx;
    auto load_frags = [&](int tt, u32x4(&fa)[TM], u32x4(&fb)[TN]) {
      const int toff = p.toff0 + cy * p.ystep + cx * p.xstep;
      if (++cx == p.nx) {
        cx = 0;
        ++cy;
      }
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
    };
    auto mfmas = [&](const u32x4(&fa)[TM], const u32x4(&fb)[TN]) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = mfma_k16<T>(fa[i], fb[j], acc[i][j]);
          } else {
            const float* af = (const float*)&fa[i];
            const float* bf = (const float*)&fb[j];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc[i][j], 0, 0, 0);
          }
        }
    };
    u32x4 fa[2][TM], fb[2][TN];
    load_frags(0, fa[0], fb[0]);
    int tt = 0;
    for (; tt + 2 <= gcur; tt += 2) {
      load_frags(tt + 1, fa[1], fb[1]);
      mfmas(fa[0], fb[0]);
      // unconditional (a read past the group's last tap stays inside the LDS
      // allocation and is discarded)
      load_frags(tt + 2, fa[0], fb[0]);
      mfmas(fa[1], fb[1]);
    }
    if (tt < gcur) mfmas(fa[0], fb[0]);
    HSTAMP(st_c);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if HALO_STAMP
    unsigned long long st_d;
    HSTAMP(st_d);
    sum_issue += st_b - st_a;
    sum_comp += st_c - st_b;
    sum_wait += st_d - st_c;
#endif
  }

#if HALO_ABL & 2
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
  // epilogue (LDS-staged, one 32x32 tile per wave at a time; see conv.hip)
  float* ct = (float*)smem + wave * (32 * 33);
  epilogue_all<T, TM * TN, TN>(a, ct, rowpix + wm * WTM, n0 + wn * WTN, sbias + wn * WTN, lane, [&](int q) {
    // the accumulator is read only through compile-time indices
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
      if (qq == q) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ct[((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r];
      }
  });
#if HALO_STAMP
  HSTAMP(st_end);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt_end)::"memory");
  if (tid == 0) {
    unsigned long long* o = (unsigned long long*)((T*)a.y + (size_t)a.n * a.ho * a.wo * a.ldy) +
                             ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
    o[0] = st_loop - st_begin;
    o[1] = sum_issue;
    o[2] = sum_comp;
    o[3] = sum_wait;
    o[4] = st_end - st_loop - sum_issue - sum_comp - sum_wait;
    o[5] = rt_begin;
    o[6] = rt_end;
    o[7] = __smid();
  }
#endif
}

// Returns 1 and launches when the halo kernel applies; 0 to let the caller fall back.
template <typename T, int TH, int TW, int BN, int WM, int WN>
int try_halo(const lic_conv_args& a, hipStream_t s, int& status) {
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
  const int budget = 160 * 1024 - 2 * hbytes - (TH * TW * 4) - BN * 4;
  int G = budget / (2 * BN * 32);
  if (G < 1) return 0;
  if (G > a.ntaps) G = a.ntaps;
  p.G = G;
  p.ngroups = (a.ntaps + G - 1) / G;
  p.tiles_y = (a.mi + TH - 1) / TH;
  p.tiles_x = (a.mj + TW - 1) / TW;
  // tap grid: row length nx = taps sharing the first tap's dy; every tap t must
  // sit at (dy0 + (t/nx)*sy, dx0 + (t%nx)*sx) (kxk convs and the transposed-conv
  // phases of functional.pack_conv_transpose2d all do)
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
  p.rp_off = 2 * hbytes + 2 * G * BN * 32;
  if (p.rp_off < epi_bytes) p.rp_off = epi_bytes;
  const int smem = p.rp_off + TH * TW * 4 + BN * 4;
  p.smem = smem;
  if (smem > 160 * 1024) return 0;
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / BN);
  auto kern = conv_halo_kernel<T, TH, TW, BN, WM, WN>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, 160 * 1024);
  if (ea != hipSuccess) {
    status = fail(std::string("halo conv: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return 1;
  }
  hipLaunchKernelGGL(kern, grid, dim3(NT), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("halo conv launch: ") + hipGetErrorString(e));
  return 1;
}

}  // namespace lic
