// Implicit-GEMM convolution on gfx950 MFMA (+ a direct VALU fallback).
//
// GEMM view: M = output lattice pixels, N = output channels, K = taps x Cin.
// Activations are NHWC, so the K slice of one pixel for one tap is a run of
// contiguous channels: every MFMA operand fragment (8 x f16 or 4 x f32 per
// lane) is one 16-byte load.  A K-step is 64 bytes per row (32 f16 / 16 f32):
//   A tile [BM pixels][64 B], B tile [BN out-channels][64 B] staged in LDS
//   (register-staged double buffer: global loads of step k+1 are in flight
//   while the MFMAs of step k run; one barrier per step), 16-B chunks
//   XOR-swizzled by (row>>2)&3 so the ds_read_b128 lane groups of the 32x32
//   fragment reads are bank-conflict free.
// f16: v_mfma_f32_32x32x16_f16 (fp32 accumulate).
// f32: v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chain); a 16-B fragment holds
//      k = 4h..4h+3 of an 8-wide slab for lane half h, consumed by 4 MFMAs.
//      The permuted k order is applied identically to A and B.
// The epilogue (bias, activation, residual / gate / GDN / half-tanh, channel
// offset + pixel-shuffle addressing, dual store) is fused.
#include "lic_common.h"

namespace lic {

template <typename T, int BM, int BN, int WM, int WN, int PRO>
__global__ __launch_bounds__(WM * WN * 64) void conv_mfma_kernel(const lic_conv_args a, const int M) {
  constexpr int NT = WM * WN * 64;
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 4 * EPC;               // elements per 64-B K-step row
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "tile");
  constexpr int A_CH = BM * 4, B_CH = BN * 4;
  constexpr int A_PT = (A_CH + NT - 1) / NT, B_PT = (B_CH + NT - 1) / NT;
  constexpr int BUF = (BM + BN) * 64;
  static_assert(WM * WN * 32 * 33 * 4 <= 2 * BUF, "epilogue slots overlap rowpix / bias");

  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + BM * 4 + BN * 4 + 2 * LIC_MAX_TAPS];
  int* rowpix = (int*)(smem + 2 * BUF);
  float* sbias = (float*)(rowpix + BM);
  int8_t* tdy = (int8_t*)(sbias + BN);
  int8_t* tdx = tdy + LIC_MAX_TAPS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int mij = a.mi * a.mj;

  if (tid < a.ntaps) { tdy[tid] = a.dy[tid]; tdx[tid] = a.dx[tid]; }
  for (int n = tid; n < BN; n += NT) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;

  // A-row decode (each thread loads chunk (tid&3) of rows (tid>>2) + r*NT/4)
  const int chunk = tid & 3;
  int a_b[A_PT], a_iy[A_PT], a_ix[A_PT];
  bool a_ok[A_PT];
#pragma unroll
  for (int r = 0; r < A_PT; ++r) {
    const int q = tid + r * NT;
    const int row = q >> 2;
    const int m = m0 + row;
    a_ok[r] = (q < A_CH) && (m < M);
    int b = 0, i = 0, j = 0;
    if (a_ok[r]) {
      b = m / mij;
      const int rem = m - b * mij;
      i = rem / a.mj;
      j = rem - i * a.mj;
    }
    a_b[r] = b;
    a_iy[r] = i * a.isy;
    a_ix[r] = j * a.isx;
    if (q < A_CH && chunk == 0) {
      int base = -1;
      if (a_ok[r]) {
        int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
        if (a.out_shuffle == 2) { oy *= 2; ox *= 2; }
        base = (b * a.ho + oy) * a.wo + ox;
      }
      rowpix[row] = base;
    }
  }

  const T* __restrict__ xg = (const T*)a.x;
  const T* __restrict__ wg = (const T*)a.wgt;
  const int kc_steps = a.cpad / BK;
  const int nsteps = a.ntaps * kc_steps;

  u32x4 ra[A_PT], rb[B_PT];
  __syncthreads();

  // Loads are unconditional (clamped addresses, zero-select afterwards) so that
  // no exec-masked branch sits between a global load and its LDS store.
  auto gload = [&](int step) {
    const int t = step / kc_steps;
    const int c0 = (step - t * kc_steps) * BK;
    const int dy = tdy[t], dx = tdx[t];
    const int ch = c0 + chunk * EPC;
#pragma unroll
    for (int r = 0; r < A_PT; ++r) {
      const int iy = a_iy[r] + dy, ix = a_ix[r] + dx;
      const bool ok = a_ok[r] && ch < a.ci && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      const int64_t off = ok ? ((int64_t)(a_b[r] * a.h + iy) * a.w + ix) * a.ldx + ch : 0;
      u32x4 v = *(const u32x4*)(xg + off);
      if (!ok) v = u32x4{0u, 0u, 0u, 0u};
      ra[r] = v;
    }
#pragma unroll
    for (int r = 0; r < B_PT; ++r) {
      int q = tid + r * NT;
      if (B_CH % NT != 0 && q >= B_CH) q = B_CH - 4 + chunk;
      const int n = q >> 2;
      rb[r] = *(const u32x4*)(wg + ((int64_t)(n0 + n) * a.ntaps + t) * a.cpad + c0 + chunk * EPC);
    }
  };

  auto sstore = [&](int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int r = 0; r < A_PT; ++r) {
      const int q = tid + r * NT;
      if (A_CH % NT == 0 || q < A_CH) {
        const int row = q >> 2;
        u32x4 v = ra[r];
        if constexpr (PRO == LIC_PRO_SQUARE) {
          T* e = (T*)&v;
#pragma unroll
          for (int k = 0; k < EPC; ++k) {
            const float f = to_f(e[k]);
            e[k] = from_f<T>(f * f);
          }
        }
        *(u32x4*)(base + row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4)) = v;
      }
    }
#pragma unroll
    for (int r = 0; r < B_PT; ++r) {
      const int q = tid + r * NT;
      if (B_CH % NT == 0 || q < B_CH) {
        const int row = q >> 2;
        *(u32x4*)(base + BM * 64 + row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4)) = rb[r];
      }
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  const int lrow = lane & 31, lhalf = lane >> 5;

  auto compute = [&](int buf) {
    const char* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + lhalf;
      u32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 32 + lrow;
        fa[i] = *(const u32x4*)(base + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 32 + lrow;
        fb[j] = *(const u32x4*)(base + BM * 64 + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            half8 av = *(half8*)&fa[i];
            half8 bv = *(half8*)&fb[j];
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc[i][j], 0, 0, 0);
          } else {
            const float* af = (const float*)&fa[i];
            const float* bf = (const float*)&fb[j];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  if (nsteps > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int step = 0; step < nsteps; ++step) {
      const int cur = step & 1;
      if (step + 1 < nsteps) gload(step + 1);
      compute(cur);
      if (step + 1 < nsteps) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // Epilogue.  Each wave stages one 32x32 accumulator tile at a time through its
  // own LDS slot (the accumulator is only indexed with compile-time constants),
  // then lane l finishes row l>>1, channels (l&1)*16 .. +15 of that tile: bias,
  // activation, residual / gate / GDN / half-tanh, channel-offset + shuffle
  // addressing, contiguous stores.
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

template <typename T, int BM, int BN, int WM, int WN>
static int launch_mfma(const lic_conv_args& a, int M, hipStream_t s) {
  dim3 grid((M + BM - 1) / BM, a.copad / BN);
  if (a.prologue == LIC_PRO_SQUARE)
    hipLaunchKernelGGL((conv_mfma_kernel<T, BM, BN, WM, WN, LIC_PRO_SQUARE>), grid, dim3(WM * WN * 64), 0, s, a, M);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<T, BM, BN, WM, WN, LIC_PRO_NONE>), grid, dim3(WM * WN * 64), 0, s, a, M);
  LIC_CHECK_LAUNCH();
  return 0;
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
  bool mfma_ok = !a.force_direct && a.groups == 1 && a.prologue != LIC_PRO_ABS && a.ci % EPC == 0 && a.cpad % BK == 0 &&
                 a.ldx % EPC == 0 && ((uintptr_t)a.x % 16 == 0) && ((uintptr_t)a.wgt % 16 == 0) &&
                 a.copad % 32 == 0 && a.ci >= EPC;
  if (mfma_ok && !a.force_mfma_generic) {
    int st = 0;
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
  if (a->out_shuffle != 0 && a->out_shuffle != 2) return fail("conv: out_shuffle must be 0 or 2");
  if (a->out_shuffle == 2 && (a->r1 || a->g || a->r2 || a->co % 4)) return fail("conv: shuffle with residual");
  if (a->epi < 0 || a->epi > LIC_EPI_RES_ACT) return fail("conv: bad epilogue");
  if ((a->epi == LIC_EPI_GATE || (a->epi >= LIC_EPI_GDN_DIV && a->epi <= LIC_EPI_GDN_SQRT)) && !a->g) return fail("conv: epilogue needs g");
  if ((a->epi == LIC_EPI_GATE || a->epi == LIC_EPI_HALF_TANH) && !a->r2) return fail("conv: epilogue needs r2");
  if (!a->x || !a->y || !a->wgt) return fail("conv: null tensor");
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == LIC_F32) return conv_dispatch<float>(*a, s);
  if (a->dtype == LIC_F16) return conv_dispatch<half_t>(*a, s);
  return fail("conv: bad dtype");
}
