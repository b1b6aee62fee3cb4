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
#pragma once
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

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
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
        if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
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
            acc[i][j] = mfma_k16<T>(fa[i], fb[j], acc[i][j]);
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

template <typename T, int BM, int BN, int WM, int WN>
int launch_mfma(const lic_conv_args& a, int M, hipStream_t s) {
  dim3 grid((M + BM - 1) / BM, a.copad / BN);
  if (a.prologue == LIC_PRO_SQUARE)
    hipLaunchKernelGGL((conv_mfma_kernel<T, BM, BN, WM, WN, LIC_PRO_SQUARE>), grid, dim3(WM * WN * 64), 0, s, a, M);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<T, BM, BN, WM, WN, LIC_PRO_NONE>), grid, dim3(WM * WN * 64), 0, s, a, M);
  LIC_CHECK_LAUNCH();
  return 0;
}

}  // namespace lic
