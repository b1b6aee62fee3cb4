// Window attention on MFMA for 8x8 windows (64 tokens) and head_dim <= 32 (gfx950).
//
// One wave per (image, window, head); a workgroup holds 4 or 8 heads of one window.
// Scores are computed transposed, S^T = K Q^T (keys on the accumulator rows,
// queries on the lanes), so the softmax over keys of a query is a reduction over
// the lane's own registers plus one exchange with lane^32, and the probability
// registers feed O^T = V^T P^T directly as the B operand (the guide's
// "accumulator as the next MFMA's operand": registers 8s..8s+7 are k-step s with
// the permuted key order 16s + 8(e>>2) + 4h + (e&3); V^T is staged in LDS and read
// in that same order).  O^T puts 4 consecutive channels of one query in a lane,
// stored as 8/16-byte runs at the query's original (un-rolled) pixel.
//   fp16: v_mfma_f32_32x32x16_f16 (head_dim padded to 16/32 with zeros)
//   fp32: v_mfma_f32_32x32x2_f32 (exact fp32 products)
//   fp32, mfma_mode 2 ("fp32x6", SPLIT): Q, K, V and P split on the fly into three bf16 parts
//         (conv_split.h), each dot as the 6 part products x0y0 + x0y1 + x1y0 + x0y2 + x1y1 + x2y0
//         on v_mfma_f32_32x32x16_bf16 in the fp16 path's fragment layout (96 MFMAs of 32 cycles
//         per wave instead of 128 of 64 cycles; dropped terms <= 2^-26 of each product)
// Score = dot*scale + rel-pos bias (+ -100 region mask for WBA, -inf last
// row/column mask for WMSA), softmax as max / exp(s-max) / sum / divide.
#include "lic_common.h"
#include "conv_split.h"

namespace lic {

constexpr int AT_N = 64;   // tokens per window (ws = 8)
constexpr int VT_LD = 68;  // padded row (elements) of the V^T staging image

// 8 fp32 values (two float4) -> their three bf16 parts as MFMA fragments (8 x 16-bit each)
__device__ __forceinline__ void split8_bf16(float4 lo, float4 hi, u32x4 (&out)[3]) {
  uint2 pl[3], ph[3];
  split4<2>(lo, LIC_PRO_NONE, 1.f, pl);
  split4<2>(hi, LIC_PRO_NONE, 1.f, ph);
#pragma unroll
  for (int p = 0; p < 3; ++p) out[p] = u32x4{pl[p].x, pl[p].y, ph[p].x, ph[p].y};
}

template <typename T, int NW, int SPLIT = 0>
__global__ __launch_bounds__(NW * 64) void win_attn_mfma_kernel(const lic_attn_args a) {
  static_assert(!SPLIT || sizeof(T) == 4, "split products are for fp32 data");
  using SM = SplitMode<2>;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int d = a.c / a.heads;
  constexpr int ws = 8;
  const int nwx = a.w / ws, nwy = a.h / ws;
  const int hgroups = (a.heads + NW - 1) / NW;
  int bid = blockIdx.x;
  const int hg = bid % hgroups;
  bid /= hgroups;
  const int wx = bid % nwx;
  bid /= nwx;
  const int wy = bid % nwy;
  const int b = bid / nwy;
  const int h = hg * NW + wave;
  const bool active = h < a.heads;
  const int hc = active ? h : 0;

  // Every LDS image is private to its wave (no cross-wave data: only wave-local
  // ordering is needed, see wave_lds_sync).
  __shared__ __attribute__((aligned(16))) T vT[NW][32 * VT_LD];
  __shared__ float tab[NW][(2 * ws - 1) * (2 * ws - 1)];

  // token t -> original pixel (roll(-shift) + window_partition as addressing),
  // computed in registers by each lane that needs it
  auto pix_of = [&](int t) -> int {
    int py = wy * ws + t / ws + a.shift, px = wx * ws + t % ws + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return (b * a.h + py) * a.w + px;
  };
  const int pix_lr0 = pix_of(lr), pix_lr1 = pix_of(32 + lr);
  for (int k = lane; k < (2 * ws - 1) * (2 * ws - 1); k += 64) tab[wave][k] = a.table[k * a.tab_sr + hc * a.tab_sh];

  const T* qkv = (const T*)a.qkv;
  const int64_t ldq = a.ldqkv;
  const int qoff = hc * d, koff = a.c + hc * d, voff = 2 * a.c + hc * d;
  // fp16: K/Q fragments straight from the qkv map (lane (row, h) holds channels
  // 16s + 8h .. +7), issued before the V^T staging so all reads are in flight at once
  u32x4 kf[2][2] = {}, qf[2][2] = {};
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 16 * s + 8 * lh;
      if (ch >= d) continue;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const T* tp = qkv + (int64_t)(t2 ? pix_lr1 : pix_lr0) * ldq;
        kf[s][t2] = *(const u32x4*)(tp + koff + ch);
        qf[s][t2] = *(const u32x4*)(tp + qoff + ch);
      }
    }
  }
  // V^T staging: lane t loads its V row with 16-byte loads (d % (16 / sizeof(T)) == 0)
  // and scatters it transposed into vT[c][t] (zeros for c >= d)
  {
    constexpr int VE = 16 / (int)sizeof(T);
    const T* vp = qkv + (int64_t)pix_of(lane) * ldq + voff;
#pragma unroll
    for (int c0 = 0; c0 < 32; c0 += VE) {
      u32x4 raw = {0u, 0u, 0u, 0u};
      if (c0 < d) raw = *(const u32x4*)(vp + c0);
      const T* e = (const T*)&raw;
#pragma unroll
      for (int k = 0; k < VE; ++k) vT[wave][(c0 + k) * VT_LD + lane] = e[k];
    }
  }
  wave_lds_sync();  // the wave's tab / V^T writes before its reads (wave-private images)

  // fp32 keeps the reference's order (q*scale before the dot unless scale_after);
  // fp16 operands stay unscaled and the scale is applied to the fp32 dot
  const float pre = (sizeof(T) == 4 && !a.scale_after) ? a.scale : 1.f;
  const float scale = (sizeof(T) == 4 && !a.scale_after) ? 1.f : a.scale;
  floatx16 S[2][2];  // [key tile][query tile]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) S[x][y][r] = 0.f;

  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (16 * s >= d) break;
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
          S[tj][ti] = mfma_k16<T>(kf[s][tj], qf[s][ti], S[tj][ti]);
    }
  } else if constexpr (SPLIT) {
    // lane (row, h) splits channels 16s + 8h .. +7 of its key / (pre-scaled) query rows
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (16 * s >= d) break;
      const int ch = 16 * s + 8 * lh;
      u32x4 kp[2][3], qp[2][3];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const float* tp = (const float*)qkv + (int64_t)(t2 ? pix_lr1 : pix_lr0) * ldq;
        float4 k0 = make_float4(0.f, 0.f, 0.f, 0.f), k1 = k0, q0 = k0, q1 = k0;
        if (ch < d) {
          k0 = *(const float4*)(tp + koff + ch);
          k1 = *(const float4*)(tp + koff + ch + 4);
          q0 = *(const float4*)(tp + qoff + ch);
          q1 = *(const float4*)(tp + qoff + ch + 4);
        }
        q0 = make_float4(q0.x * pre, q0.y * pre, q0.z * pre, q0.w * pre);
        q1 = make_float4(q1.x * pre, q1.y * pre, q1.z * pre, q1.w * pre);
        split8_bf16(k0, k1, kp[t2]);
        split8_bf16(q0, q1, qp[t2]);
      }
#pragma unroll
      for (int pr = SM::NPROD - 1; pr >= 0; --pr)   // smallest products first
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
            S[tj][ti] = mfma_k16<bf16_t>(kp[tj][SM::PA[pr]], qp[ti][SM::PB[pr]], S[tj][ti]);
    }
  } else {
    for (int k = 0; k < d; k += 2) {
      const int ch = k + lh;
      float kf[2], qf[2];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int64_t pt = t2 ? pix_lr1 : pix_lr0;
        kf[t2] = ch < d ? to_f(qkv[pt * ldq + koff + ch]) : 0.f;
        qf[t2] = ch < d ? to_f(qkv[pt * ldq + qoff + ch]) * pre : 0.f;
      }
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
          S[tj][ti] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[tj], qf[ti], S[tj][ti], 0, 0, 0);
    }
  }

  // scale + bias + mask + softmax over keys (rows) for each query (lane column).
  // Register r of key tile tj holds key j = 32tj + 8(r>>2) + 4h + (r&3), i.e. key row
  // 4tj + (r>>2), column 4h + (r&3): the bias index (iy-jy+7)*15 + (ix-jx+7) is a
  // per-lane base minus a compile-time offset.  Masks can only differ from zero in
  // the last window row / column (uniform branch).
  const int split = ws - a.shift;
  const bool last_row = wy == nwy - 1, last_col = wx == nwx - 1;
  const bool mask_on = a.mask_kind != 0 && (last_row || last_col);
  auto reg_wba = [&](int y, int x) {
    const int ly = y < a.h - ws ? 0 : (y < a.h - a.shift ? 1 : 2);
    const int lx = x < a.w - ws ? 0 : (x < a.w - a.shift ? 1 : 2);
    return ly * 3 + lx;
  };
  constexpr float L2E = 1.4426950408889634f;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti) {
    const int i = 32 * ti + lr;
    const int iy = i / ws, ix = i % ws;
    const float* trow = &tab[wave][(iy + ws - 1) * (2 * ws - 1) + (ix + ws - 1) - 4 * lh];
    float mx = -INFINITY;
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = S[tj][ti][r] * scale + trow[-((4 * tj + (r >> 2)) * (2 * ws - 1) + (r & 3))];
        S[tj][ti][r] = v;
      }
    if (mask_on) {
      const int my_reg = a.mask_kind == 1 ? reg_wba(wy * ws + iy, wx * ws + ix) : 0;
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int jy = 4 * tj + (r >> 2), jx = 4 * lh + (r & 3);
          if (a.mask_kind == 1) {
            if (reg_wba(wy * ws + jy, wx * ws + jx) != my_reg) S[tj][ti][r] += -100.0f;
          } else if ((last_row && ((iy < split) != (jy < split))) || (last_col && ((ix < split) != (jx < split)))) {
            S[tj][ti][r] = -INFINITY;
          }
        }
    }
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[tj][ti][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mxl = mx * L2E;
    float sum = 0.f;
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(S[tj][ti][r], L2E, -mxl));
        S[tj][ti][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) S[tj][ti][r] *= inv;
  }

  // O^T[c][i] = sum_j V^T[c][j] P^T[j][i]
  floatx16 O[2];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[ti][r] = 0.f;
  const T* vrow = &vT[wave][lr * VT_LD];
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int j0 = 32 * tj + 16 * s2 + 4 * lh;
        u32x4 va;
        *(uint2*)&va = *(const uint2*)(vrow + j0);
        *((uint2*)&va + 1) = *(const uint2*)(vrow + j0 + 8);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
          u32x4 pb;
          T* pe = (T*)&pb;
#pragma unroll
          for (int e = 0; e < 8; ++e) pe[e] = from_f<T>(S[tj][ti][8 * s2 + e]);
          O[ti] = mfma_k16<T>(va, pb, O[ti]);
        }
      }
  } else if constexpr (SPLIT) {
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int j0 = 32 * tj + 16 * s2 + 4 * lh;
        u32x4 vp[3];
        split8_bf16(*(const float4*)(vrow + j0), *(const float4*)(vrow + j0 + 8), vp);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
          const int r0 = 8 * s2;
          u32x4 pp[3];
          split8_bf16(make_float4(S[tj][ti][r0], S[tj][ti][r0 + 1], S[tj][ti][r0 + 2], S[tj][ti][r0 + 3]),
                      make_float4(S[tj][ti][r0 + 4], S[tj][ti][r0 + 5], S[tj][ti][r0 + 6], S[tj][ti][r0 + 7]), pp);
#pragma unroll
          for (int pr = SM::NPROD - 1; pr >= 0; --pr)
            O[ti] = mfma_k16<bf16_t>(vp[SM::PA[pr]], pp[SM::PB[pr]], O[ti]);
        }
      }
  } else {
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * tj + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float va = vrow[j];
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) O[ti] = __builtin_amdgcn_mfma_f32_32x32x2f32(va, S[tj][ti][r], O[ti], 0, 0, 0);
      }
  }
  if (!active) return;
  // lane (query i, half h) holds channels c = 8g + 4h + (0..3), g = 0..3
  // d % 8 == 0, so a lane's 4 channels are all in range or all out; with an aligned
  // output (checked at dispatch) they go out as one 8-B (fp16) / 16-B (fp32) store
  T* out = (T*)a.out;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti) {
    const int i = 32 * ti + lr;
    T* op = out + (int64_t)(ti ? pix_lr1 : pix_lr0) * a.ldo + h * d;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 8 * g + 4 * lh;
      if (c0 >= d) continue;
      if constexpr (sizeof(T) == 2) {
        uint2 pk;
        T* e = (T*)&pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = from_f<T>(O[ti][4 * g + k]);
        *(uint2*)(op + c0) = pk;
      } else {
        *(float4*)(op + c0) = make_float4(O[ti][4 * g], O[ti][4 * g + 1], O[ti][4 * g + 2], O[ti][4 * g + 3]);
      }
    }
  }
}

int win_attn_mfma_dispatch(const lic_attn_args& a, hipStream_t s, int& status) {
  const int d = a.c / a.heads;
  if (a.ws != 8 || d > 32 || d % 8 || a.ldqkv % 8 || a.force_valu) return 0;
  if ((uintptr_t)a.qkv % 16 || (uintptr_t)a.out % 16 || a.ldo % 4) return 0;
  // fp16 with 8+ heads on a big map: 8 waves (all heads of a window in one workgroup,
  // one L2; 64x64 WBA 97 -> 77 us).  Small maps keep 4 waves for more workgroups, fp32
  // for the LDS (its V^T image is twice the size)
  const int64_t windows = (int64_t)a.n * (a.h / 8) * (a.w / 8);
  const int nw = (a.dtype != LIC_F32 && a.heads >= 8 && windows >= 1024) ? 8 : 4;
  const int64_t blocks = windows * ((a.heads + nw - 1) / nw);
  if (a.dtype == LIC_F16) {
    if (nw == 8) hipLaunchKernelGGL((win_attn_mfma_kernel<half_t, 8>), dim3((unsigned)blocks), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((win_attn_mfma_kernel<half_t, 4>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  } else if (a.dtype == LIC_BF16) {
    if (nw == 8) hipLaunchKernelGGL((win_attn_mfma_kernel<bf16_t, 8>), dim3((unsigned)blocks), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((win_attn_mfma_kernel<bf16_t, 4>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  } else if (a.mfma_mode == 2) {
    hipLaunchKernelGGL((win_attn_mfma_kernel<float, 4, 1>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((win_attn_mfma_kernel<float, 4>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("attn mfma launch: ") + hipGetErrorString(e));
  return 1;
}

}  // namespace lic
