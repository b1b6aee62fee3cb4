// Shifted-window multi-head self-attention core (gfx950).
//
// One wave (64 lanes) per (image, window, head-group).  Lane l owns query token
// i = l % N of head (l / N) in the group, N = ws*ws (64, 16 or 4 tokens), so a
// wave covers 64/N heads.  q/k/v of the group are staged in LDS as fp32 (the
// cyclic roll and window partition are pure address arithmetic on the NHWC
// qkv map), the N scores of a query live in registers, softmax is computed in
// registers in the reference op order (max, exp(s - max), sum, p/sum), and the
// output token is written back at its original (un-rolled) pixel.
//   WBA  (layers/win_attention.py:85-116): s = (q*scale)·k + B[h][i][j] (+ -100 mask)
//   WMSA (model/Block_unet.py:233-240):    s = (q·k)*scale + B[h][i][j] (-inf mask)
#include "lic_common.h"

namespace lic {

template <typename T, int N, int D>
__global__ __launch_bounds__(64) void win_attn_kernel(const lic_attn_args a) {
  constexpr int HPW = 64 / N;  // heads per wave
  const int d = D > 0 ? D : a.c / a.heads;
  const int ws = a.ws;
  const int nwx = a.w / ws, nwy = a.h / ws;
  const int ngroups = (a.heads + HPW - 1) / HPW;
  int bid = blockIdx.x;
  const int grp = bid % ngroups;
  bid /= ngroups;
  const int wx = bid % nwx;
  bid /= nwx;
  const int wy = bid % nwy;
  const int b = bid / nwy;

  extern __shared__ float sm[];  // [3][HPW][N][d+1]
  const int dp = d + 1;
  float* sq = sm;
  float* sk = sm + HPW * N * dp;
  float* sv = sk + HPW * N * dp;

  const T* qkv = (const T*)a.qkv;
  // cooperative load: element e -> (head hh, token t, channel c)
  const int per = HPW * N * d;
  for (int e = threadIdx.x; e < per; e += 64) {
    const int c = e % d;
    const int t = (e / d) % N;
    const int hh = e / (d * N);
    const int h = grp * HPW + hh;
    float qv = 0.f, kv = 0.f, vv = 0.f;
    if (h < a.heads) {
      const int sy = wy * ws + t / ws, sx = wx * ws + t % ws;
      int py = sy + a.shift, px = sx + a.shift;
      if (py >= a.h) py -= a.h;
      if (px >= a.w) px -= a.w;
      const T* p = qkv + (((int64_t)b * a.h + py) * a.w + px) * a.ldqkv + h * d + c;
      qv = to_f(p[0]);
      kv = to_f(p[a.c]);
      vv = to_f(p[2 * a.c]);
    }
    sq[(hh * N + t) * dp + c] = qv;
    sk[(hh * N + t) * dp + c] = kv;
    sv[(hh * N + t) * dp + c] = vv;
  }
  __syncthreads();

  const int lane = threadIdx.x;
  const int hh = lane / N, i = lane % N;
  const int h = grp * HPW + hh;
  if (h >= a.heads) return;
  const float scale = a.scale;
  const float* qrow = sq + (hh * N + i) * dp;
  const float* kb = sk + hh * N * dp;
  const float* vb = sv + hh * N * dp;
  constexpr int DQ = D > 0 ? D : 1;
  float qreg[DQ];
  if constexpr (D > 0) {
#pragma unroll
    for (int c = 0; c < D; ++c) qreg[c] = a.scale_after ? qrow[c] : qrow[c] * scale;
  }
  auto qv = [&](int c) -> float {
    if constexpr (D > 0) return qreg[c];
    else return a.scale_after ? qrow[c] : qrow[c] * scale;
  };

  // region labels for the masks
  const int iy = i / ws, ix = i % ws;
  const int sy = wy * ws + iy, sx = wx * ws + ix;
  auto reg_wba = [&](int y, int x) {
    const int ly = y < a.h - ws ? 0 : (y < a.h - a.shift ? 1 : 2);
    const int lx = x < a.w - ws ? 0 : (x < a.w - a.shift ? 1 : 2);
    return ly * 3 + lx;
  };
  const int my_reg = a.mask_kind == 1 ? reg_wba(sy, sx) : 0;
  const int split = ws - a.shift;  // WMSA: s = p - shift
  const bool last_row = (wy == nwy - 1), last_col = (wx == nwx - 1);

  float s[N];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float* kj = kb + j * dp;
    float dot = 0.f;
    if constexpr (D > 0) {
#pragma unroll
      for (int c = 0; c < D; ++c) dot += qv(c) * kj[c];
    } else {
      for (int c = 0; c < d; ++c) dot += qv(c) * kj[c];
    }
    if (a.scale_after) dot = dot * scale;
    const int jy = j / ws, jx = j % ws;
    const int r = (iy - jy + ws - 1) * (2 * ws - 1) + (ix - jx + ws - 1);
    float v = dot + a.table[r * a.tab_sr + h * a.tab_sh];
    if (a.mask_kind == 1) {
      if (reg_wba(wy * ws + jy, wx * ws + jx) != my_reg) v += -100.0f;
    } else if (a.mask_kind == 2) {
      bool m = false;
      if (last_row && ((iy < split) != (jy < split))) m = true;
      if (last_col && ((ix < split) != (jx < split))) m = true;
      if (m) v = -INFINITY;
    }
    s[j] = v;
    mx = fmaxf(mx, v);
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    s[j] = expf(s[j] - mx);
    sum += s[j];
  }
  const float inv = 1.0f / sum;
  int py = sy + a.shift, px = sx + a.shift;
  if (py >= a.h) py -= a.h;
  if (px >= a.w) px -= a.w;
  T* out = (T*)a.out + (((int64_t)b * a.h + py) * a.w + px) * a.ldo + h * d;
  for (int c = 0; c < d; ++c) {
    float o = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) o += (s[j] * inv) * vb[j * dp + c];
    out[c] = from_f<T>(o);
  }
}

template <typename T, int N, int D>
static int launch_attn(const lic_attn_args& a, hipStream_t s) {
  constexpr int HPW = 64 / N;
  const int d = a.c / a.heads;
  const int ngroups = (a.heads + HPW - 1) / HPW;
  const int64_t blocks = (int64_t)a.n * (a.h / a.ws) * (a.w / a.ws) * ngroups;
  const size_t shm = (size_t)3 * HPW * N * (d + 1) * sizeof(float);
  if (shm > 64 * 1024) return fail("attn: head_dim too large");
  hipLaunchKernelGGL((win_attn_kernel<T, N, D>), dim3((unsigned)blocks), dim3(64), shm, s, a);
  LIC_CHECK_LAUNCH();
  return 0;
}

template <typename T, int N>
static int attn_dispatch_d(const lic_attn_args& a, hipStream_t s) {
  switch (a.c / a.heads) {
    case 8: return launch_attn<T, N, 8>(a, s);
    case 16: return launch_attn<T, N, 16>(a, s);
    case 24: return launch_attn<T, N, 24>(a, s);
    case 32: return launch_attn<T, N, 32>(a, s);
    default: return launch_attn<T, N, 0>(a, s);
  }
}

int win_attn_mfma_dispatch(const lic_attn_args& a, hipStream_t s, int& status);

template <typename T>
static int attn_dispatch(const lic_attn_args& a, hipStream_t s) {
  int status = 0;
  if (win_attn_mfma_dispatch(a, s, status)) return status;
  switch (a.ws) {
    case 8: return attn_dispatch_d<T, 64>(a, s);
    case 4: return attn_dispatch_d<T, 16>(a, s);
    case 2: return attn_dispatch_d<T, 4>(a, s);
    default: return fail("attn: window size must be 2, 4 or 8");
  }
}

}  // namespace lic

extern "C" int lic_win_attn_fwd(const lic_attn_args* a, lic_stream_t stream) {
  using namespace lic;
  if (!a || !a->qkv || !a->out || !a->table) return fail("attn: null tensor");
  if (a->heads <= 0 || a->c % a->heads) return fail("attn: C % heads != 0");
  if (a->h % a->ws || a->w % a->ws) return fail("attn: H, W must be multiples of the window");
  if (a->shift < 0 || a->shift >= a->ws) return fail("attn: 0 <= shift < ws");
  if (a->mfma_mode != 0 && !(a->mfma_mode == 2 && a->dtype == LIC_F32))
    return fail("attn: mfma_mode must be 0, or 2 with fp32 data");
  if (a->n * (int64_t)a->h * a->w == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == LIC_F32) return attn_dispatch<float>(*a, s);
  if (a->dtype == LIC_F16) return attn_dispatch<half_t>(*a, s);
  if (a->dtype == LIC_BF16) return attn_dispatch<bf16_t>(*a, s);
  return fail("attn: bad dtype");
}
