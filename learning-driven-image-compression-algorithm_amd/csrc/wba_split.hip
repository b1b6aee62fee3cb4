// fp32x6 WinBasedAttention core in one launch: qkv Linear + shifted-window attention
// (layers/win_attention.py:85-116 qkv -> q*scale, q k^T + relative-position bias (+ -100 region mask),
// softmax, attn v; :154-209 roll / window partition / reverse), for C = 192, 8 heads of 24 channels,
// 8x8 windows -- the Win_noShift_Attention blocks at 64x64 (layers/layers.py:87-102).
//
// Unfused, the qkv 1x1 conv writes a 3C fp32 map (302 MB per call at 64^2 x 32) that the attention
// kernel reads straight back.  Here one workgroup owns one window: its 64 tokens are split once into
// three bf16 planes in LDS, the qkv GEMM of a group of 4 heads goes to LDS, the attention of those
// heads reads it there; with PROJ the attention output is split into the (then free) planes and the
// proj Linear + shortcut finish the block in the same launch (out = x + proj(attn)), else the attention
// output goes to HBM for a separate proj launch.
//
// Bit-identical to the unfused fp32x6 path (conv_split_wd VT 1x1 + win_attn_mfma_kernel<float, 4, 1>):
// every output element sees the same MFMA sequence -- the qkv accumulator runs over the 12 16-channel
// steps in order with the six part products smallest first, 32-channel chunk k split from (-1)^k x and
// the running sum negated at each chunk start (conv_split_wd.h WD_ALT), finished as -acc + bias; the
// attention takes q * scale, K / Q / V / P split by split8_bf16 and the same product order per tile; the
// proj runs the virtual-tap sequence again on the split attention output, then (-acc + bias) + x.
// tests/test_gpu_attn.py::test_fused_wba_bit_exact checks torch.equal against the unfused launches.
#include "lic_common.h"
#include "conv_split.h"

namespace lic {

int wd_env(const char* name, int def);   // conv_split_wd.hip

namespace {

constexpr int WB_C = 192, WB_HEADS = 8, WB_D = 24, WB_WS = 8, WB_T = 64;
constexpr int WB_XS = 200;              // bf16 per token row of a plane: 192 + 8 pad (400 B, conflict-free b128 reads)
constexpr int WB_QS = 100;              // floats per token row of the q / k / v buffers (4 heads x 24 + 4 pad)
constexpr int WB_PLANE = WB_T * WB_XS * 2;          // 25600 B
constexpr int WB_XP = 3 * WB_PLANE;                 // 76800 B
constexpr int WB_QKV = 3 * WB_T * WB_QS * 4;        // 76800 B
constexpr int WB_TAB = 4 * 225 * 4;                 // 3600 B
constexpr int WB_LDS = WB_XP + WB_QKV + WB_TAB;
static_assert(WB_LDS <= 160 * 1024, "LDS");

__device__ __forceinline__ void split8(float4 lo, float4 hi, u32x4 (&out)[3]) {
  uint2 pl[3], ph[3];
  split4<2>(lo, LIC_PRO_NONE, 1.f, pl);
  split4<2>(hi, LIC_PRO_NONE, 1.f, ph);
#pragma unroll
  for (int p = 0; p < 3; ++p) out[p] = u32x4{pl[p].x, pl[p].y, ph[p].x, ph[p].y};
}

}  // namespace

// diagnostic build only (-DW6_STAMP=1, tools/wba_stamps.py): wave 0's per-phase cycle sums (s_memtime),
// written past the end of the output (the caller allocates room); outputs stay valid
#ifndef W6_STAMP
#define W6_STAMP 0
#endif
#if W6_STAMP
#define W6T(v)                                                                           \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#else
#define W6T(v)
#endif

// Persistent: a workgroup per CU walks windows blockIdx.x, + gridDim.x, ...; the next window's
// activations are loaded into registers before the current one's last attention phase (which issues no
// loads), so their HBM latency hides behind it.
template <bool PROJ>
__global__ __launch_bounds__(512, 1) void wba_qkv_attn_kernel(const lic_wba_args a) {
  using SM = SplitMode<2>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xp = smem;                                   // [3 parts][64 tokens][WB_XS] bf16
  float* qkv = (float*)(smem + WB_XP);               // [q, k, v][64 tokens][WB_QS]
  float* tab = (float*)(smem + WB_XP + WB_QKV);      // [4 heads][225]

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int nwx = a.w / WB_WS, nwy = a.h / WB_WS;
  const int nwin = a.n * nwy * nwx;
  // token t of window `win` -> pixel of the un-rolled map (roll(-shift) + window_partition as addressing)
  auto pix_of = [&](int win, int t) -> int {
    const int wx = win % nwx, r = win / nwx, wy = r % nwy, b = r / nwy;
    int py = wy * WB_WS + t / WB_WS + a.shift, px = wx * WB_WS + t % WB_WS + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return (b * a.h + py) * a.w + px;
  };
  float4 v[6];   // this thread's 6 float4 of the (next) window: token f / 48, channels 4 (f % 48) ..
  auto load_x = [&](int win) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int f = tid + 512 * i, t = f / 48, ch = (f % 48) * 4;
      v[i] = *(const float4*)(a.x + (int64_t)pix_of(win, t) * a.ldx + ch);
    }
  };
  if ((int)blockIdx.x < nwin) load_x(blockIdx.x);
#if W6_STAMP
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, t6 = 0, t7 = 0, te = 0;
  unsigned long long s_a = 0, s_b0 = 0, s_gemm = 0, s_b1 = 0, s_s = 0, s_sm = 0, s_pv = 0, s_be = 0;
#endif

  for (int win = blockIdx.x; win < nwin; win += gridDim.x) {
    W6T(t0);
    floatx16 Ok0, Ok1;   // PROJ: this wave's attention output of head group 0 / 1 (head 4g + wave/2)
    const int wx = win % nwx, wy = (win / nwx) % nwy;
    // ---- phase A: the window's 64 x 192 fp32 activations -> three bf16 planes; 32-channel chunk k
    // carries the sign (-1)^k of the unfused kernel's chunk k (conv_split_wd.h, WD_ALT).  (The previous
    // window's last qkv phase, the only reader of the planes, ended at a barrier.)
    {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int f = tid + 512 * i, t = f / 48, ch = (f % 48) * 4;
        uint2 parts[3];
        split4<2>(v[i], LIC_PRO_NONE, ((ch >> 5) & 1) ? -1.f : 1.f, parts);
#pragma unroll
        for (int p = 0; p < 3; ++p) *(uint2*)(xp + p * WB_PLANE + t * (WB_XS * 2) + ch * 2) = parts[p];
      }
    }

    W6T(t1);
#if W6_STAMP
    s_a += t1 - t0;
#endif
    const int nsteps = WB_C / 16;   // 12 sixteen-channel steps of the qkv reduction
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.qkv_wsplit, (short)0, (int)(18 * nsteps * 3 * 1024), 0x00020000);

    for (int g = 0; g < 2; ++g) {   // head groups: heads 4g .. 4g+3
      // planes written (g = 0); the previous group's / window's attention done with qkv / tab
      __syncthreads();
      W6T(t2);

      // ---- phase B: qkv of the group, 2 token tiles x 9 column tiles (q, k, v x 3 of 32) = 18 tiles.
      // Wave w owns local n-tile w for BOTH token tiles, so each weight fragment it loads from L2 feeds
      // two MFMAs (a v1 assignment of one token tile per wave loaded every fragment twice per CU:
      // profiles/r06/wba_f32x6_stamps_v1.txt, GEMM 47 % of the cycles); the ninth n-tile goes by token
      // tile to waves 2g, 2g+1 (waves w and w + 4 share a SIMD: SIMDs 0, 1 take group 0's extra tiles
      // and 2, 3 group 1's, so every SIMD does the same work over the window).  Per output tile the
      // products and their order are v1's: bit-identical.
      const bool ex = (wave >> 1) == g;
      const int tx = wave & 1;
      auto gemm = [&](auto exc) {
        constexpr bool EX = decltype(exc)::value;
        constexpr int NB = EX ? 2 : 1;   // n-tiles: this wave's, + local tile 8
        int jt[NB], which[NB], sub[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int nt = i == 0 ? wave : 8;
          which[i] = nt / 3;
          sub[i] = nt % 3;
          jt[i] = which[i] * 6 + 3 * g + sub[i];   // packed n-tile of qkv columns which*192 + 96g + 32*sub
        }
        floatx16 acc[2], accx;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = accx[r] = 0.f;
        auto load_b = [&](int s, u32x4(&fb)[3][NB]) {
#pragma unroll
          for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p)
              fb[p][i] = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, ((jt[i] * nsteps + s) * 3 + p) * 1024, 0);
        };
        u32x4 fb[3][3][NB], fa[2][3];   // ring of 3 steps: the weights of step s+2 load during step s
        load_b(0, fb[0]);
        load_b(1, fb[1]);
#pragma unroll
        for (int s = 0; s < 12; ++s) {
          if (s + 2 < 12) load_b(s + 2, fb[(s + 2) % 3]);
          if (s > 0 && (s & 1) == 0) {   // chunk start: the running sum changes sign with the chunk's parts
            acc[0] = -acc[0];
            acc[1] = -acc[1];
            if constexpr (EX) accx = -accx;
          }
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int p = 0; p < 3; ++p)
              fa[tt][p] = *(const u32x4*)(xp + p * WB_PLANE + (32 * tt + lr) * (WB_XS * 2) + lh * 16 + s * 32);
#pragma unroll
          for (int pr = SM::NPROD - 1; pr >= 0; --pr) {   // smallest products first
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) acc[tt] = mfma_k16<bf16_t>(fa[tt][SM::PA[pr]], fb[s % 3][SM::PB[pr]][0], acc[tt]);
            if constexpr (EX)
              accx = mfma_k16<bf16_t>(tx ? fa[1][SM::PA[pr]] : fa[0][SM::PA[pr]], fb[s % 3][SM::PB[pr]][NB - 1], accx);
          }
        }
        // six chunks (even): the running sum is -(x w); out = -acc + bias, to the group's q / k / v buffer
        auto store = [&](const floatx16& c, int wh, int sb, int mt) {
          const int col = 32 * sb + lr;
          const float bias = a.qkv_bias[wh * WB_C + 96 * g + col];
          float* dst = qkv + wh * (WB_T * WB_QS) + col;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int t = 32 * mt + 8 * (r >> 2) + 4 * lh + (r & 3);
            dst[t * WB_QS] = -c[r] + bias;
          }
        };
        store(acc[0], which[0], sub[0], 0);
        store(acc[1], which[0], sub[0], 1);
        if constexpr (EX) store(accx, which[NB - 1], sub[NB - 1], tx);
      };
      if (ex) gemm(std::true_type{});
      else gemm(std::false_type{});
      W6T(t3);
      for (int k = tid; k < 4 * 225; k += 512) {
        const int hl = k / 225, e = k - hl * 225;
        tab[k] = a.table[e * a.tab_sr + (4 * g + hl) * a.tab_sh];
      }
      __syncthreads();
      // the next window's activations: loaded now, consumed by its phase A (phase C issues no loads)
      if (g == 1 && win + (int)gridDim.x < nwin) load_x(win + gridDim.x);
      W6T(t4);

      // ---- phase C: attention of the group's 4 heads, wave = (head, query tile); the unfused kernel's
      // per-tile arithmetic (attention_mfma.hip, SPLIT) with q / k / v read from LDS
      {
        const int hl = wave >> 1, ti = wave & 1, h = 4 * g + hl;
        const float* qb = qkv + 24 * hl;
        const float* kb = qkv + WB_T * WB_QS + 24 * hl;
        const float* vb = qkv + 2 * WB_T * WB_QS + 24 * hl;
        const float pre = a.scale;
        floatx16 S[2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[x][r] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int ch = 16 * s + 8 * lh;
          u32x4 kp[2][3], qp[3];
          const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) {
            float4 k0 = z, k1 = z;
            if (ch < WB_D) {
              const float* kr = kb + (32 * tj + lr) * WB_QS + ch;
              k0 = *(const float4*)kr;
              k1 = *(const float4*)(kr + 4);
            }
            split8(k0, k1, kp[tj]);
          }
          float4 q0 = z, q1 = z;
          if (ch < WB_D) {
            const float* qr = qb + (32 * ti + lr) * WB_QS + ch;
            q0 = *(const float4*)qr;
            q1 = *(const float4*)(qr + 4);
          }
          q0 = make_float4(q0.x * pre, q0.y * pre, q0.z * pre, q0.w * pre);
          q1 = make_float4(q1.x * pre, q1.y * pre, q1.z * pre, q1.w * pre);
          split8(q0, q1, qp);
#pragma unroll
          for (int pr = SM::NPROD - 1; pr >= 0; --pr)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) S[tj] = mfma_k16<bf16_t>(kp[tj][SM::PA[pr]], qp[SM::PB[pr]], S[tj]);
        }
        W6T(t5);
        // bias + mask + softmax over the keys of query i (lane column); key j of register r of tile tj:
        // j = 32 tj + 8 (r >> 2) + 4 h + (r & 3)
        const int split = WB_WS - a.shift;
        const bool last_row = wy == nwy - 1, last_col = wx == nwx - 1;
        const bool mask_on = a.mask_kind != 0 && (last_row || last_col);
        auto reg_wba = [&](int y, int x) {
          const int ly = y < a.h - WB_WS ? 0 : (y < a.h - a.shift ? 1 : 2);
          const int lx = x < a.w - WB_WS ? 0 : (x < a.w - a.shift ? 1 : 2);
          return ly * 3 + lx;
        };
        constexpr float L2E = 1.4426950408889634f;
        const int i = 32 * ti + lr;
        const int iy = i / WB_WS, ix = i % WB_WS;
        const float* trow = &tab[hl * 225 + (iy + WB_WS - 1) * 15 + (ix + WB_WS - 1) - 4 * lh];
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[tj][r] = S[tj][r] * 1.f + trow[-((4 * tj + (r >> 2)) * 15 + (r & 3))];
        if (mask_on) {
          const int my_reg = a.mask_kind == 1 ? reg_wba(wy * WB_WS + iy, wx * WB_WS + ix) : 0;
#pragma unroll
          for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int jy = 4 * tj + (r >> 2), jx = 4 * lh + (r & 3);
              if (a.mask_kind == 1) {
                if (reg_wba(wy * WB_WS + jy, wx * WB_WS + jx) != my_reg) S[tj][r] += -100.0f;
              } else if ((last_row && ((iy < split) != (jy < split))) || (last_col && ((ix < split) != (jx < split)))) {
                S[tj][r] = -INFINITY;
              }
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[tj][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mxl = mx * L2E;
        float sum = 0.f;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(S[tj][r], L2E, -mxl));
            S[tj][r] = e;
            sum += e;
          }
        sum += __shfl_xor(sum, 32);
        const float inv = 1.0f / sum;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[tj][r] *= inv;

        W6T(t6);
        // O^T[c][i] = sum_j V^T[c][j] P^T[j][i]: lane (c = lr, half lh) reads V^T row c in the permuted
        // key order of P's registers (keys j0 .. j0+3 and j0+8 .. j0+11)
        floatx16 O;
#pragma unroll
        for (int r = 0; r < 16; ++r) O[r] = 0.f;
        const bool cok = lr < WB_D;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int j0 = 32 * tj + 16 * s2 + 4 * lh;
            float e[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) e[k] = cok ? vb[(j0 + (k & 3) + 8 * (k >> 2)) * WB_QS + lr] : 0.f;
            u32x4 vp[3], pp[3];
            split8(make_float4(e[0], e[1], e[2], e[3]), make_float4(e[4], e[5], e[6], e[7]), vp);
            const int r0 = 8 * s2;
            split8(make_float4(S[tj][r0], S[tj][r0 + 1], S[tj][r0 + 2], S[tj][r0 + 3]),
                   make_float4(S[tj][r0 + 4], S[tj][r0 + 5], S[tj][r0 + 6], S[tj][r0 + 7]), pp);
#pragma unroll
            for (int pr = SM::NPROD - 1; pr >= 0; --pr) O = mfma_k16<bf16_t>(vp[SM::PA[pr]], pp[SM::PB[pr]], O);
          }
        // lane (query i, half lh) holds channels 8q + 4lh + (0..3), q = 0..3 (24 valid)
        if constexpr (PROJ) {
          if (g == 0) Ok0 = O;
          else Ok1 = O;
        } else {
          float* op = a.out + (int64_t)pix_of(win, i) * a.ldo + h * WB_D;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c0 = 8 * q + 4 * lh;
            if (c0 < WB_D) *(float4*)(op + c0) = make_float4(O[4 * q], O[4 * q + 1], O[4 * q + 2], O[4 * q + 3]);
          }
        }
      }
      W6T(t7);
#if W6_STAMP
      s_b0 += t2 - (g == 0 ? t1 : te); s_gemm += t3 - t2; s_b1 += t4 - t3; s_s += t5 - t4; s_sm += t6 - t5; s_pv += t7 - t6;
      te = t7;
#endif
    }
    __syncthreads();   // every wave past this window's phase C (and its qkv GEMMs: the planes are free)
    if constexpr (PROJ) {
      // ---- phase D: the attention output split into the planes (32-channel chunk k from (-1)^k o), then
      // the proj Linear as the unfused virtual-tap launch computes it, + bias + x, at the tokens' pixels
      {
        const int hl = wave >> 1, ti = wave & 1, i = 32 * ti + lr;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const int c0 = (4 * g + hl) * WB_D + 8 * q + 4 * lh;   // 8q + 4lh < 24: q < 3
            const floatx16& Og = g ? Ok1 : Ok0;
            uint2 parts[3];
            split4<2>(make_float4(Og[4 * q], Og[4 * q + 1], Og[4 * q + 2], Og[4 * q + 3]),
                      LIC_PRO_NONE, ((c0 >> 5) & 1) ? -1.f : 1.f, parts);
#pragma unroll
            for (int p = 0; p < 3; ++p) *(uint2*)(xp + p * WB_PLANE + i * (WB_XS * 2) + c0 * 2) = parts[p];
          }
      }
      __syncthreads();
      // 2 token tiles x 6 column tiles: waves 0-3 take two (n-tiles w/2 and 4 + w/2), waves 4-7 one, so the
      // two waves of every SIMD (w, w + 4) hold three tiles together
      const int mt = wave & 1;
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)a.proj_wsplit, (short)0, (int)(6 * nsteps * 3 * 1024), 0x00020000);
      auto proj = [&](auto cnt_c) {
        constexpr int CNT = decltype(cnt_c)::value;
        int jt[CNT];
        jt[0] = wave >> 1;
        if constexpr (CNT > 1) jt[1] = 4 + (wave >> 1);
        floatx16 acc[CNT];
#pragma unroll
        for (int c = 0; c < CNT; ++c)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
        const char* arow = xp + (32 * mt + lr) * (WB_XS * 2) + lh * 16;
        auto load_b = [&](int st, u32x4(&fb)[3][CNT]) {
#pragma unroll
          for (int c = 0; c < CNT; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p)
              fb[p][c] = __builtin_amdgcn_raw_buffer_load_b128(prs, lane * 16, ((jt[c] * nsteps + st) * 3 + p) * 1024, 0);
        };
        u32x4 fb[3][3][CNT], fa[3];
        load_b(0, fb[0]);
        load_b(1, fb[1]);
#pragma unroll
        for (int st = 0; st < 12; ++st) {
          if (st + 2 < 12) load_b(st + 2, fb[(st + 2) % 3]);
          if (st > 0 && (st & 1) == 0)
#pragma unroll
            for (int c = 0; c < CNT; ++c) acc[c] = -acc[c];
#pragma unroll
          for (int p = 0; p < 3; ++p) fa[p] = *(const u32x4*)(arow + p * WB_PLANE + st * 32);
#pragma unroll
          for (int pr = SM::NPROD - 1; pr >= 0; --pr)
#pragma unroll
            for (int c = 0; c < CNT; ++c) acc[c] = mfma_k16<bf16_t>(fa[SM::PA[pr]], fb[st % 3][SM::PB[pr]][c], acc[c]);
        }
        // (-acc + bias) + x, as the unfused epilogue (ct = acc * -1, + bias, + r1).  Register r holds
        // token 32 mt + 8 (r >> 2) + 4 lh + (r & 3): window row 4 mt + (r >> 2), column 4 lh + (r & 3)
        int rowb[4], colx[4];
        {
          const int wb = win / (nwx * nwy);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            int py = wy * WB_WS + 4 * mt + k + a.shift, px = wx * WB_WS + 4 * lh + k + a.shift;
            if (py >= a.h) py -= a.h;
            if (px >= a.w) px -= a.w;
            rowb[k] = (wb * a.h + py) * a.w;
            colx[k] = px;
          }
        }
#pragma unroll
        for (int c = 0; c < CNT; ++c) {
          const int col = 32 * jt[c] + lr;
          const float bias = a.proj_bias[col];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t px = rowb[r >> 2] + colx[r & 3];
            a.out[px * a.ldo + col] = (-acc[c][r] + bias) + a.x[px * a.ldx + col];
          }
        }
      };
      if (wave < 4) proj(std::integral_constant<int, 2>{});
      else proj(std::integral_constant<int, 1>{});
    }
    __syncthreads();   // every wave done with this window before the next window's planes / qkv
#if W6_STAMP
    {
      unsigned long long tz = 0;
      W6T(tz);
      s_be += tz - te;
    }
#endif
  }
#if W6_STAMP
  if (tid == 0) {
    unsigned long long* o = (unsigned long long*)(a.out + (size_t)a.n * a.h * a.w * a.ldo) + (size_t)blockIdx.x * 8;
    o[0] = s_a; o[1] = s_b0; o[2] = s_gemm; o[3] = s_b1; o[4] = s_s; o[5] = s_sm; o[6] = s_pv; o[7] = s_be;
  }
#endif
}

}  // namespace lic

using namespace lic;

extern "C" int lic_wba_qkv_attn_fwd(const lic_wba_args* a, lic_stream_t stream) {
  if (!a) return fail("wba: null args");
  if (a->c != WB_C || a->heads != WB_HEADS || a->ws != WB_WS || a->h % WB_WS || a->w % WB_WS || a->n < 1 ||
      a->shift < 0 || a->shift >= WB_WS || a->mask_kind < 0 || a->mask_kind > 2)
    return fail("wba: the fused kernel takes C = 192, 8 heads, 8x8 windows, H and W multiples of 8");
  if (!a->x || !a->out || !a->qkv_wsplit || !a->qkv_bias || !a->table || (a->proj_wsplit && !a->proj_bias))
    return fail("wba: null pointer");
  if (a->proj_wsplit && ((uintptr_t)a->proj_wsplit & 15)) return fail("wba: proj pack not 16-byte aligned");
  {   // the persistent walker prefetches the next window of x while other workgroups store: out may not
      // overlap x in either mode (and x is the proj shortcut with proj_wsplit)
    const int64_t npix = (int64_t)a->n * a->h * a->w;
    const uintptr_t x0 = (uintptr_t)a->x, x1 = x0 + (uintptr_t)(((npix - 1) * a->ldx + WB_C) * 4);
    const uintptr_t o0 = (uintptr_t)a->out, o1 = o0 + (uintptr_t)(((npix - 1) * a->ldo + WB_C) * 4);
    if (x0 < o1 && o0 < x1) return fail("wba: out must not overlap x");
  }
  if (a->ldx < WB_C || a->ldx % 4 || a->ldo < WB_C || a->ldo % 4 || ((uintptr_t)a->x & 15) || ((uintptr_t)a->out & 15) ||
      ((uintptr_t)a->qkv_wsplit & 15))
    return fail("wba: x / out need 16-byte aligned rows (ld a multiple of 4, >= 192)");
  if ((int64_t)a->n * a->h * a->w * (a->ldx > a->ldo ? a->ldx : a->ldo) >= (1LL << 31))
    return fail("wba: map too large for 32-bit pixel offsets");
  hipStream_t s = (hipStream_t)stream;
  const hipError_t ea = a->proj_wsplit ? ensure_dyn_lds((const void*)wba_qkv_attn_kernel<true>, WB_LDS)
                                       : ensure_dyn_lds((const void*)wba_qkv_attn_kernel<false>, WB_LDS);
  if (ea != hipSuccess) return fail(std::string("wba: dynamic LDS attribute: ") + hipGetErrorString(ea));
  const int64_t windows = (int64_t)a->n * (a->h / WB_WS) * (a->w / WB_WS);
  static int cus[64] = {0};   // one workgroup per CU (157 KB of LDS each), persistent over the windows
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail("wba: hipGetDevice");
  if (cus[dev] <= 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return fail("wba: CU count");
  const int64_t grid = windows < cus[dev] ? windows : cus[dev];
  if (a->proj_wsplit) hipLaunchKernelGGL(wba_qkv_attn_kernel<true>, dim3((unsigned)grid), dim3(512), WB_LDS, s, *a);
  else hipLaunchKernelGGL(wba_qkv_attn_kernel<false>, dim3((unsigned)grid), dim3(512), WB_LDS, s, *a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(std::string("wba launch: ") + hipGetErrorString(e));
}
