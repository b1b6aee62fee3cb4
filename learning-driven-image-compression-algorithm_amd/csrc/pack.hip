// Weight packing for the conv kernels' [copad][ntaps][cpad] layout, on the device, in one launch
// (include/lic.h lic_pack_taps).  The training path re-packs every conv weight at every step --
// forward pack, transposed + mirrored dgrad pack, stride-s dgrad phases, transposed-conv phases --
// which torch spelled as a zero fill, a flip and a casting copy per pack (and two launches per tap
// before that): ~1300 small launches per net_unet_ha_hs step (rocprofv3 trace r04v).  Here every
// pack is one grid-stride pass that reads the fp32 weight through four signed element strides (a
// flip is a negative stride, a phase a stride of s taps), writes the zero padding itself and
// converts with round-to-nearest-even -- the bytes torch's cast produced.
#include "lic_common.h"

namespace lic {
namespace {

// 32-bit index math (a pack and its source weight stay below 2^31 elements, checked on the host):
// the 64-bit divisions of a first version made the batched launch ~4x slower.
template <typename T>
__device__ __forceinline__ void pack_one(const float* __restrict__ src, int so, int sc, int sy, int sx, int no, int nc,
                                         int ntx, int ntap, int cpad, T* __restrict__ dst, int i) {
  const int r = i / cpad;
  const int c = i - r * cpad;
  const int o = r / ntap;
  const int t = r - o * ntap;
  float v = 0.f;
  if (o < no && c < nc) {
    const int ty = t / ntx, tx = t - ty * ntx;
    v = src[o * so + c * sc + ty * sy + tx * sx];
  }
  dst[i] = from_f<T>(v);
}

template <typename T>
__global__ __launch_bounds__(256) void pack_taps_kernel(const float* __restrict__ src, int so, int sc, int sy, int sx,
                                                        int no, int nc, int nty, int ntx, T* __restrict__ dst,
                                                        int copad, int cpad) {
  const int ntap = nty * ntx;
  const int total = copad * ntap * cpad;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x)
    pack_one<T>(src, so, sc, sy, sx, no, nc, ntx, ntap, cpad, dst, i);
}

template <typename T>
hipError_t launch_pack(const float* src, int64_t so, int64_t sc, int64_t sy, int64_t sx, int no, int nc, int nty,
                       int ntx, void* dst, int copad, int cpad, hipStream_t s) {
  const int64_t total = (int64_t)copad * nty * ntx * cpad;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_taps_kernel<T>, dim3(blocks), dim3(256), 0, s, src, (int)so, (int)sc, (int)sy, (int)sx, no,
                     nc, nty, ntx, (T*)dst, copad, cpad);
  return hipGetLastError();
}

// The kernels index the source with 32-bit element offsets: every stride and the farthest element
// the view can reach must fit.
bool pack_strides_fit(int64_t so, int64_t sc, int64_t sy, int64_t sx, int no, int nc, int nty, int ntx) {
  const int64_t lim = ((int64_t)1 << 31) - 1;
  auto mag = [](int64_t v) { return v < 0 ? -v : v; };
  if (mag(so) > lim || mag(sc) > lim || mag(sy) > lim || mag(sx) > lim) return false;
  const int64_t reach = mag((int64_t)(no > 0 ? no - 1 : 0) * so) + mag((int64_t)(nc > 0 ? nc - 1 : 0) * sc) +
                        mag((int64_t)(nty - 1) * sy) + mag((int64_t)(ntx - 1) * sx);
  return reach <= lim;
}

// All of a step's packs in one launch: desc = n descriptors of LIC_PACK_DESC_WORDS int64 each
// (include/lic.h), sorted by first_block; block b packs elements [(b - first_block) * PACK_BLOCK_ELEMS, +
// PACK_BLOCK_ELEMS) of the descriptor whose block range holds b (binary search).
constexpr int PACK_BLOCK_ELEMS = 2048;

template <typename T>
__device__ __forceinline__ void pack_span(const float* __restrict__ src, int so, int sc, int sy, int sx, int no, int nc,
                                          int ntx, int ntap, int cpad, T* __restrict__ dst, int base, int total) {
  const int end = min(base + PACK_BLOCK_ELEMS, total);
  for (int i = base + threadIdx.x; i < end; i += blockDim.x)
    pack_one<T>(src, so, sc, sy, sx, no, nc, ntx, ntap, cpad, dst, i);
}

__global__ __launch_bounds__(256) void pack_taps_batch_kernel(const int64_t* __restrict__ desc, int n) {
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[(int64_t)mid * LIC_PACK_DESC_WORDS + 13] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* d = desc + (int64_t)lo * LIC_PACK_DESC_WORDS;
  const float* src = (const float*)d[0];
  void* dst = (void*)d[1];
  const int no = (int)d[6], nc = (int)d[7], nty = (int)d[8], ntx = (int)d[9], copad = (int)d[10], cpad = (int)d[11];
  const int dtype = (int)d[12];
  const int ntap = nty * ntx;
  const int total = copad * ntap * cpad;
  const int base = (b - (int)d[13]) * PACK_BLOCK_ELEMS;
  const int so = (int)d[2], sc = (int)d[3], sy = (int)d[4], sx = (int)d[5];
  if (dtype == LIC_F16) pack_span<half_t>(src, so, sc, sy, sx, no, nc, ntx, ntap, cpad, (half_t*)dst, base, total);
  else if (dtype == LIC_BF16) pack_span<bf16_t>(src, so, sc, sy, sx, no, nc, ntx, ntap, cpad, (bf16_t*)dst, base, total);
  else pack_span<float>(src, so, sc, sy, sx, no, nc, ntx, ntap, cpad, (float*)dst, base, total);
}

}  // namespace
}  // namespace lic

extern "C" int32_t lic_pack_block_elems(void) { return lic::PACK_BLOCK_ELEMS; }

extern "C" int lic_pack_taps_batch(const int64_t* desc, int32_t n, int32_t nblocks, lic_stream_t stream) {
  if (!desc || n <= 0 || nblocks <= 0) return lic::fail("lic_pack_taps_batch: need descriptors and blocks");
  hipLaunchKernelGGL(lic::pack_taps_batch_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, desc, n);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lic::fail(std::string("lic_pack_taps_batch: ") + hipGetErrorString(e));
  return 0;
}

extern "C" int lic_pack_taps(int32_t dtype, const float* src, int64_t so, int64_t sc, int64_t sy, int64_t sx,
                             int32_t no, int32_t nc, int32_t nty, int32_t ntx, void* dst, int32_t copad,
                             int32_t cpad, lic_stream_t stream) {
  if (!src || !dst) return lic::fail("lic_pack_taps: null pointer");
  if (no < 0 || nc < 0 || nty <= 0 || ntx <= 0 || copad <= 0 || cpad <= 0 || no > copad || nc > cpad)
    return lic::fail("lic_pack_taps: bad sizes (need 0 <= no <= copad, 0 <= nc <= cpad, taps > 0)");
  if ((int64_t)nty * ntx > LIC_MAX_TAPS * 4) return lic::fail("lic_pack_taps: too many taps");
  if ((int64_t)copad * nty * ntx * cpad >= ((int64_t)1 << 31)) return lic::fail("lic_pack_taps: pack of 2^31 elements or more");
  if (!lic::pack_strides_fit(so, sc, sy, sx, no, nc, nty, ntx))
    return lic::fail("lic_pack_taps: source strides or extent do not fit 32-bit element offsets");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case LIC_F32: e = lic::launch_pack<float>(src, so, sc, sy, sx, no, nc, nty, ntx, dst, copad, cpad, s); break;
    case LIC_F16: e = lic::launch_pack<lic::half_t>(src, so, sc, sy, sx, no, nc, nty, ntx, dst, copad, cpad, s); break;
    case LIC_BF16: e = lic::launch_pack<lic::bf16_t>(src, so, sc, sy, sx, no, nc, nty, ntx, dst, copad, cpad, s); break;
    default: return lic::fail("lic_pack_taps: dtype must be LIC_F32, LIC_F16 or LIC_BF16");
  }
  if (e != hipSuccess) return lic::fail(std::string("lic_pack_taps: ") + hipGetErrorString(e));
  return 0;
}
