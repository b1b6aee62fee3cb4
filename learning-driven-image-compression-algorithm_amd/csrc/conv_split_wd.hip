// Dispatch of the weights-direct split-precision convolutions (conv_split_wd.h): which tile
// configuration a launch takes.  The configurations are instantiated in four translation units
// (conv_split_wd_{vt,small,big,7x7}.hip) so that the library builds them in parallel.
#include "conv_split_wd.h"
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

namespace lic {

int wd_env(const char* name, int def) {
  static std::mutex mu;
  static std::map<std::string, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(name);
  if (it != cache.end()) return it->second;
  const char* e = getenv(name);
  const int v = e ? atoi(e) : def;
  cache[name] = v;
  return v;
}

// Returns 1 and launches when a weights-direct tile applies, 0 to let the caller try the
// LDS-staged split kernel (conv_halo_split.hip) or the exact-fp32 kernels.
int conv_split_wd_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.mfma_mode != 2 || !a.wgt_split || a.dtype != LIC_F32) return 0;
  if (a.groups != 1 || a.ntaps < 1 || a.force_direct || a.force_mfma_generic) return 0;
  if (a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE && a.prologue != LIC_PRO_ABS) return 0;
  // 1x1 (qkv / proj Linear, GDN x^2, skips) on big maps: the split of an activation is shared by all
  // 192 output channels of the tile
  if (a.ntaps == 1 && a.mi >= 8 && a.mj >= 16 && (int64_t)a.n * a.mi * a.mj >= 65536 && a.cpad % 32 == 0)
    return wd_dispatch_vt(a, s, status);
  if (wd_dispatch_small(a, s, status)) return 1;
  if (a.ntaps == 49) return wd_dispatch_7x7(a, s, status);
  return wd_dispatch_big(a, s, status);
}

}  // namespace lic
