// Error handling and library info for liblic.
#include "lic_common.h"
#include <cstring>
#include <mutex>
#include <set>
#include <tuple>

namespace lic {
static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
int fail(const std::string& s) {
  g_err = s;
  return 1;
}

hipError_t ensure_dyn_lds(const void* kern, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  const auto key = std::make_tuple(kern, dev, bytes);
  std::lock_guard<std::mutex> g(mu);
  if (done.count(key)) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert(key);
  return e;
}
}  // namespace lic

extern "C" const char* lic_last_error(void) { return lic::g_err.c_str(); }
extern "C" const char* lic_version(void) {
  static char buf[96];
  static std::once_flag once;
  std::call_once(once, [] {
    snprintf(buf, sizeof(buf), "liblic 0.6 gfx950 (abi %d, src %s)", (int)LIC_ABI_VERSION, lic_source_hash());
  });
  return buf;
}
extern "C" int32_t lic_abi_version(void) { return LIC_ABI_VERSION; }
extern "C" int64_t lic_args_size(int32_t which) {
  switch (which) {
    case LIC_ARGS_CONV: return (int64_t)sizeof(lic_conv_args);
    case LIC_ARGS_ATTN: return (int64_t)sizeof(lic_attn_args);
    case LIC_ARGS_RATE: return (int64_t)sizeof(lic_rate_args);
    case LIC_ARGS_RANS: return (int64_t)sizeof(lic_rans_args);
    case LIC_ARGS_WGRAD: return (int64_t)sizeof(lic_wgrad_args);
    case LIC_ARGS_RESUNIT: return (int64_t)sizeof(lic_resunit_args);
    case LIC_ARGS_WBA: return (int64_t)sizeof(lic_wba_args);
    case LIC_ARGS_WBA16: return (int64_t)sizeof(lic_wba16_args);
    default: return -1;
  }
}
extern "C" int lic_device_arch(char* buf, int32_t len) {
  hipDeviceProp_t p;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return lic::fail("no HIP device");
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return lic::fail("hipGetDeviceProperties failed");
  std::strncpy(buf, p.gcnArchName, (size_t)len - 1);
  buf[len - 1] = 0;
  return 0;
}
