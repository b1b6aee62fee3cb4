// Error handling and library info for liblic.
#include "lic_common.h"
#include <cstring>

namespace lic {
static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
int fail(const std::string& s) {
  g_err = s;
  return 1;
}
}  // namespace lic

extern "C" const char* lic_last_error(void) { return lic::g_err.c_str(); }
extern "C" const char* lic_version(void) { return "liblic 0.1 gfx950"; }
extern "C" int lic_device_arch(char* buf, int32_t len) {
  hipDeviceProp_t p;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return lic::fail("no HIP device");
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return lic::fail("hipGetDeviceProperties failed");
  std::strncpy(buf, p.gcnArchName, (size_t)len - 1);
  buf[len - 1] = 0;
  return 0;
}
