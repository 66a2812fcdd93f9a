// Host-side runtime of libverl_amd: error reporting and diagnostics.
#include <stdarg.h>
#include <stdio.h>

#include "va_common.h"

namespace va {

static thread_local char g_err[512] = {0};

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char *what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return VA_E_LAUNCH;
  }
  return VA_OK;
}

}  // namespace va

extern "C" int va_abi_version(void) { return VA_ABI_VERSION; }

extern "C" const char *va_last_error(void) { return va::g_err; }

extern "C" int va_device_info(int *num_cu, int *arch_major, int *arch_minor) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    va::set_error("hipGetDevice failed");
    return VA_E_LAUNCH;
  }
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) {
    va::set_error("hipGetDeviceProperties failed");
    return VA_E_LAUNCH;
  }
  if (num_cu) *num_cu = p.multiProcessorCount;
  if (arch_major) *arch_major = p.major;
  if (arch_minor) *arch_minor = p.minor;
  return VA_OK;
}
