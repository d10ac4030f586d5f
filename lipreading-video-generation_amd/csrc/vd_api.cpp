// vd_api.cpp -- library-level entry points: version, errors, device info.
#include "vd_common.h"
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

namespace {
thread_local char g_err[512] = "";
}

namespace vd {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VD_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return VD_OK;
}
}  // namespace vd

extern "C" {

int vd_version(void) { return VDIFF_ABI_VERSION; }

const char* vd_last_error(void) { return g_err; }

int vd_device_info(char* buf, int buflen) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return vd::fail(VD_ELAUNCH, "hipGetDevice failed");
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess)
    return vd::fail(VD_ELAUNCH, "hipGetDeviceProperties failed");
  snprintf(buf, (size_t)buflen, "%s;%s;%d;%zu", p.name, p.gcnArchName, p.multiProcessorCount,
           (size_t)p.totalGlobalMem);
  return VD_OK;
}

}  // extern "C"
