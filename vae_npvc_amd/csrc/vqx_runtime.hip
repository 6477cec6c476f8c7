// Error reporting and version of the libvqx C ABI.
#include "vqx_common.h"
#include <stdarg.h>
#include <stdio.h>

namespace vqx {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return -2;
  }
  return 0;
}
}  // namespace vqx

extern "C" const char* vqx_last_error(void) { return vqx::g_err; }
extern "C" int vqx_version(void) { return VQX_ABI_VERSION; }
