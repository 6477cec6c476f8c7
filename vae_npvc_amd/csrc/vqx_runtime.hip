// Error reporting and version of the libvqx C ABI.
#include <hip/hip_ext.h>
#include <stdarg.h>
#include <stdio.h>

#include <vector>

#include "vqx_common.h"

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

// A compute stream restricted to all but `reserve_cus` of the device's CUs
// (hipExtStreamCreateWithCUMask), for measuring what co-resident work (RCCL's
// all-reduce kernels under data parallelism) costs the step: bench.py
// --reserve-cus wraps it as a torch ExternalStream.  Mask bit i is CU i / 8 of
// XCD i % 8 (measured with tools/lab/cu_map.cpp, profiles/r04/cu_reserve.txt;
// a mask that leaves an XCD no CU is ignored by the runtime), so clearing the
// top `reserve_cus` bits takes reserve_cus / 8 CUs from every XCD.
extern "C" int vqx_stream_create_cu_mask(int32_t reserve_cus, vqx_stream_t* out, int32_t* cus_used) {
  if (!out) { vqx::set_error("vqx_stream_create_cu_mask: null stream pointer"); return -1; }
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    vqx::set_error("vqx_stream_create_cu_mask: no device");
    return -2;
  }
  if (reserve_cus < 0 || reserve_cus >= n) {
    vqx::set_error("vqx_stream_create_cu_mask: reserve %d of %d CUs", reserve_cus, n);
    return -1;
  }
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int i = 0; i < n; ++i) mask[i / 32] |= 1u << (i % 32);
  for (int k = 0; k < reserve_cus; ++k) {  // the top bits: even over the XCDs
    const int i = n - 1 - k;
    mask[i / 32] &= ~(1u << (i % 32));
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) {
    vqx::set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    return -2;
  }
  *out = (vqx_stream_t)s;
  if (cus_used) *cus_used = n - reserve_cus;
  return 0;
}

extern "C" int vqx_stream_destroy(vqx_stream_t stream) {
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) {
    vqx::set_error("hipStreamDestroy: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}
