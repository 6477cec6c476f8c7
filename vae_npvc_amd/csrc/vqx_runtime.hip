// Error reporting and version of the libvqx C ABI.
#include <hip/hip_ext.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

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

// ---------------------------------------------------------------------------
// Host mailbox for the step statistics (round 6).  A recipe loop reads the
// step's loss values on the host every step (reference bin/train.py:128-132).
// Reading them through an event or a copy puts a marker packet on the compute
// stream, and each such marker idles the stream ~6 us while the next kernel
// waits for it.  Instead the snapshot kernel writes the values straight into
// mapped, coherent pinned host memory and then a per-slot sequence number
// behind a system-scope release; the host polls the number.  Nothing but a
// one-workgroup kernel enters the stream.
struct MailboxHeader {
  int32_t slots, floats;
};

extern "C" int vqx_mailbox_create(int32_t slots, int32_t floats, void** host, void** dev) {
  if (slots < 1 || floats < 1 || floats > 64 || !host || !dev) {
    vqx::set_error("vqx_mailbox_create: 1 <= floats <= 64 per slot, slots >= 1");
    return -1;
  }
  // [slots] uint32 sequence numbers, then [slots][floats] f32 values
  const size_t bytes = (size_t)slots * 4 + (size_t)slots * floats * 4;
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) { vqx::set_error("hipHostMalloc: %s", hipGetErrorString(e)); return -2; }
  memset(h, 0, bytes);
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    vqx::set_error("hipHostGetDevicePointer: %s", hipGetErrorString(e));
    return -2;
  }
  *host = h;
  *dev = d;
  return 0;
}

extern "C" int vqx_mailbox_destroy(void* host) {
  const hipError_t e = hipHostFree(host);
  if (e != hipSuccess) { vqx::set_error("hipHostFree: %s", hipGetErrorString(e)); return -2; }
  return 0;
}

namespace vqx {
// values first (system-scope stores), then every thread's stores released to
// the system before lane 0 of the one wave stores the sequence number
__global__ __launch_bounds__(64) void mailbox_publish_kernel(const float* __restrict__ src, int n, float* dev_copy,
                                                             float* box, uint32_t* seqp, uint32_t seq) {
  const int t = threadIdx.x;
  if (t < n) {
    const float v = src[t];
    if (dev_copy) dev_copy[t] = v;
    __hip_atomic_store(box + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the values before the number
  __syncthreads();
  if (t == 0) __hip_atomic_store(seqp, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace vqx

extern "C" int vqx_mailbox_publish(const float* src, int32_t n, float* dev_copy, void* box_dev, int32_t slot,
                                   int32_t slots, int32_t floats, uint32_t seq, vqx_stream_t stream) {
  if (!src || !box_dev || n < 1 || n > floats || floats > 64 || slot < 0 || slot >= slots) {
    vqx::set_error("vqx_mailbox_publish: bad arguments");
    return -1;
  }
  uint32_t* seqp = (uint32_t*)box_dev + slot;
  float* box = (float*)((uint32_t*)box_dev + slots) + (size_t)slot * floats;
  hipLaunchKernelGGL(vqx::mailbox_publish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, src, n, dev_copy, box,
                     seqp, seq);
  return vqx::launch_status("vqx_mailbox_publish");
}
