// Which CUs (XCD, SE, CU) a 512-workgroup grid lands on, on the default
// stream and on streams from hipExtStreamCreateWithCUMask with K CUs masked
// off, to read the mask-bit -> CU mapping behind bench.py --reserve-cus
// (profiles/r04/cu_reserve.txt).  Each workgroup spins ~20 us so the grid is
// resident at once, then records s_getreg(HW_ID) and s_getreg(XCC_ID).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void where(unsigned* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) {  // ~20 us at 100 MHz
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  }
}

static void run(const char* name, hipStream_t s, unsigned* d, int grid) {
  hipLaunchKernelGGL(where, dim3(grid), dim3(256), 0, s, d);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(2 * grid);
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  std::map<int, int> per_xcd;
  std::set<unsigned> cus;
  std::map<int, std::set<unsigned>> cus_per_xcd;
  for (int b = 0; b < grid; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
    per_xcd[xcc]++;
    cus.insert(key);
    cus_per_xcd[xcc].insert(key);
  }
  printf("%-26s distinct CUs %zu | per XCD: workgroups / CUs", name, cus.size());
  for (auto& kv : per_xcd) printf("  x%d %d/%zu", kv.first, kv.second, cus_per_xcd[kv.first].size());
  printf("\n");
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = 2 * cus;
  unsigned* d;
  CK(hipMalloc(&d, 2 * grid * 4));
  run("default stream", 0, d, grid);
  for (int reserve : {8, 16, 32, 64}) {
    for (int pattern = 0; pattern < 2; ++pattern) {
      std::vector<uint32_t> mask((cus + 31) / 32, 0u);
      for (int i = 0; i < cus; ++i) mask[i / 32] |= 1u << (i % 32);
      for (int k = 0; k < reserve; ++k) {
        // pattern 0: evenly spaced bits (bench.py --reserve-cus); 1: the highest bits
        const int i = pattern == 0 ? (int)(((long long)k * cus) / reserve) : cus - 1 - k;
        mask[i / 32] &= ~(1u << (i % 32));
      }
      hipStream_t s;
      CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
      char name[64];
      snprintf(name, sizeof(name), "mask -%d (%s)", reserve, pattern == 0 ? "spread" : "top bits");
      run(name, s, d, grid);
      CK(hipStreamDestroy(s));
    }
  }
  return 0;
}
