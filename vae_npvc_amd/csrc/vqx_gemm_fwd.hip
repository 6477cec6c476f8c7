// Instantiations of the conv GEMM for MODE_FWD (see vqx_gemm_inst.h).
#include "vqx_gemm_inst.h"

namespace vqx {
template void launch_mode_dt<MODE_FWD>(const GemmParams&, int, bool, bool, hipStream_t);
}  // namespace vqx
