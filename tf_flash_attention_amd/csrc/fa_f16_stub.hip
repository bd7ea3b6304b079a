// fp16 MFMA backward not compiled in yet: the generic kernels serve fp16 backward.
#include "fa_kernels.h"
namespace fa {
bool bwd_f16_supported(const BwdArgs&) { return false; }
hipError_t launch_bwd_f16(const BwdArgs&, hipStream_t) { return hipErrorNotSupported; }
}  // namespace fa
