// temporary: MFMA fp16 path not yet compiled in
#include "fa_kernels.h"
namespace fa {
bool fwd_f16_supported(const FwdArgs&) { return false; }
hipError_t launch_fwd_f16(const FwdArgs&, hipStream_t) { return hipErrorNotSupported; }
bool bwd_f16_supported(const BwdArgs&) { return false; }
hipError_t launch_bwd_f16(const BwdArgs&, hipStream_t) { return hipErrorNotSupported; }
}
