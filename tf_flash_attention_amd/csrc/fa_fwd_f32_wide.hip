// fa_fwd_f32_wide.hip — fp32 fused attention forward for 128 < max(d, v_d) <= 256: the kernel of
// fa_fwd_f32_impl.h at D = 256 with 32-key tiles (two 64 KB K / V slots beside the 128 KB Q image).
// One wave per SIMD holds the 128 scaled Q fragments and the 128 Oᵀ accumulator registers; this
// translation unit is built with VGPR-form MFMAs (Makefile VGPR_FORM), without which hipcc keeps the
// accumulators in AGPRs and spills 50-68 VGPRs.
#include "fa_fwd_f32_impl.h"

namespace fa {

hipError_t launch_fwd_f32_wide(const FwdArgs& a, hipStream_t s) { return launch_t<256, 32>(a, s); }

}  // namespace fa
