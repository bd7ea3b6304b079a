// fa_fwd_f32.hip — fp32 fused attention forward for max(d, v_d) <= 128 (kernel: fa_fwd_f32_impl.h);
// 128 < max(d, v_d) <= 256 goes to fa_fwd_f32_wide.hip.
#include "fa_fwd_f32_impl.h"

namespace fa {

bool fwd_f32_supported(const FwdArgs& a) {
  return a.d >= 1 && a.v_d >= 1 && a.d <= 256 && a.v_d <= 256 && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f32(const FwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_t<32>(a, s);
  if (dm <= 64) return launch_t<64>(a, s);
  if (dm <= 128) return launch_t<128>(a, s);
  return launch_fwd_f32_wide(a, s);
}

}  // namespace fa
