// fa_kernels.h — launch-argument structs and launcher entry points shared by
// the C-ABI host layer (fa_api.hip) and the kernel translation units.
#ifndef TF_FLASH_ATTENTION_AMD_FA_KERNELS_H_
#define TF_FLASH_ATTENTION_AMD_FA_KERNELS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fa_rules.h"

namespace fa {

struct FwdArgs {
  const void* Q;
  const void* K;
  const void* V;
  void* O;
  void* l;
  void* m;
  int64_t b;
  int32_t d, v_d;
  double scale;  // 1/sqrt(d)
  Rule rule;
};

struct BwdArgs {
  const void* Q;
  const void* K;
  const void* V;
  const void* O;
  const void* l;
  const void* m;
  const void* dO;
  void* dQ;
  void* dK;
  void* dV;
  void* ws_dQ;   // accumulator: b*d*nq of AccT
  void* ws_D;    // b*nq AccT
  void* ws_lse;  // b*nq AccT
  int64_t b;
  int32_t d, v_d;
  double scale;
  Rule rule;
};

// generic (any dtype) path — fa_generic.hip
hipError_t launch_fwd_generic(int dtype, const FwdArgs& a, hipStream_t s);
hipError_t launch_bwd_generic(int dtype, const BwdArgs& a, hipStream_t s);
int generic_max_channels(int dtype);

// fp16 MFMA path — fa_fwd_f16.hip / fa_bwd_f16.hip.  Return hipErrorNotSupported
// when the shape is outside what the MFMA kernels take (caller falls back).
bool fwd_f16_supported(const FwdArgs& a);
hipError_t launch_fwd_f16(const FwdArgs& a, hipStream_t s);
// streamlined fp16 forward for d == v_d in {64, 128} under full / interval rules — fa_fwd_f16_fast.hip
bool fwd_f16_fast_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_fast(const FwdArgs& a, hipStream_t s);
// paired-block fp16 forward for 32 < max(d, v_d) <= 64 (one wave per SIMD) — fa_fwd_f16_pp.hip
bool fwd_f16_pp_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_pp(const FwdArgs& a, hipStream_t s);
// ping-pong fp16 forward (8 waves, two groups alternating MFMA / softmax phases) — fa_fwd_f16_pingpong.hip
bool fwd_f16_pingpong_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_pingpong(const FwdArgs& a, hipStream_t s);
// one-wave-per-SIMD fp16 forward with a hand-placed gap stream, full policy, 32 < max(d, v_d) <= 64 —
// diag/fa_fwd_f16_gap.hip (diagnostic library only: FA_FWD_VARIANT 26xx)
bool fwd_f16_gap_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_gap(const FwdArgs& a, hipStream_t s);
// one-wave gap-stream fp16 forward for 64 < max(d, v_d) <= 128 (full / causal default) — fa_fwd_f16_gap128.hip
bool fwd_f16_gap128_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_gap128(const FwdArgs& a, hipStream_t s);
// ping-pong fp16 forward for 64 < max(d, v_d) <= 128 — fa_fwd_f16_pingpong128.hip
bool fwd_f16_pingpong128_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_pingpong128(const FwdArgs& a, hipStream_t s);
// fp16 forward on MFMA for 128 < max(d, v_d) <= 256: every rule (interval rules by key ranges, strided /
// 2d windows by per-element masks) and any alignment or length (element-wise staging where K / V are not
// 16-B aligned) — fa_fwd_f16_wide.hip
bool fwd_f16_wide_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_wide(const FwdArgs& a, hipStream_t s);
// persistent band forward for 1d unit-stride local windows, 32 < max(d, v_d) <= 64 — fa_fwd_f16_band.hip
bool fwd_f16_band_supported(const FwdArgs& a);
hipError_t launch_fwd_f16_band(const FwdArgs& a, hipStream_t s);
bool bwd_f16_supported(const BwdArgs& a);
// fp32 MFMA forward — fa_fwd_f32.hip
bool fwd_f32_supported(const FwdArgs& a);
hipError_t launch_fwd_f32(const FwdArgs& a, hipStream_t s);
hipError_t launch_fwd_f32_wide(const FwdArgs& a, hipStream_t s);  // fa_fwd_f32_wide.hip (D = 256)
// fp32 MFMA backward (two-pass) — fa_bwd_f32.hip
bool bwd_f32_supported(const BwdArgs& a);
hipError_t launch_bwd_f32(const BwdArgs& a, hipStream_t s);
hipError_t launch_bwd_f32_wide(const BwdArgs& a, hipStream_t s);  // fa_bwd_f32_wide.hip (D = 256, after the prep)
hipError_t launch_bwd_f16(const BwdArgs& a, hipStream_t s);
// fp64 MFMA forward and two-pass backward (d, v_d <= 128) — fa_f64.hip
bool fwd_f64_supported(const FwdArgs& a);
hipError_t launch_fwd_f64(const FwdArgs& a, hipStream_t s);
bool bwd_f64_supported(const BwdArgs& a);
hipError_t launch_bwd_f64(const BwdArgs& a, hipStream_t s);
// dK / dV pass at D = 128 with 64 keys a wave (one wave per SIMD, dK / dV in AGPRs) —
// diag/fa_bwd_f16_k64.hip (diagnostic library only: FA_BWD_VARIANT 1700)
bool bwd_dkdv_k64_supported(const BwdArgs& a);
hipError_t launch_dkdv_k64(const BwdArgs& a, hipStream_t s);
// two-pass fp16 backward (dK/dV key-outer + dQ query-outer, no atomics) — fa_bwd_f16_fast.hip
bool bwd_f16_fast_supported(const BwdArgs& a);
hipError_t launch_bwd_f16_fast(const BwdArgs& a, hipStream_t s);

}  // namespace fa

#endif  // TF_FLASH_ATTENTION_AMD_FA_KERNELS_H_
