// fa_device.h — device-side helpers shared by the HIP kernels (gfx950 only).
#ifndef TF_FLASH_ATTENTION_AMD_FA_DEVICE_H_
#define TF_FLASH_ATTENTION_AMD_FA_DEVICE_H_

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdlib.h>

#include "fa_rules.h"

namespace fa {

// accumulator type per storage type: fp32 for fp16/fp32, fp64 for fp64
template <typename T> struct AccOf { using type = float; };
template <> struct AccOf<double> { using type = double; };

// l/m output element types (flash_attention_forward.cc:151-153, 187-189)
template <typename T> struct LOf { using type = T; };
template <> struct LOf<__half> { using type = float; };

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }

template <typename A, typename T> __device__ __forceinline__ A to_acc(T v) { return static_cast<A>(v); }
template <> __device__ __forceinline__ float to_acc<float, __half>(__half v) { return __half2float(v); }

template <typename T, typename A> __device__ __forceinline__ T from_acc(A v) { return static_cast<T>(v); }
template <> __device__ __forceinline__ __half from_acc<__half, float>(float v) { return __float2half(v); }

// NegInfApprox: every byte 0xFA (type_util.h:43-45) — the value m keeps for
// rows that attend nothing (flash_attention_forward.cc:360-365).
template <typename T> __device__ __forceinline__ T neg_inf_approx();
template <> __device__ __forceinline__ __half neg_inf_approx<__half>() { return __ushort_as_half((unsigned short)0xFAFA); }
template <> __device__ __forceinline__ float neg_inf_approx<float>() { return __uint_as_float(0xFAFAFAFAu); }
template <> __device__ __forceinline__ double neg_inf_approx<double>() { return __longlong_as_double((long long)0xFAFAFAFAFAFAFAFAull); }

__device__ __forceinline__ float fa_exp(float x) { return __expf(x); }
__device__ __forceinline__ double fa_exp(double x) { return exp(x); }
__device__ __forceinline__ float fa_log(float x) { return __logf(x); }
__device__ __forceinline__ double fa_log(double x) { return log(x); }

template <typename A> __device__ __forceinline__ A neg_inf() { return -__builtin_huge_valf(); }
template <> __device__ __forceinline__ double neg_inf<double>() { return -__builtin_huge_val(); }
template <typename A> __device__ __forceinline__ A pos_inf() { return __builtin_huge_valf(); }
template <> __device__ __forceinline__ double pos_inf<double>() { return __builtin_huge_val(); }

// XCD-aware bijective remap of a 1-D grid: consecutive logical ids land on the
// same XCD (blocks b and b+8 share an XCD under round-robin dispatch;
// cdna_hip_programming.md §5 "XCD swizzle must be bijective").  Speed only.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// host: hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), thread-safe
// (fa_api.hip); later launches of the same kernel on the same device skip the runtime call
hipError_t set_smem_once(const void* kern, int bytes);

// host: compute units of the current device, cached per device id (fa_api.hip; thread-safe).
// Persistent grids size themselves from it.
int device_cus();
// host: XCDs of the current device as the CU count implies (32 CUs per gfx950 XCD; a compute
// partition exposes fewer), at least 1, at most 8.  Speed only: the XCD-aware block orders
// assume round-robin dispatch over this many XCDs.
int device_xcds();

#ifdef FA_DIAG
// host, diagnostic library only (libfa_hip_diag.so, built with -DFA_DIAG for tools/): A/B and
// ablation variants are selected from the environment.  The product library has no variant code
// and reads no environment variable.
inline int diag_variant(const char* name) {
  const char* e = getenv(name);
  return e ? atoi(e) : -1;
}
#endif

}  // namespace fa

#endif  // TF_FLASH_ATTENTION_AMD_FA_DEVICE_H_
