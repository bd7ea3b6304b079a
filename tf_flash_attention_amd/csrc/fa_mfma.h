// fa_mfma.h — gfx950 MFMA-kernel helpers shared by the fp16 forward and backward
// translation units: vector types, LDS transposed reads, buffer descriptors and
// half-wave reductions.  Device code only (gfx950).
#ifndef TF_FLASH_ATTENTION_AMD_FA_MFMA_H_
#define TF_FLASH_ATTENTION_AMD_FA_MFMA_H_

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace fa {
namespace mf {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef short v4i16 __attribute__((__vector_size__(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16_t;
typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2_t;
typedef __attribute__((address_space(3))) half8 lds_half8_t;
typedef __attribute__((address_space(3))) floatx4 lds_f4_t;
typedef __attribute__((address_space(3))) float lds_f_t;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <int V>
struct IC {
  static constexpr int value = V;
};

// ds_read_b64_tr_b16: 16-lane groups read a 4-row x 16-column block column-major
__device__ __forceinline__ half4 tr_read(const lds_char_t* p) {
  const v4i16 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)p);
  return __builtin_bit_cast(half4, t);
}
__device__ __forceinline__ half8 read_b128(const lds_char_t* p) { return *reinterpret_cast<const lds_half8_t*>(p); }

// max / sum over lanes l and l^32: after the half swap one result holds the lower
// half twice and the other the upper half twice, so a symmetric op needs no select
__device__ __forceinline__ float max_pair32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_pair32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Buffer descriptor over `bytes` bytes at `p`, built from provably wave-uniform
// values (no waterfall loops around the buffer ops; guide T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// 16 bytes at byte offset `voff` + `soff` of the buffer; zeros when `out`
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff, bool out) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, out ? 0x80000000u : voff, soff, 0);
}

// 8 consecutive fp16 elements e..e+7 of the buffer row at byte offset `vrow`, any alignment (one
// 2-B load each): elements at or past n, or of a row that is out of range, read as zeros
__device__ __forceinline__ u32x4 buf_load8h(__amdgpu_buffer_rsrc_t rs, uint32_t vrow, int e, int n, bool rowok) {
  uint32_t hh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool in = rowok && e + j < n;
    hh[j] = __builtin_amdgcn_raw_buffer_load_b16(rs, in ? vrow + 2u * (uint32_t)(e + j) : 0x80000000u, 0, 0);
  }
  return u32x4{hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16)};
}

// 8 consecutive halfs starting at element e of a row of length n (zeros past n)
__device__ __forceinline__ u32x4 load_chunk8(const __half* row, int e, int n, bool vec) {
  if (vec) return (e < n) ? *reinterpret_cast<const u32x4*>(row + e) : u32x4{0, 0, 0, 0};
  unsigned short hh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) hh[j] = (e + j < n) ? __half_as_ushort(row[e + j]) : (unsigned short)0;
  return u32x4{hh[0] | (uint32_t(hh[1]) << 16), hh[2] | (uint32_t(hh[3]) << 16), hh[4] | (uint32_t(hh[5]) << 16),
               hh[6] | (uint32_t(hh[7]) << 16)};
}

__device__ __forceinline__ half8 scale8(half8 x, float s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (_Float16)((float)x[j] * s);
  return x;
}

}  // namespace mf
}  // namespace fa

#endif  // TF_FLASH_ATTENTION_AMD_FA_MFMA_H_
