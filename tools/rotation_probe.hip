// Structure probe for the d = 64 fp16 forward: how long does one barrier interval take when each
// SIMD carries ONE wave issuing a tile's matrix work (16 v_mfma_f32_32x32x16_f16) beside
//   R = 2: one wave issuing a whole tile's softmax mix (the shipped ping-pong), or
//   R = 3: two waves each issuing half a tile's softmax mix (a three-wave rotation),
//   R = 4: three waves each issuing a third of it,
// with the roles rotating every interval, one workgroup barrier per interval.
// The softmax mix of one 32-query x 64-key wave-tile: 32 v_exp_f32, 16 v_cvt_pk_f16_f32,
// 16 v_add_f32 pairs (row sums as f32 adds), 8 v_pk_maximum3_f16 and a few compares.
// Also: VALU-only throughput with 1..3 waves per SIMD.  Each wave stamps s_memtime around its
// loop; the probe prints cycles per interval and the clock (s_memtime / s_memrealtime).
// Usage: rotation_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define CLOBS "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27"

// one "unit" of the softmax mix: 4 exps, 2 conversions, 4 adds, 1 packed max (11 VALU, 4 trans)
#define UNIT                                                                                   \
  "v_exp_f32 v10, v20\n v_cvt_pk_f16_f32 v14, v21, v22\n v_exp_f32 v11, v21\n v_add_f32 v15, v22, v23\n" \
  "v_add_f32 v16, v24, v25\n v_exp_f32 v12, v22\n v_pk_maximum3_f16 v17, v20, v21, v22\n"            \
  "v_exp_f32 v13, v23\n v_cvt_pk_f16_f32 v14, v23, v24\n v_add_f32 v15, v25, v26\n v_add_f32 v16, v26, v27\n"

// half a unit: 2 exps, 1 conversion, 2 adds, 1 packed max
#define HALF_UNIT                                                                              \
  "v_exp_f32 v10, v20\n v_cvt_pk_f16_f32 v14, v21, v22\n v_exp_f32 v11, v21\n v_add_f32 v15, v22, v23\n" \
  "v_add_f32 v16, v24, v25\n v_pk_maximum3_f16 v17, v20, v21, v22\n"

template <int NU>
__device__ __forceinline__ void valu_units() {
#pragma unroll
  for (int u = 0; u < NU; ++u) asm volatile(UNIT ::: CLOBS);
}

// R roles per SIMD (waves w, w+4, w+8, ...).  Interval t: wave group g does MFMA if
// (t + g) % R == 0, else its share of a softmax (8 units / (R-1)).
// SPLIT (R = 2 only): the MFMA wave also issues half of a softmax (one half unit after each MFMA
// pair) and the VALU wave the other half (4 units): the split-softmax ping-pong.
// ACC: 0 = compiler's choice (builtin), 1 = accumulators in arch VGPRs, 2 = in AGPRs, 3 = one of each
// (the Sᵀ chain in VGPRs for the softmax, the PV chain in AGPRs), all by inline asm
template <int ACC>
__device__ __forceinline__ void mfma2(floatx16& c0, floatx16& c1, half8 a, half8 b) {
  if constexpr (ACC == 0) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
  } else if constexpr (ACC == 1) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %3, %0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %3, %1" : "+v"(c0), "+v"(c1) : "v"(a), "v"(b));
  } else if constexpr (ACC == 2) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %3, %0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %3, %1" : "+a"(c0), "+a"(c1) : "v"(a), "v"(b));
  } else {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %3, %0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %3, %1" : "+v"(c0), "+a"(c1) : "v"(a), "v"(b));
  }
}

// PRIO: 0 none, 1 the MFMA phase at s_setprio 1, 2 the VALU phases at s_setprio 1
template <int R, bool SPLIT = false, int ACC = 0, int PRIO = 0>
__global__ __launch_bounds__(256 * R) void rot(unsigned long long* out, int iters) {
  half8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 1e-3f + i); b[i] = (_Float16)(i * 1e-2f); }
  floatx16 c0 = {}, c1 = {};
  asm volatile("v_mov_b32 v20, 0x3c003c00\n v_mov_b32 v21, 0x3c003c00\n v_mov_b32 v22, 0x3c003c00\n v_mov_b32 v23, 0x3c003c00\n"
               "v_mov_b32 v24, 0x3c003c00\n v_mov_b32 v25, 0x3c003c00\n v_mov_b32 v26, 0x3c003c00\n v_mov_b32 v27, 0x3c003c00\n"
               ::: CLOBS);
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x / 256);
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ph = 0; ph < R; ++ph) {
      if ((ph + g) % R == 0) {
        if (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          mfma2<ACC>(c0, c1, a, b);
          if constexpr (SPLIT) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile(HALF_UNIT ::: CLOBS);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if (PRIO == 1) __builtin_amdgcn_s_setprio(0);
      } else {
        if (PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if constexpr (R == 2 && SPLIT) valu_units<4>();
        if constexpr (R == 2 && !SPLIT) valu_units<8>();
        if constexpr (R == 3) valu_units<4>();
        if constexpr (R == 4) { valu_units<3>(); }
        if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
      }
      __syncthreads();
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  if (threadIdx.x % 64 == 0) {
    out[(blockIdx.x * 4 * R + threadIdx.x / 64) * 2] = (t1 - t0) + (s == 12345.f);
    out[(blockIdx.x * 4 * R + threadIdx.x / 64) * 2 + 1] = r1 - r0;
  }
}

// VALU-only throughput: W waves per SIMD, each issuing NU units per iteration
template <int W>
__global__ __launch_bounds__(256 * W) void valu_only(unsigned long long* out, int iters) {
  asm volatile("v_mov_b32 v20, 0x3c003c00\n v_mov_b32 v21, 0x3c003c00\n v_mov_b32 v22, 0x3c003c00\n v_mov_b32 v23, 0x3c003c00\n"
               "v_mov_b32 v24, 0x3c003c00\n v_mov_b32 v25, 0x3c003c00\n v_mov_b32 v26, 0x3c003c00\n v_mov_b32 v27, 0x3c003c00\n"
               ::: CLOBS);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) valu_units<8>();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x % 64 == 0) out[(blockIdx.x * 4 * W + threadIdx.x / 64) * 2] = t1 - t0;
}

template <int R, bool SPLIT = false, int ACC = 0, int PRIO = 0>
void run_rot(unsigned long long* out, unsigned long long* host) {
  const int iters = 4000, blocks = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((rot<R, SPLIT, ACC, PRIO>), dim3(blocks), dim3(256 * R), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  (void)hipMemcpy(host, out, blocks * 4 * R * 16, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks * 4 * R; ++i) { cyc += (double)host[2 * i]; rt += (double)host[2 * i + 1]; }
  const double intervals = (double)iters * R;
  const double per = cyc / (blocks * 4 * R) / intervals;
  const double ghz = cyc / rt / 10.0;  // s_memrealtime runs at 100 MHz
  // matrix work: one tile (16 MFMAs) per SIMD per interval
  const double flops = 2.0 * 32 * 32 * 16 * 16 * 4 * blocks * intervals;
  printf("{\"roles\": %d, \"split\": %d, \"acc\": %d, \"prio\": %d, \"cycles_per_interval\": %.1f, \"clock_ghz\": %.3f, \"tflops\": %.1f}\n", R,
         (int)SPLIT, ACC, PRIO, per, ghz,
         flops / ms / 1e9);
}

template <int W>
void run_valu(unsigned long long* out, unsigned long long* host) {
  const int iters = 4000, blocks = 256;
  hipLaunchKernelGGL((valu_only<W>), dim3(blocks), dim3(256 * W), 0, 0, out, iters);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(host, out, blocks * 4 * W * 16, hipMemcpyDeviceToHost);
  double cyc = 0;
  for (int i = 0; i < blocks * 4 * W; ++i) cyc += (double)host[2 * i];
  const double per_unit = cyc / (blocks * 4 * W) / iters / 8;
  // per SIMD: W waves each issued a unit in per_unit cycles
  printf("{\"valu_waves_per_simd\": %d, \"cycles_per_unit_per_wave\": %.1f, \"simd_cycles_per_unit\": %.1f}\n", W,
         per_unit, per_unit / W);
}

int main() {
  unsigned long long *out, *host;
  (void)hipMalloc(&out, 256 * 16 * 16);
  host = (unsigned long long*)malloc(256 * 16 * 16);
  run_valu<1>(out, host);
  run_rot<2, false, 0, 0>(out, host);
  run_rot<2, false, 0, 1>(out, host);
  run_rot<2, false, 0, 2>(out, host);
  run_rot<2, false, 0, 0>(out, host);
  run_rot<2, false, 0, 1>(out, host);
  run_rot<2, false, 0, 2>(out, host);
  return 0;
}
