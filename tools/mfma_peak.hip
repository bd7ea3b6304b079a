// Chip-wide fp16 MFMA throughput probe (one and two waves per SIMD): every wave
// issues v_mfma_f32_32x32x16_f16 on 4 independent accumulators, optionally with
// NE independent v_exp_f32 and NA v_add_f32 between consecutive MFMAs, to read
// kernel measurements against what the matrix pipe sustains under full load and
// how much VALU hides beside it.  Usage: mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NE, int NA>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  half8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 1e-3f + i); b[i] = (_Float16)(i * 1e-2f); }
  floatx16 c[4] = {};
  float e[8];
  for (int i = 0; i < 8; ++i) e[i] = threadIdx.x * 1e-4f * i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c[j], 0, 0, 0);
#pragma unroll
      for (int x = 0; x < NE; ++x) e[x] = __builtin_amdgcn_exp2f(e[x]);
#pragma unroll
      for (int x = 0; x < NA; ++x) e[4 + (x & 3)] += 1.0f;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c[0][i] + c[1][i] + c[2][i] + c[3][i];
  for (int i = 0; i < 8; ++i) s += e[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NE, int NA>
void run(float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 10000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int blocks = 256 * wps;  // 4 waves per block: one per SIMD
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((probe<NE, NA>), dim3(blocks), dim3(256), 0, 0, out, iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * blocks * 4;
    printf("{\"exp_per_mfma\": %d, \"add_per_mfma\": %d, \"waves_per_simd\": %d, \"tflops\": %.1f}\n", NE, NA, wps,
           flops / ms / 1e9);
  }
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096);
  run<0, 0>(out);
  run<1, 0>(out);
  run<2, 0>(out);
  run<3, 0>(out);
  run<0, 4>(out);
  run<2, 2>(out);
  run<4, 0>(out);
  return 0;
}
