// MFMA-shape probe for the d = 64 fp16 forward's ping-pong (round 5).  Question: does a tile's
// matrix work issued as 32 x v_mfma_f32_16x16x32_f16 (16 cycles each) cost the partner softmax wave
// less than 16 x v_mfma_f32_32x32x16_f16 (32 cycles each), and does the chip hold a higher clock?
// (MI355X_MICROARCH.md 'DVFS give-back' (7): in bare loops the 16x16x32 shape delivered 1.12-1.15x
// the FLOP/s of 32x32x16 at equal cycles, on random data.)
//
// One workgroup per CU, two waves per SIMD, one barrier per interval, roles alternating as in
// fa_fwd_f16_pingpong.hip: in every interval one wave of each SIMD issues one 32-query x 64-key
// tile's matrix work (Sᵀ and PV: 16 MFMAs of 32x32x16 or 32 of 16x16x32, random operands) and
// the other the softmax of one wave-tile (32 exp2, 16 cvt_pk, 8 pk_maximum3, 16 dot2c: the shipped
// kernel's common path, written as C++ on opaque inputs).
//   mode 0: 32x32x16 beside the softmax      mode 1: 16x16x32 beside the softmax
//   mode 2: 32x32x16, partner idle           mode 3: 16x16x32, partner idle
//   mode 4: softmax, partner idle
//   mode 11: 32x32x16 with the Sᵀ and PV chains interleaved (four chains in flight) beside the softmax;
//   mode 12: the same, partner idle
//   modes 5-10: the softmax as a hand-ordered asm stream (tools/gen/softmax_stream.py): lag 1 / dlag 1
//   alone (5) and beside 32x32x16 (6); lag 2 alone (7) and beside (8); dlag 2 alone (9) and beside (10)
// Prints cycles per interval, the in-kernel clock, the MFMA TF/s and the softmax wave's own cycles
// per interval (barrier release to its last VALU issue).  Usage: shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "gen/softmax_stream.h"

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ _Float16 rnd_h(uint32_t x) {
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  return (_Float16)(((int)(x & 0xFFFF) - 32768) * (1.f / 16384.f));
}

// one wave-tile's softmax as a hand-ordered stream: LAG / DLAG as in tools/gen/softmax_stream.py
template <int LAG, int DLAG>
__device__ __forceinline__ void softmax_asm(const float (&s)[32], uint32_t (&p)[16], float (&l)[4], uint32_t& m) {
  float t[6];
#define SIN "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]), "v"(s[8]), "v"(s[9]), \
            "v"(s[10]), "v"(s[11]), "v"(s[12]), "v"(s[13]), "v"(s[14]), "v"(s[15]), "v"(s[16]), "v"(s[17]), "v"(s[18]), \
            "v"(s[19]), "v"(s[20]), "v"(s[21]), "v"(s[22]), "v"(s[23]), "v"(s[24]), "v"(s[25]), "v"(s[26]), "v"(s[27]), \
            "v"(s[28]), "v"(s[29]), "v"(s[30]), "v"(s[31])
#define POUT "=&v"(p[0]), "=&v"(p[1]), "=&v"(p[2]), "=&v"(p[3]), "=&v"(p[4]), "=&v"(p[5]), "=&v"(p[6]), "=&v"(p[7]), \
             "=&v"(p[8]), "=&v"(p[9]), "=&v"(p[10]), "=&v"(p[11]), "=&v"(p[12]), "=&v"(p[13]), "=&v"(p[14]), "=&v"(p[15]), \
             "+v"(l[0]), "+v"(l[1]), "+v"(l[2]), "+v"(l[3]), "=&v"(m)
  if constexpr (LAG == 1 && DLAG == 1)
    asm volatile(SOFTMAX_STREAM_L1_D1 : POUT, "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]) : SIN);
  else if constexpr (LAG == 2 && DLAG == 1)
    asm volatile(SOFTMAX_STREAM_L2_D1 : POUT, "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]) : SIN);
  else
    asm volatile(SOFTMAX_STREAM_L1_D2 : POUT, "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]) : SIN);
#undef SIN
#undef POUT
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(unsigned long long* out, float* sink, int iters) {
  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);  // group: waves 0-3 / 4-7
  half8 fa[4], fb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fa[j][e] = rnd_h(tid * 131 + j * 17 + e + blockIdx.x * 7919);
      fb[j][e] = rnd_h(tid * 71 + j * 29 + e * 3 + 101 + blockIdx.x * 104729);
    }
  floatx16 c32[4] = {};
  floatx4 c16[16] = {};
  float s[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) s[i] = -(float)((tid * 37 + i * 11) % 97) * 0.09f;
  float l[4] = {0.f, 0.f, 0.f, 0.f};
  uint32_t pm = 0;
  constexpr bool ASM = MODE >= 5 && MODE <= 10;
  constexpr int LAG = (MODE == 7 || MODE == 8) ? 2 : 1, DLAG = (MODE == 9 || MODE == 10) ? 2 : 1;
  const bool do_mfma = (MODE != 4 && MODE != 5 && MODE != 7 && MODE != 9), do_soft = (MODE != 2 && MODE != 3 && MODE != 12);
  unsigned long long soft_cyc = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      if (((ph + g) & 1) == 0) {
        if (do_mfma) {
          __builtin_amdgcn_s_setprio(1);
          if constexpr (MODE == 11 || MODE == 12) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int t = 0; t < 2; ++t) {
                c32[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[(k + t) & 3], fb[k], c32[t], 0, 0, 0);
                c32[2 + t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[(k + t) & 3], fa[k], c32[2 + t], 0, 0, 0);
              }
          } else if constexpr (MODE != 1 && MODE != 3) {
            // Sᵀ: 2 chains x 4 k-steps; PV: 2 chains x 4 k-steps
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int t = 0; t < 2; ++t) c32[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[(k + t) & 3], fb[k], c32[t], 0, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int u = 0; u < 2; ++u) c32[2 + u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[(k + u) & 3], fa[k], c32[2 + u], 0, 0, 0);
          } else {
            // Sᵀ: 8 chains (4 key blocks x 2 query blocks) x 2 k-steps; PV: 8 chains x 2 k-steps
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int t = 0; t < 8; ++t) c16[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[(k + t) & 3], fb[(2 * k + t) & 3], c16[t], 0, 0, 0);
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int u = 0; u < 8; ++u) c16[8 + u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[(k + u) & 3], fa[(3 * k + u) & 3], c16[8 + u], 0, 0, 0);
          }
          __builtin_amdgcn_s_setprio(0);
        }
      } else if (do_soft) {
        const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < 32; i += 4) asm volatile("" : "+v"(s[i]), "+v"(s[i + 1]), "+v"(s[i + 2]), "+v"(s[i + 3]));
        uint32_t p[16];
        if constexpr (ASM) {
          uint32_t mm;
          softmax_asm<LAG, DLAG>(s, p, l, mm);
          pm ^= mm;
          asm volatile("s_nop 0" ::: "memory");
          soft_cyc += __builtin_amdgcn_s_memtime() - ts0;
        } else {
#pragma unroll
        for (int x = 0; x < 16; ++x)
          p[x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s[2 * x]), (_Float16)__builtin_amdgcn_exp2f(s[2 * x + 1])});
        auto H = [&](int x) { return __builtin_bit_cast(half2v, p[x]); };
        auto M3 = [](half2v a, half2v b, half2v c) { return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c); };
        half2v a0 = M3(H(0), H(1), H(2)), b0 = M3(H(8), H(9), H(10));
        a0 = M3(a0, H(3), H(4)); b0 = M3(b0, H(11), H(12));
        a0 = M3(a0, H(5), H(6)); b0 = M3(b0, H(13), H(14));
        const half2v m = M3(M3(a0, H(7), H(15)), b0, b0);
        pm ^= __builtin_bit_cast(uint32_t, m);
        const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
        for (int x = 0; x < 16; ++x) l[x & 3] = __builtin_amdgcn_fdot2(H(x), one2, l[x & 3], false);
        __builtin_amdgcn_sched_barrier(0);
        soft_cyc += __builtin_amdgcn_s_memtime() - ts0;
        }
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float acc = l[0] + l[1] + l[2] + l[3] + (float)pm;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += c32[j][i];
#pragma unroll
  for (int j = 0; j < 16; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += c16[j][i];
  sink[blockIdx.x * 512 + tid] = acc;
  if ((tid & 63) == 0) {
    out[(blockIdx.x * 8 + (tid >> 6)) * 2] = t1 - t0;
    out[(blockIdx.x * 8 + (tid >> 6)) * 2 + 1] = r1 - r0;
    out[256 * 8 * 2 + blockIdx.x * 8 + (tid >> 6)] = soft_cyc;
  }
}

template <int MODE>
void run(unsigned long long* out, float* sink, unsigned long long* host) {
  const int iters = 20000, blocks = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 4; ++rep) {  // the clock ramps over the first launches
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(512), 0, 0, out, sink, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  (void)hipMemcpy(host, out, blocks * 8 * 24, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0, sc = 0;
  for (int i = 0; i < blocks * 8; ++i) { cyc += (double)host[2 * i]; rt += (double)host[2 * i + 1]; sc += (double)host[blocks * 16 + i]; }
  const double per = cyc / (blocks * 8) / (2.0 * iters);
  const double ghz = cyc / rt / 10.0;  // s_memrealtime: 100 MHz
  // matrix work: one tile (16 x 32x32x16 = 32 x 16x16x32) per SIMD per interval
  const bool mf = !(MODE == 4 || MODE == 5 || MODE == 7 || MODE == 9);  // (11, 12: MFMAs)
  const double flops = mf ? 2.0 * 32 * 32 * 16 * 16 * 4 * blocks * 2.0 * iters : 0.0;
  // each wave runs the softmax in iters intervals (half of them)
  const double soft = sc / (blocks * 8) / iters;
  printf("{\"mode\": %d, \"cycles_per_interval\": %.1f, \"softmax_wave_cycles\": %.1f, \"clock_ghz\": %.3f, \"ms\": %.3f, \"mfma_tflops\": %.1f}\n",
         MODE, per, soft, ghz, ms, flops / ms / 1e9);
}

int main() {
  unsigned long long *out, *host;
  float* sink;
  (void)hipMalloc(&out, 256 * 8 * 24);
  (void)hipMalloc(&sink, 256 * 512 * 4);
  host = (unsigned long long*)malloc(256 * 8 * 24);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, sink, host);
    run<1>(out, sink, host);
    run<2>(out, sink, host);
    run<3>(out, sink, host);
    run<4>(out, sink, host);
    run<5>(out, sink, host);
    run<6>(out, sink, host);
    run<7>(out, sink, host);
    run<8>(out, sink, host);
    run<9>(out, sink, host);
    run<10>(out, sink, host);
    run<11>(out, sink, host);
    run<12>(out, sink, host);
  }
  return 0;
}
