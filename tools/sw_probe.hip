// Single-wave-per-SIMD probe for the d = 64 fp16 forward (round 5).  Question: with ONE wave per
// SIMD owning 64 queries (blocks A and B, staggered by half a tile), can one basic block carry a
// tile-half's 16 MFMAs (Sᵀ of one block, PV of the other) and the other block's softmax (32 exp2,
// 16 cvt_pk, packed max, 16 dot2c row sums) interleaved by sched_group_barrier, at close to the
// matrix pipe's 512 cycles?  The two-wave ping-pong (tools/shape_probe.hip mode 0) spends ≈ 1066
// cycles per interval for the same work.
//   mode 0: compiler-scheduled segment (no pinning)
//   mode 1: pinned, per MFMA: 1 MFMA, 2 transcendental, 3 VALU
//   mode 2: pinned, per MFMA: 1 MFMA, 2 transcendental, 2 VALU (the rest after the last MFMA)
//   mode 3: MFMAs only (the matrix floor)
//   mode 4: VALU only (the issue floor of the softmax alone)
//   mode 5: the segment written as 8 chunks fenced by sched_barrier(0), each chunk 2 MFMAs (one Sᵀ,
//           one PV) and one eighth of the softmax (4 exp2, 2 cvt_pk, 2 dot2c, one max step)
//   mode 6: as 5 with 4 chunks of 4 MFMAs
// One workgroup of 4 waves (one per SIMD) per CU, random operands.  Prints cycles per segment
// (s_memtime), the in-kernel clock and the MFMA TF/s.  Build with -mllvm -amdgpu-mfma-vgpr-form=1
// (accumulators in VGPRs: the softmax reads them without v_accvgpr_read copies).  Usage: sw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ _Float16 rnd_h(uint32_t x) {
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  return (_Float16)(((int)(x & 0xFFFF) - 32768) * (1.f / 16384.f));
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void probe(unsigned long long* out, float* sink, int iters) {
  const int tid = threadIdx.x;
  half8 kf[4][2], qa[4], qb[4], vf[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      kf[s][0][e] = rnd_h(tid * 131 + s * 17 + e + blockIdx.x * 7919);
      kf[s][1][e] = rnd_h(tid * 137 + s * 19 + e + blockIdx.x * 7);
      qa[s][e] = rnd_h(tid * 71 + s * 29 + e * 3 + 101);
      qb[s][e] = rnd_h(tid * 73 + s * 23 + e * 5 + 103);
      vf[s][0][e] = rnd_h(tid * 79 + s * 31 + e * 7 + 107);
      vf[s][1][e] = rnd_h(tid * 83 + s * 37 + e * 11 + 109);
    }
  }
  // scores come out of the MFMAs, P from the softmax
  floatx16 sa[2] = {}, sb[2] = {}, oa[2] = {}, ob[2] = {};
  uint32_t pa[4][4], pb[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int x = 0; x < 4; ++x) pa[s][x] = pb[s][x] = 0x3c003c00u;
  float la[4] = {0.f, 0.f, 0.f, 0.f}, lb[4] = {0.f, 0.f, 0.f, 0.f};
  uint32_t pm = 0;
  constexpr bool MF = MODE != 4, SM = MODE != 3;
  constexpr int NCH = MODE == 5 ? 8 : 4;  // (modes 5, 6) chunks per segment

  // one segment: Sᵀ of block X (sx) and PV of block X (ox, with px); softmax of block Y (sy -> py),
  // row sums of Y's previous P (ly)
  auto segment = [&](floatx16 (&sx)[2], const half8 (&qx)[4], floatx16 (&ox)[2], uint32_t (&px)[4][4],
                     const floatx16 (&sy)[2], uint32_t (&py)[4][4], float (&ly)[4]) __attribute__((always_inline)) {
    if constexpr (SM) {
      const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 4; ++x) ly[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, py[s][x]), one2, ly[x], false);
    }
    if constexpr (MF) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          sx[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[s][t], qx[s], s == 0 ? floatx16{} : sx[t], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const half8 p = __builtin_bit_cast(half8, u32x4{px[s][0], px[s][1], px[s][2], px[s][3]});
#pragma unroll
        for (int u = 0; u < 2; ++u) ox[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, ox[u], 0, 0, 0);
      }
    }
    if constexpr (SM) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const float s0 = sy[s >> 1][8 * (s & 1) + 2 * x], s1 = sy[s >> 1][8 * (s & 1) + 2 * x + 1];
          py[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0), (_Float16)__builtin_amdgcn_exp2f(s1)});
        }
      auto H = [&](int s_, int x) { return __builtin_bit_cast(half2v, py[s_][x]); };
      auto M3 = [](half2v a, half2v b, half2v c) { return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c); };
      half2v a0 = M3(H(0, 0), H(0, 1), H(0, 2)), b0 = M3(H(2, 0), H(2, 1), H(2, 2));
      a0 = M3(a0, H(0, 3), H(1, 0)); b0 = M3(b0, H(2, 3), H(3, 0));
      a0 = M3(a0, H(1, 1), H(1, 2)); b0 = M3(b0, H(3, 1), H(3, 2));
      pm ^= __builtin_bit_cast(uint32_t, M3(M3(a0, H(1, 3), H(3, 3)), b0, b0));
    }
    if constexpr (MODE == 1 || MODE == 2) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x400, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, MODE == 1 ? 3 : 2, 0);
      }
    }
  };
  // modes 5 / 6: chunk k of a segment carries Sᵀ k-step(s) and PV k-step(s) of block X and pairs
  // 2k..2k+1 (mode 5) of block Y's softmax, fenced
  auto segment_chunked = [&](floatx16 (&sx)[2], const half8 (&qx)[4], floatx16 (&ox)[2], uint32_t (&px)[4][4],
                             const floatx16 (&sy)[2], uint32_t (&py)[4][4], float (&ly)[4]) __attribute__((always_inline)) {
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
    uint32_t pn[4][4];
    half2v mx2[2] = {{(_Float16)0.f, (_Float16)0.f}, {(_Float16)0.f, (_Float16)0.f}};
    constexpr int MPC = 16 / NCH;  // MFMAs per chunk
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int m = 0; m < MPC; ++m) {
        const int idx = ch * MPC + m;  // 0..15: even Sᵀ, odd PV (k-step idx / 4, chain)
        const int k = (idx >> 1) >> 1, t = (idx >> 1) & 1;
        if ((idx & 1) == 0) {
          sx[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[k][t], qx[k], k == 0 ? floatx16{} : sx[t], 0, 0, 0);
        } else {
          const half8 p = __builtin_bit_cast(half8, u32x4{px[k][0], px[k][1], px[k][2], px[k][3]});
          ox[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[k][t], p, ox[t], 0, 0, 0);
        }
      }
      // pairs (s, x) = 16 / NCH pairs of block Y
#pragma unroll
      for (int j = 0; j < 16 / NCH; ++j) {
        const int pr = ch * (16 / NCH) + j, s_ = pr >> 2, x = pr & 3;
        const float s0 = sy[s_ >> 1][8 * (s_ & 1) + 2 * x], s1 = sy[s_ >> 1][8 * (s_ & 1) + 2 * x + 1];
        pn[s_][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0), (_Float16)__builtin_amdgcn_exp2f(s1)});
        mx2[pr & 1] = __builtin_elementwise_maximum(mx2[pr & 1], __builtin_bit_cast(half2v, pn[s_][x]));
        ly[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, py[s_][x]), one2, ly[x], false);
        asm volatile("" : "+v"(pn[s_][x]), "+v"(ly[x]), "+v"(mx2[pr & 1]));  // (pinned in its chunk)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_)
#pragma unroll
      for (int x = 0; x < 4; ++x) py[s_][x] = pn[s_][x];
    pm ^= __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(mx2[0], mx2[1]));
  };
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 4) {  // (no MFMAs: keep the scores opaque so the softmax stays in the loop)
#pragma unroll
      for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(sa[t]), "+v"(sb[t]));
    }
    if constexpr (MODE == 5 || MODE == 6) {
      segment_chunked(sa, qa, oa, pa, sb, pb, lb);
      segment_chunked(sb, qb, ob, pb, sa, pa, la);
    } else {
      segment(sa, qa, oa, pa, sb, pb, lb);
      __builtin_amdgcn_sched_barrier(0);
      segment(sb, qb, ob, pb, sa, pa, la);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float acc = la[0] + la[1] + la[2] + la[3] + lb[0] + lb[1] + lb[2] + lb[3] + (float)pm;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += oa[0][i] + oa[1][i] + ob[0][i] + ob[1][i] + sa[0][i] + sb[1][i];
  sink[blockIdx.x * 256 + tid] = acc;
  if ((tid & 63) == 0) {
    out[(blockIdx.x * 4 + (tid >> 6)) * 2] = t1 - t0;
    out[(blockIdx.x * 4 + (tid >> 6)) * 2 + 1] = r1 - r0;
  }
}

template <int MODE>
void run(unsigned long long* out, float* sink, unsigned long long* host) {
  const int iters = 20000, blocks = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(256), 0, 0, out, sink, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  (void)hipMemcpy(host, out, blocks * 4 * 16, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks * 4; ++i) { cyc += (double)host[2 * i]; rt += (double)host[2 * i + 1]; }
  const double per = cyc / (blocks * 4) / (2.0 * iters);
  const double ghz = cyc / rt / 10.0;
  const double flops = MODE == 4 ? 0.0 : 2.0 * 32 * 32 * 16 * 16 * 4 * blocks * 2.0 * iters;
  printf("{\"mode\": %d, \"cycles_per_segment\": %.1f, \"clock_ghz\": %.3f, \"ms\": %.3f, \"mfma_tflops\": %.1f}\n", MODE, per, ghz, ms,
         flops / ms / 1e9);
}

int main() {
  unsigned long long *out, *host;
  float* sink;
  (void)hipMalloc(&out, 256 * 4 * 16);
  (void)hipMalloc(&sink, 256 * 256 * 4);
  host = (unsigned long long*)malloc(256 * 4 * 16);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, sink, host);
    run<1>(out, sink, host);
    run<2>(out, sink, host);
    run<3>(out, sink, host);
    run<4>(out, sink, host);
    run<5>(out, sink, host);
    run<6>(out, sink, host);
  }
  return 0;
}
