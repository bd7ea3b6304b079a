// Issue-cost probe for the softmax instructions of the fp16 forward: cycles per wave-instruction
// of v_exp_f32, v_exp_f16 (plain and SDWA into the high half), v_cvt_pk_f16_f32, v_dot2c_f32_f16,
// v_pk_maximum3_f16, v_pk_add_f16 and v_add_f32, with one wave per SIMD, alone and NX of them
// between consecutive v_mfma_f32_32x32x16_f16.  Each wave times its loop with s_memtime (shader
// cycles).  Usage: valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define R8(X) X X X X X X X X

// eight independent instructions of each kind (v10..v17 destinations, v20..v27 sources)
#define OP_EXP32 "v_exp_f32 v10, v20\n v_exp_f32 v11, v21\n v_exp_f32 v12, v22\n v_exp_f32 v13, v23\n" \
                 "v_exp_f32 v14, v24\n v_exp_f32 v15, v25\n v_exp_f32 v16, v26\n v_exp_f32 v17, v27\n"
#define OP_EXP16 "v_exp_f16 v10, v20\n v_exp_f16 v11, v21\n v_exp_f16 v12, v22\n v_exp_f16 v13, v23\n" \
                 "v_exp_f16 v14, v24\n v_exp_f16 v15, v25\n v_exp_f16 v16, v26\n v_exp_f16 v17, v27\n"
#define SDW " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
#define OP_EXP16H "v_exp_f16_sdwa v10, v20" SDW "v_exp_f16_sdwa v11, v21" SDW "v_exp_f16_sdwa v12, v22" SDW \
                  "v_exp_f16_sdwa v13, v23" SDW "v_exp_f16_sdwa v14, v24" SDW "v_exp_f16_sdwa v15, v25" SDW \
                  "v_exp_f16_sdwa v16, v26" SDW "v_exp_f16_sdwa v17, v27" SDW
#define OP_CVT "v_cvt_pk_f16_f32 v10, v20, v21\n v_cvt_pk_f16_f32 v11, v22, v23\n v_cvt_pk_f16_f32 v12, v24, v25\n" \
               "v_cvt_pk_f16_f32 v13, v26, v27\n v_cvt_pk_f16_f32 v14, v20, v22\n v_cvt_pk_f16_f32 v15, v21, v23\n" \
               "v_cvt_pk_f16_f32 v16, v24, v26\n v_cvt_pk_f16_f32 v17, v25, v27\n"
#define OP_DOT "v_dot2c_f32_f16 v10, v20, v21\n v_dot2c_f32_f16 v11, v22, v23\n v_dot2c_f32_f16 v12, v24, v25\n" \
               "v_dot2c_f32_f16 v13, v26, v27\n v_dot2c_f32_f16 v14, v20, v22\n v_dot2c_f32_f16 v15, v21, v23\n" \
               "v_dot2c_f32_f16 v16, v24, v26\n v_dot2c_f32_f16 v17, v25, v27\n"
#define OP_PMAX "v_pk_maximum3_f16 v10, v20, v21, v22\n v_pk_maximum3_f16 v11, v22, v23, v24\n" \
                "v_pk_maximum3_f16 v12, v24, v25, v26\n v_pk_maximum3_f16 v13, v26, v27, v20\n" \
                "v_pk_maximum3_f16 v14, v20, v22, v24\n v_pk_maximum3_f16 v15, v21, v23, v25\n" \
                "v_pk_maximum3_f16 v16, v24, v26, v20\n v_pk_maximum3_f16 v17, v25, v27, v21\n"
#define OP_PADD "v_pk_add_f16 v10, v20, v21\n v_pk_add_f16 v11, v22, v23\n v_pk_add_f16 v12, v24, v25\n" \
                "v_pk_add_f16 v13, v26, v27\n v_pk_add_f16 v14, v20, v22\n v_pk_add_f16 v15, v21, v23\n" \
                "v_pk_add_f16 v16, v24, v26\n v_pk_add_f16 v17, v25, v27\n"
#define OP_ADD "v_add_f32 v10, v20, v21\n v_add_f32 v11, v22, v23\n v_add_f32 v12, v24, v25\n" \
               "v_add_f32 v13, v26, v27\n v_add_f32 v14, v20, v22\n v_add_f32 v15, v21, v23\n" \
               "v_add_f32 v16, v24, v26\n v_add_f32 v17, v25, v27\n"
#define OP_FMAMIX "v_fma_mix_f32 v10, v20, v21, v22 op_sel_hi:[1,1,0]\n v_fma_mix_f32 v11, v22, v23, v24 op_sel_hi:[1,1,0]\n" \
                  "v_fma_mix_f32 v12, v24, v25, v26 op_sel_hi:[1,1,0]\n v_fma_mix_f32 v13, v26, v27, v20 op_sel_hi:[1,1,0]\n" \
                  "v_fma_mix_f32 v14, v20, v22, v24 op_sel_hi:[1,1,0]\n v_fma_mix_f32 v15, v21, v23, v25 op_sel_hi:[1,1,0]\n" \
                  "v_fma_mix_f32 v16, v24, v26, v20 op_sel_hi:[1,1,0]\n v_fma_mix_f32 v17, v25, v27, v21 op_sel_hi:[1,1,0]\n"

#define CLOBS "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27"

// KIND selects the instruction; MF = 0: 64 of them per iteration, alone; MF = 1: 8 MFMAs per
// iteration with 8 of them after each
template <int KIND, int MF>
__global__ __launch_bounds__(256) void probe(unsigned long long* out, int iters) {
  half8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 1e-3f + i); b[i] = (_Float16)(i * 1e-2f); }
  floatx16 c = {};
  asm volatile("v_mov_b32 v20, 0x3c003c00\n v_mov_b32 v21, 0x3c003c00\n v_mov_b32 v22, 0x3c003c00\n v_mov_b32 v23, 0x3c003c00\n"
               "v_mov_b32 v24, 0x3c003c00\n v_mov_b32 v25, 0x3c003c00\n v_mov_b32 v26, 0x3c003c00\n v_mov_b32 v27, 0x3c003c00\n"
               ::: CLOBS);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define BODY(OPS)                                                                                   \
  if constexpr (MF == 0) {                                                                          \
    asm volatile(R8(OPS) ::: CLOBS);                                                                \
  } else {                                                                                          \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                 \
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);                                 \
      asm volatile(OPS ::: CLOBS);                                                                  \
    }                                                                                               \
  }
    if constexpr (KIND == 0) { BODY(OP_EXP32) }
    if constexpr (KIND == 1) { BODY(OP_EXP16) }
    if constexpr (KIND == 2) { BODY(OP_EXP16H) }
    if constexpr (KIND == 3) { BODY(OP_CVT) }
    if constexpr (KIND == 4) { BODY(OP_DOT) }
    if constexpr (KIND == 5) { BODY(OP_PMAX) }
    if constexpr (KIND == 6) { BODY(OP_PADD) }
    if constexpr (KIND == 7) { BODY(OP_ADD) }
    if constexpr (KIND == 8) { BODY(OP_FMAMIX) }
  }
  asm volatile("s_nop 0" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c[i];
  if (threadIdx.x % 64 == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = (t1 - t0) + (s == 12345.f);
}

static const char* kNames[] = {"v_exp_f32", "v_exp_f16", "v_exp_f16_sdwa_hi", "v_cvt_pk_f16_f32", "v_dot2c_f32_f16",
                               "v_pk_maximum3_f16", "v_pk_add_f16", "v_add_f32", "v_fma_mix_f32"};

template <int KIND, int MF>
void run(unsigned long long* out, unsigned long long* host) {
  const int iters = 2000, blocks = 256;
  hipLaunchKernelGGL((probe<KIND, MF>), dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(host, out, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < blocks * 4; ++i) sum += (double)host[i];
  const double cyc = sum / (blocks * 4) / iters;  // per iteration
  if (MF == 0)
    printf("{\"op\": \"%s\", \"beside_mfma\": false, \"cycles_per_instr\": %.2f}\n", kNames[KIND], cyc / 64);
  else
    printf("{\"op\": \"%s\", \"beside_mfma\": true, \"cycles_per_mfma_gap_with_8\": %.2f}\n", kNames[KIND], cyc / 8);
}

template <int K>
void run_all(unsigned long long* out, unsigned long long* host) {
  run<K, 0>(out, host);
  run<K, 1>(out, host);
}

int main() {
  unsigned long long *out, host[256 * 4];
  (void)hipMalloc(&out, sizeof(host));
  run_all<0>(out, host);
  run_all<0>(out, host);  // warm clocks, repeat
  run_all<1>(out, host);
  run_all<2>(out, host);
  run_all<3>(out, host);
  run_all<4>(out, host);
  run_all<5>(out, host);
  run_all<6>(out, host);
  run_all<7>(out, host);
  run_all<8>(out, host);
  return 0;
}
