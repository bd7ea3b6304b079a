// Single-wave VALU timing probe (round 5): issue cost and dependent latency of the softmax
// instructions of the fp16 forward, and whether a transcendental overlaps independent VALU work of
// the same wave.  One wave per SIMD (256-thread workgroups, one per CU), each sequence run 64 times
// in a loop and timed with s_memtime.  Prints cycles per sequence element.  Usage: trans_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CL "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v30", "v31", "v32", "v33"
#define R4(X) X X X X
#define R16(X) R4(X) R4(X) R4(X) R4(X)

// each sequence is 16 "elements"; the per-element cost is printed
#define S_EXP R16("v_exp_f32 v10, v20\n v_exp_f32 v11, v21\n")          // 2 indep exps / element
#define S_ADD R16("v_add_f32 v10, v20, v21\n v_add_f32 v11, v22, v23\n")  // 2 indep adds
#define S_EXP_ADD R16("v_exp_f32 v10, v20\n v_add_f32 v11, v22, v23\n")   // exp + indep add
#define S_EXP_CVT R16("v_exp_f32 v10, v20\n v_cvt_pk_f16_f32 v11, v22, v23\n")
#define S_EXP_DOT R16("v_exp_f32 v10, v20\n v_dot2c_f32_f16 v11, v22, v23\n")
#define S_EXP_MAX R16("v_exp_f32 v10, v20\n v_pk_maximum3_f16 v11, v22, v23, v24\n")
#define S_EXP2_ADD2 R16("v_exp_f32 v10, v20\n v_exp_f32 v12, v21\n v_add_f32 v11, v22, v23\n v_add_f32 v13, v24, v25\n")
#define S_EXP_ADD3 R16("v_exp_f32 v10, v20\n v_add_f32 v11, v22, v23\n v_add_f32 v12, v24, v25\n v_add_f32 v13, v26, v27\n")
#define S_EXP_DEP R16("v_exp_f32 v10, v20\n v_add_f32 v20, v10, v21\n")   // exp -> dependent add -> next exp
#define S_ADD_DEP R16("v_add_f32 v10, v10, v21\n v_add_f32 v10, v10, v22\n")  // dependent add chain
#define S_DOT_DEP R16("v_dot2c_f32_f16 v10, v22, v23\n v_dot2c_f32_f16 v10, v24, v25\n")  // one dot2c chain
#define S_MAX_DEP R16("v_pk_maximum3_f16 v10, v10, v22, v23\n v_pk_maximum3_f16 v10, v10, v24, v25\n")
#define S_CVT_DEP R16("v_exp_f32 v10, v20\n v_exp_f32 v11, v21\n v_cvt_pk_f16_f32 v12, v10, v11\n")  // exp,exp,cvt of them
#define S_PAIR8 R4("v_exp_f32 v10, v20\n v_exp_f32 v11, v21\n v_exp_f32 v12, v22\n v_exp_f32 v13, v23\n v_cvt_pk_f16_f32 v30, v10, v11\n v_exp_f32 v14, v24\n v_exp_f32 v15, v25\n v_cvt_pk_f16_f32 v31, v12, v13\n v_dot2c_f32_f16 v16, v30, v26\n v_exp_f32 v10, v20\n v_cvt_pk_f16_f32 v32, v14, v15\n v_dot2c_f32_f16 v17, v31, v26\n")
#define S_SEXP R16("s_nop 0\n v_exp_f32 v10, v20\n")   // s_nop + exp

template <int K>
__global__ __launch_bounds__(256, 1) void seq(unsigned long long* out, int iters) {
  asm volatile(
      "v_mov_b32 v20, 0.5\n v_mov_b32 v21, -0.25\n v_mov_b32 v22, 0x3c003c00\n v_mov_b32 v23, 0x3c003c00\n"
      "v_mov_b32 v24, 0x3c003c00\n v_mov_b32 v25, 0x3c003c00\n v_mov_b32 v26, 0x3c003c00\n v_mov_b32 v27, 0x3c003c00\n"
      "v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n" ::: CL);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (K == 0) asm volatile(S_EXP ::: CL);
    if constexpr (K == 1) asm volatile(S_ADD ::: CL);
    if constexpr (K == 2) asm volatile(S_EXP_ADD ::: CL);
    if constexpr (K == 3) asm volatile(S_EXP_CVT ::: CL);
    if constexpr (K == 4) asm volatile(S_EXP_DOT ::: CL);
    if constexpr (K == 5) asm volatile(S_EXP_MAX ::: CL);
    if constexpr (K == 6) asm volatile(S_EXP2_ADD2 ::: CL);
    if constexpr (K == 7) asm volatile(S_EXP_ADD3 ::: CL);
    if constexpr (K == 8) asm volatile(S_EXP_DEP ::: CL);
    if constexpr (K == 9) asm volatile(S_ADD_DEP ::: CL);
    if constexpr (K == 10) asm volatile(S_DOT_DEP ::: CL);
    if constexpr (K == 11) asm volatile(S_MAX_DEP ::: CL);
    if constexpr (K == 12) asm volatile(S_CVT_DEP ::: CL);
    if constexpr (K == 13) asm volatile(S_PAIR8 ::: CL);
    if constexpr (K == 14) asm volatile(S_SEXP ::: CL);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

static const char* kName[] = {"exp,exp", "add,add", "exp,add", "exp,cvt_pk", "exp,dot2c", "exp,pk_max3", "exp,exp,add,add",
                              "exp,add,add,add", "exp->dep add", "add dep chain (2)", "dot2c dep chain (2)", "pk_max3 dep chain (2)",
                              "exp,exp,cvt(dep)", "8-exp softmax slice (12 instr)", "s_nop0,exp"};

template <int K>
void run(unsigned long long* out, unsigned long long* host) {
  const int iters = 2000, blocks = 256;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((seq<K>), dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipDeviceSynchronize();
  }
  (void)hipMemcpy(host, out, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double cyc = 0;
  for (int i = 0; i < blocks * 4; ++i) cyc += (double)host[i];
  const double per = cyc / (blocks * 4) / iters / 16.0;
  printf("{\"seq\": %d, \"name\": \"%s\", \"cycles_per_element\": %.2f}\n", K, kName[K], per);
}

int main() {
  unsigned long long *out, *host;
  (void)hipMalloc(&out, 256 * 4 * 8);
  host = (unsigned long long*)malloc(256 * 4 * 8);
  run<0>(out, host); run<1>(out, host); run<2>(out, host); run<3>(out, host); run<4>(out, host);
  run<5>(out, host); run<6>(out, host); run<7>(out, host); run<8>(out, host); run<9>(out, host);
  run<10>(out, host); run<11>(out, host); run<12>(out, host); run<13>(out, host); run<14>(out, host);
  return 0;
}
