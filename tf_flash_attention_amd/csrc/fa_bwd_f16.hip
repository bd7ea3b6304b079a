// fa_bwd_f16.hip — fp16 fused attention backward on gfx950 MFMA.
//
// Replaces the reference's BackwardImpl (flash_attention.cu:1079-1967): scalar
// SIMT GEMMs with a global spin lock around every read-modify-write of dQ.
// Here (FA2 order, no locks):
//   prep   : D = rowsum(dO∘O) and lse2 = m·log2e + log2(l) per query (fp32);
//   main   : one workgroup = 4 waves = 128 keys of one (batch, head) slice; each
//            wave owns 32 keys and keeps K, V (as MFMA B operands) and its dK, dV
//            accumulators in registers for the whole sweep over the query tiles
//            the rule allows (fa_rules.h q_range_for_k_block).  Per 32-query tile:
//              S  = Q'ᵀK   with C = -lse2  ->  P  = exp2(S)        (Q' = Q·scale·log2e)
//              dP = dOᵀV   with C = -D     ->  dS = P∘dP·scale
//              dV += dO·P,  dK += Q'·dS   (scores' accumulator tiles are the B operands)
//              dSᵀ -> LDS, then dQ[c][q] += Σ_key K[c][key]·dSᵀ[key][q] on MFMA and
//              fp32 atomics into a workspace (cdna_hip_programming.md App. B 'Attention backward');
//   cast   : dQ workspace -> fp16.
// All MFMAs are v_mfma_f32_32x32x16_f16 (fp32 accumulation).
#include "fa_device.h"
#include "fa_kernels.h"

#include <stdlib.h>

namespace fa {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((__vector_size__(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16_t;
typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2_t;
typedef __attribute__((address_space(3))) floatx4 lds_f4_t;
typedef __attribute__((address_space(3))) float lds_f_t;

constexpr int kThreads = 256;
constexpr int kBK = 128;  // keys per workgroup (4 waves x 32)
constexpr int kBQ = 32;   // queries per tile
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ half4 tr_read(const lds_char_t* base, uint32_t off) {
  const v4i16 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(base + off));
  return __builtin_bit_cast(half4, t);
}
__device__ __forceinline__ half4 read_b64(const lds_char_t* base, uint32_t off) {
  return *reinterpret_cast<const __attribute__((address_space(3))) half4*>(base + off);
}

// [rows][32] fp16 image, 64-B rows; 8-byte chunk c of row r stored at chunk c ^ ((r>>2)&7):
// conflict-free for 32-lane ds_read_b64 down a column and for ds_read_b64_tr_b16 blocks.
__device__ __forceinline__ uint32_t qimg(int row, int col) {  // col multiple of 4
  return row * 64 + ((((col >> 2) ^ (row >> 2)) & 7) << 3);
}
// [rows][128] fp16 image (K tile), 256-B rows; 16-byte chunk c stored at chunk c ^ (r & 15)
__device__ __forceinline__ uint32_t kimg(int row, int col) {  // col multiple of 4
  return row * 256 + ((((col >> 3) ^ row) & 15) << 4) + ((col & 4) << 1);
}

__device__ __forceinline__ u32x4 ld16(const __half* p) { return *reinterpret_cast<const u32x4*>(p); }

// 8 halfs at row[e..e+7], zero past n (vector path when the whole chunk is in range)
__device__ __forceinline__ u32x4 load_chunk8(const __half* row, int e, int n, bool vec) {
  if (vec && e + 8 <= n) return ld16(row + e);
  unsigned short h[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (e + j < n) ? __half_as_ushort(row[e + j]) : (unsigned short)0;
  return u32x4{h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16), h[4] | (uint32_t(h[5]) << 16),
               h[6] | (uint32_t(h[7]) << 16)};
}

__device__ __forceinline__ u32x4 scale_chunk(u32x4 v, float s) {
  half8 x = __builtin_bit_cast(half8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (_Float16)((float)x[j] * s);
  return __builtin_bit_cast(u32x4, x);
}

template <int D>
struct BSmem {
  static constexpr int kK = D * 256;    // K tile image [D][128]
  static constexpr int kQ = D * 64;     // Q' tile image [D][32]
  static constexpr int kO = D * 64;     // dO tile image [D][32]
  static constexpr int kS = kBK * 64;   // dSᵀ image [128][32]
  static constexpr int offQ = kK, offO = offQ + kQ, offS = offO + kO, offR = offS + kS;
  static constexpr int kTotal = offR + 2 * kBQ * 4;  // + lse2[32], D[32]
};

// ---------------------------------------------------------------------------
// prep: D = rowsum(dO∘O) (fp32), lse2 = m*log2e + log2(l) (+inf if the row attends nothing)
__global__ __launch_bounds__(kThreads) void bwd_f16_prep_kernel(BwdArgs a) {
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t total = a.b * (int64_t)nq;
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= total) return;
  const int64_t bi = i / nq;
  const int q = i % nq;
  const __half* O = static_cast<const __half*>(a.O) + bi * (int64_t)vd * nq + q;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq + q;
  float D = 0.f;
  for (int v = 0; v < vd; ++v) D += __half2float(O[(int64_t)v * nq]) * __half2float(dO[(int64_t)v * nq]);
  const float l = static_cast<const float*>(a.l)[i];
  const float m = __half2float(static_cast<const __half*>(a.m)[i]);
  static_cast<float*>(a.ws_D)[i] = D;
  static_cast<float*>(a.ws_lse)[i] = (l > 0.f) ? m * kLog2e + __log2f(l) : __builtin_huge_valf();
}

__global__ __launch_bounds__(kThreads) void bwd_f16_cast_kernel(const float* src, __half* dst, int64_t n) {
  const int64_t i = (blockIdx.x * (int64_t)kThreads + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(src + i);
    dst[i] = __float2half(v[0]); dst[i + 1] = __float2half(v[1]);
    dst[i + 2] = __float2half(v[2]); dst[i + 3] = __float2half(v[3]);
  } else {
    for (int64_t j = i; j < n; ++j) dst[j] = __float2half(src[j]);
  }
}

// ---------------------------------------------------------------------------
template <int D, int POL>
__global__ __launch_bounds__(kThreads, (D >= 128 ? 1 : 2)) void bwd_f16_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = BSmem<D>;

  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;  // earliest (heaviest under causal) key blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const float c2 = (float)a.scale * kLog2e;

  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  float* dQacc = static_cast<float*>(a.ws_dQ) + bi * (int64_t)d * nq;
  const bool kvec = ((nk & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.dO) & 15) == 0);

  lds_char_t* Kt = smem;
  lds_char_t* Qs = smem + S::offQ;
  lds_char_t* Os = smem + S::offO;
  lds_char_t* St = smem + S::offS;
  lds_f_t* lse_s = (lds_f_t*)(smem + S::offR);
  lds_f_t* D_s = lse_s + kBQ;

  // ---- B-operand fragments of this wave's 32 keys: lane (r,h) holds X[c = 16s + 8h + j][key = 32w + r]
  auto stage_kv_tile = [&](const __half* X, int nrows) {
    for (int idx = tid; idx < D * 16; idx += kThreads) {  // [D][128]: 16 chunks of 8 keys per row
      const int c = idx >> 4, m = idx & 15;
      const u32x4 v = (c < nrows) ? load_chunk8(X + (int64_t)c * nk, k0 + 8 * m, nk, kvec) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<lds_u32x4_t*>(Kt + kimg(c, 8 * m)) = v;
    }
  };
  auto read_b_frags = [&](half8 (&f)[D / 16]) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const half4 x = tr_read(Kt, kimg(16 * s + 8 * (g >> 1) + 4 * e + tq, 32 * w + 16 * (g & 1) + 4 * tp));
        if (e == 0) f[s].lo = x; else f[s].hi = x;
      }
  };
  half8 vfr[D / 16], kfr[D / 16];
  stage_kv_tile(V, vd);
  __syncthreads();
  read_b_frags(vfr);
  __syncthreads();
  stage_kv_tile(K, d);  // K stays resident: the A operand of the dQ product
  __syncthreads();
  read_b_frags(kfr);

  floatx16 dv[D / 32], dk[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dv[u][i] = 0.f; dk[u][i] = 0.f; }

  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / kBQ) * kBQ;
  const int key = k0 + 32 * w + r;
  const bool kvalid = key < nk;
  const int ko = (POL != 0 && kvalid) ? seq_order(a.rule.k, a.rule, key) : 0;
  const int wk0 = k0 + 32 * w, wk1 = min(wk0 + 31, nk - 1);
  const bool wave_keys = wk0 < nk;

  for (int q0 = qt0; q0 < qe; q0 += kBQ) {
    __syncthreads();  // previous tile's readers are done
    // ---- stage Q' = Q·c2, dO ([D][32] images), lse2, D
    for (int idx = tid; idx < 2 * D * 4; idx += kThreads) {
      const int which = idx >= D * 4, j = which ? idx - D * 4 : idx;
      const int c = j >> 2, m = j & 3;
      lds_char_t* img = which ? Os : Qs;
      u32x4 v = {0, 0, 0, 0};
      if (c < (which ? vd : d)) {
        v = load_chunk8((which ? dO : Q) + (int64_t)c * nq, q0 + 8 * m, nq, qvec);
        if (!which) v = scale_chunk(v, c2);
      }
      *reinterpret_cast<lds_u32x2_t*>(img + qimg(c, 8 * m)) = v.xy;
      *reinterpret_cast<lds_u32x2_t*>(img + qimg(c, 8 * m + 4)) = v.zw;
    }
    if (tid < kBQ) {
      const int q = q0 + tid;
      lse_s[tid] = (q < nq) ? glse[q] : __builtin_huge_valf();
      D_s[tid] = (q < nq) ? gD[q] : 0.f;
    }
    __syncthreads();

    int cls = 0;
    if (wave_keys) cls = (POL != 0) ? tile_class(a.rule, q0, min(q0 + kBQ, nq) - 1, wk0, wk1) : 2;
    if (cls != 0) {
      // row constants as the initial accumulators: C_S = -lse2[q], C_dP = -D[q], q = (i&3) + 8(i>>2) + 4h
      floatx16 sacc, pacc;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const floatx4 l4 = *reinterpret_cast<const lds_f4_t*>(lse_s + 8 * gq + 4 * h);
        const floatx4 d4 = *reinterpret_cast<const lds_f4_t*>(D_s + 8 * gq + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sacc[4 * gq + j] = -l4[j];
          pacc[4 * gq + j] = -d4[j];
        }
      }
      // S = Q'ᵀK - lse2, dP = dOᵀV - D; A operands (Xᵀ: row q, k = channel) by transposed reads
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        half8 qa, oa;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t off = qimg(16 * s + 8 * (g >> 1) + 4 * e + tq, 16 * (g & 1) + 4 * tp);
          const half4 x = tr_read(Qs, off);
          const half4 y = tr_read(Os, off);
          if (e == 0) { qa.lo = x; oa.lo = y; } else { qa.hi = x; oa.hi = y; }
        }
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa, kfr[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa, vfr[s], pacc, 0, 0, 0);
      }
      // P = exp2(S) (masked -> 0), dS = P * dP' * scale; rows q in registers, key on the lane
      const float sc = (float)a.scale;
      half8 pf[2], sf[2];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = __builtin_amdgcn_exp2f(sacc[i]);
        if (cls == 1 || !kvalid) {
          const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          bool ok = kvalid;
          if (POL != 0) ok &= (q >= nq) | check_orders_bf(a.rule, q < nq ? seq_order(a.rule.q, a.rule, q) : 0, ko);
          p = ok ? p : 0.f;
        }
        pf[i >> 3][i & 7] = (_Float16)p;
        sf[i >> 3][i & 7] = (_Float16)(p * pacc[i] * sc);
      }
      // dV += dO·P, dK += Q'·dS: A = X[row v/c][k = q], element j <- q = 16s + 8(j>>2) + 4h + (j&3)
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          half8 oa, qa;
          oa.lo = read_b64(Os, qimg(32 * u + r, 16 * s + 4 * h));
          oa.hi = read_b64(Os, qimg(32 * u + r, 16 * s + 8 + 4 * h));
          qa.lo = read_b64(Qs, qimg(32 * u + r, 16 * s + 4 * h));
          qa.hi = read_b64(Qs, qimg(32 * u + r, 16 * s + 8 + 4 * h));
          dv[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa, pf[s], dv[u], 0, 0, 0);
          dk[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa, sf[s], dk[u], 0, 0, 0);
        }
      // dSᵀ[key][q] -> LDS: registers 4gq..4gq+3 are q = 8gq + 4h + 0..3
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        half4 x;
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = sf[gq >> 1][4 * (gq & 1) + j];
        *reinterpret_cast<__attribute__((address_space(3))) half4*>(St + qimg(32 * w + r, 8 * gq + 4 * h)) = x;
      }
    } else {
      // this wave's keys take no part in the tile: its dSᵀ rows are zero
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const half4 z = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
        *reinterpret_cast<__attribute__((address_space(3))) half4*>(St + qimg(32 * w + r, 8 * gq + 4 * h)) = z;
      }
    }
    __syncthreads();
    // ---- dQ[c][q] += Σ_key K[c][key] dSᵀ[key][q]: wave w owns channel rows 32w..32w+31
    if (32 * w < D && 32 * w < d) {
      floatx16 qacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) qacc[i] = 0.f;
#pragma unroll
      for (int s = 0; s < kBK / 16; ++s) {
        const half8 ka = __builtin_bit_cast(half8,
                                            *reinterpret_cast<const lds_u32x4_t*>(Kt + kimg(32 * w + r, 16 * s + 8 * h)));
        half8 sb;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const half4 x = tr_read(St, qimg(16 * s + 8 * (g >> 1) + 4 * e + tq, 16 * (g & 1) + 4 * tp));
          if (e == 0) sb.lo = x; else sb.hi = x;
        }
        qacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka, sb, qacc, 0, 0, 0);
      }
      const int q = q0 + r;
      if (q < nq) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int c = 32 * w + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (c < d) atomicAdd(dQacc + (int64_t)c * nq + q, qacc[i]);
        }
      }
    }
  }

  // ---- dK = (Σ Q'·dS)/c2, dV: rows c/v = 32u + (i&3) + 8(i>>2) + 4h, column key
  if (!kvalid) return;
  __half* dK = static_cast<__half*>(a.dK) + bi * (int64_t)d * nk;
  __half* dV = static_cast<__half*>(a.dV) + bi * (int64_t)vd * nk;
  const float inv_c2 = 1.f / c2;
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dK[(int64_t)c * nk + key] = __float2half(dk[u][i] * inv_c2);
      if (c < vd) dV[(int64_t)c * nk + key] = __float2half(dv[u][i]);
    }
}

template <int D>
hipError_t launch_main(const BwdArgs& a, hipStream_t s) {
  const int64_t nkb = (a.rule.k.n + kBK - 1) / kBK;
  const int smem = BSmem<D>::kTotal;
  auto kern = a.rule.policy == 0 ? bwd_f16_kernel<D, 0> : bwd_f16_kernel<D, 1>;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(kThreads), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool bwd_f16_supported(const BwdArgs& a) {
  if (max(a.d, a.v_d) > 128) return bwd_f16_fast_supported(a);  // the 256-channel two-pass kernels
  return a.d >= 1 && a.v_d >= 1 && a.d <= 128 && a.v_d <= 128 &&
         a.b * ((a.rule.k.n + kBK - 1) / kBK) < (1ll << 31);
}

hipError_t launch_bwd_f16(const BwdArgs& a, hipStream_t s) {
  // the two-pass kernels take the shapes they support (diagnostic library: FA_BWD_VARIANT=0 pins
  // this single-pass atomic kernel for A/B runs; it holds at most 128 channels, so shapes past
  // that always go to the two-pass kernels)
  const int dm = max(a.d, a.v_d);
#ifdef FA_DIAG
  const bool pinned = diag_variant("FA_BWD_VARIANT") == 0 && dm <= 128;
#else
  constexpr bool pinned = false;
#endif
  if (!pinned && bwd_f16_fast_supported(a)) return launch_bwd_f16_fast(a, s);
  if (dm > 128) return hipErrorInvalidValue;
  const int nq = a.rule.q.n;
  hipError_t e = hipMemsetAsync(a.ws_dQ, 0, sizeof(float) * (size_t)a.b * a.d * nq, s);
  if (e != hipSuccess) return e;
  const int64_t nrows = a.b * (int64_t)nq;
  hipLaunchKernelGGL(bwd_f16_prep_kernel, dim3((unsigned)((nrows + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                     a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = dm <= 32 ? launch_main<32>(a, s) : (dm <= 64 ? launch_main<64>(a, s) : launch_main<128>(a, s));
  if (e != hipSuccess) return e;
  const int64_t n = a.b * (int64_t)a.d * nq;
  hipLaunchKernelGGL(bwd_f16_cast_kernel, dim3((unsigned)((n / 4 + kThreads) / kThreads)), dim3(kThreads), 0, s,
                     static_cast<const float*>(a.ws_dQ), static_cast<__half*>(a.dQ), n);
  return hipGetLastError();
}

}  // namespace fa
