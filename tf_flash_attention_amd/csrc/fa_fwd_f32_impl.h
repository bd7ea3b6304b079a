// fa_fwd_f32_impl.h — the fp32 MFMA forward kernel template and its launcher, shared by
// fa_fwd_f32.hip (D <= 128) and fa_fwd_f32_wide.hip (D = 256, built with VGPR-form MFMAs).
//
// fp32 fused attention forward on gfx950 MFMA (v_mfma_f32_32x32x2_f32).
//
// gfx950 has no reduced-precision (xf32) path: the f32-input MFMA is a k-ordered
// fmaf chain at the f32 vector rate (157 TF/s), so this kernel keeps full fp32
// numerics (the rtol 1e-5 parity target) while taking the arithmetic off the
// VALU.  Same structure as the fp16 kernel (fa_fwd_f16.hip): transposed scores
// Sᵀ = Kᵀ·Q (key on the MFMA rows, one query per lane), online softmax in
// registers, and Oᵀ = V·Pᵀ where the Sᵀ accumulator registers ARE the B
// operand of the 32x32x2 PV steps (register j of a tile is key
// (j&3) + 8(j>>2) + 4h: pairing lane halves h = 0/1 gives the k-step), so P
// never leaves registers.  V is staged transposed ([key][v]) so its A operand
// is a conflict-free 32-lane row read.
#pragma once
#include "fa_device.h"
#include "fa_kernels.h"

namespace fa {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) float lds_f_t;

constexpr int kThreads = 256;
constexpr int kBM = 128;   // query rows per workgroup (4 waves x 32)
constexpr int kBN = 64;    // keys per tile (32 at D = 256: two 64-key tiles of 256 channels would not fit LDS)
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.f;

__device__ __forceinline__ float xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

template <int D, int BN>
struct Smem32 {
  static constexpr int kVP = D + 1;               // V [BN keys][D+1] (transposed, padded)
  static constexpr int kK = D * BN;               // K [D][BN]
  static constexpr int kV = BN * kVP;
  static constexpr int kBuf = kK + kV;            // floats
  static constexpr int kQ = D * kBM;              // Q [D][128] (aliases the buffers)
  static constexpr int kTotal = 4 * ((2 * kBuf > kQ) ? 2 * kBuf : kQ);  // bytes
};

template <int D, int POL, int BN = kBN>
__global__ __launch_bounds__(kThreads, D >= 128 ? 1 : 2) void fwd_f32_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_f_t* smem = (lds_f_t*)smem_raw;
  using S = Smem32<D, BN>;
  constexpr int kT = BN / 32;  // 32-key MFMA row blocks per tile
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const float c2 = (float)a.scale * kLog2e;

  const float* Q = static_cast<const float*>(a.Q) + bi * (int64_t)d * nq;
  const float* K = static_cast<const float*>(a.K) + bi * (int64_t)d * nk;
  const float* V = static_cast<const float*>(a.V) + bi * (int64_t)vd * nk;

  // ---- Q tile -> LDS [D][128]; B-operand fragments (pre-scaled by scale*log2e):
  //      qf[s] = Q[c = 2s + h][q = 32w + r]
  for (int idx = tid; idx < D * kBM; idx += kThreads) {
    const int c = idx / kBM, qq = idx % kBM;
    smem[idx] = (c < d && q0 + qq < nq) ? Q[(int64_t)c * nq + q0 + qq] : 0.f;
  }
  __syncthreads();
  float qf[D / 2];
#pragma unroll
  for (int s = 0; s < D / 2; ++s) qf[s] = smem[(2 * s + h) * kBM + 32 * w + r] * c2;
  __syncthreads();

  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / BN) * BN;
  const int ntiles = (ke > kb) ? (ke - kt0 + BN - 1) / BN : 0;
  const int wq0 = q0 + 32 * w;
  const int wq1 = min(wq0 + 31, nq - 1);
  const bool wave_active = wq0 < nq;
  const int qi = wq0 + r;
  const int qo = (POL == 2 && qi < nq) ? seq_order(a.rule.q, a.rule, qi) : 0;
  // POL 1 (interval rules, see fa_fwd_f16.hip): lane key interval + wave bounds
  int klo = 0, kspan = 0, wlo_min = 0, wlo_max = 0, whi_min = 0, whi_max = 0;
  if (POL == 1 && wave_active) {
    int khi;
    key_interval(a.rule, min(qi, nq - 1), &klo, &khi);
    kspan = max(khi - klo + 1, 0);
    const int last = min(31, nq - 1 - wq0);
    wlo_min = __builtin_amdgcn_readfirstlane(klo);
    whi_min = __builtin_amdgcn_readfirstlane(khi);
    wlo_max = __builtin_amdgcn_readlane(klo, last);
    whi_max = __builtin_amdgcn_readlane(khi, last);
  }
  const bool kvec = ((nk & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);

  // ---- staging: K [D][BN] as stored; V transposed to [BN][D+1]
  constexpr int kChunks = D * (BN / 4);              // 4-float chunks per tensor tile
  constexpr int kCPT = (kChunks + kThreads - 1) / kThreads;
  floatx4 kreg[kCPT], vreg[kCPT];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = tid + kThreads * j, c = idx / (BN / 4), m = idx % (BN / 4), e = k0 + 4 * m;
      floatx4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (idx < kChunks) {
        if (kvec && e + 4 <= nk) {
          if (c < d) kv = *reinterpret_cast<const floatx4*>(K + (int64_t)c * nk + e);
          if (c < vd) vv = *reinterpret_cast<const floatx4*>(V + (int64_t)c * nk + e);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (c < d && e + i < nk) kv[i] = K[(int64_t)c * nk + e + i];
            if (c < vd && e + i < nk) vv[i] = V[(int64_t)c * nk + e + i];
          }
        }
      }
      kreg[j] = kv;
      vreg[j] = vv;
    }
  };
  auto store_tile = [&](int buf) {
    lds_f_t* kb_ = smem + buf * S::kBuf;
    lds_f_t* vb_ = kb_ + S::kK;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = tid + kThreads * j, c = idx / (BN / 4), m = idx % (BN / 4);
      if (idx < kChunks) {
        *reinterpret_cast<__attribute__((address_space(3))) floatx4*>(kb_ + c * BN + 4 * m) = kreg[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) vb_[(4 * m + i) * S::kVP + c] = vreg[j][i];
      }
    }
  };

  floatx16 acc_o[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_o[u][i] = 0.f;
  float m_run = 0.f, l_run = 0.f, m_max = kNegInf;
  bool m_set = false;
  floatx16 negm;
#pragma unroll
  for (int i = 0; i < 16; ++i) negm[i] = 0.f;

  if (ntiles > 0) load_tile(kt0);
  for (int it = 0; it < ntiles; ++it) {
    const int k0 = kt0 + it * BN;
    store_tile(it & 1);
    if (it + 1 < ntiles) load_tile(k0 + BN);
    __syncthreads();

    const int k1 = k0 + BN - 1;
    int cls;
    if (!wave_active) cls = 0;
    else if (POL == 0) cls = k1 < nk ? 2 : 1;
    else if (POL == 1) cls = (wlo_min > k1 || whi_max < k0) ? 0 : ((wlo_max <= k0 && whi_min >= k1) ? 2 : 1);
    else {
      cls = tile_class(a.rule, wq0, wq1, k0, min(k1, nk - 1));
      if (cls == 2 && k1 >= nk) cls = 1;
    }
    if (cls == 0) continue;
    const lds_f_t* kbuf = smem + (it & 1) * S::kBuf;
    const lds_f_t* vbuf = kbuf + S::kK;

    // Sᵀ - m: A = Kᵀ (lane: key 32t + r, channel 2s + h), B = Q' fragments
    floatx16 st[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      st[t] = negm;
#pragma unroll
      for (int s = 0; s < D / 2; ++s)
        st[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kbuf[(2 * s + h) * BN + 32 * t + r], qf[s], st[t], 0, 0, 0);
    }
    if (cls == 1) {
      const int base = k0 + 4 * h - klo;
#pragma unroll
      for (int t = 0; t < kT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = 32 * t + (i & 3) + 8 * (i >> 2);
          bool ok;
          if (POL == 1) {
            ok = (unsigned)(base + off) < (unsigned)kspan;
          } else {
            const int key = k0 + off + 4 * h;
            ok = key < nk;
            if (POL == 2) ok &= check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, key));
          }
          st[t][i] = ok ? st[t][i] : kNegInf;
        }
    }
    float mt;
    {
      float mx[kT];  // one max chain per 32-key block
#pragma unroll
      for (int t = 0; t < kT; ++t) mx[t] = fmaxf(st[t][0], st[t][1]);
#pragma unroll
      for (int i = 2; i < 16; i += 2)
#pragma unroll
        for (int t = 0; t < kT; ++t) mx[t] = fmaxf(fmaxf(mx[t], st[t][i]), st[t][i + 1]);
      mt = mx[0];
#pragma unroll
      for (int t = 1; t < kT; ++t) mt = fmaxf(mt, mx[t]);
      mt = fmaxf(mt, xor32(mt));
    }
    m_max = fmaxf(m_max, m_run + mt);
    const bool seed = !m_set && (mt != kNegInf);
    if (__any((mt > kRescaleThr) | seed)) {
      const float delta = m_set ? fmaxf(mt, 0.f) : (seed ? mt : 0.f);
      const float alpha = m_set ? __builtin_amdgcn_exp2f(-delta) : 1.f;
      m_run += delta;
      m_set = m_set || seed;
      l_run *= alpha;
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc_o[u][i] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
#pragma unroll
        for (int t = 0; t < kT; ++t) st[t][i] -= delta;
        negm[i] = -m_run;
      }
    }
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int t = 0; t < kT; ++t)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        st[t][i] = __builtin_amdgcn_exp2f(st[t][i]);
        st[t][i + 1] = __builtin_amdgcn_exp2f(st[t][i + 1]);
        ls0 += st[t][i];
        ls1 += st[t][i + 1];
      }
    l_run += ls0 + ls1;
    // Oᵀ[v][q] += Σ_key V[v][key] P[key][q]: k-step = register j of tile t (keys
    // 32t + (j&3) + 8(j>>2) + 4h for lane halves h), A = V[key][v = 32u + r] (transposed image)
#pragma unroll
    for (int t = 0; t < kT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int keyl = 32 * t + (j & 3) + 8 * (j >> 2) + 4 * h;
#pragma unroll
        for (int u = 0; u < D / 32; ++u)
          acc_o[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(vbuf[keyl * S::kVP + 32 * u + r], st[t][j], acc_o[u], 0,
                                                          0, 0);
      }
  }

  if (!wave_active) return;
  const float l_tot = l_run + xor32(l_run);
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi < nq) {
    float* O = static_cast<float*>(a.O) + bi * (int64_t)vd * nq;
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (v < vd) O[(int64_t)v * nq + qi] = acc_o[u][i] * inv;
      }
    if (h == 0) {
      float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
      float* mo = static_cast<float*>(a.m) + bi * (int64_t)nq;
      if (l_tot > 0.f) {
        const float mT = m_max * kLn2;
        lo[qi] = l_tot * __builtin_amdgcn_exp2f(m_run - m_max);
        mo[qi] = mT;
      } else {
        lo[qi] = 0.f;
        mo[qi] = neg_inf_approx<float>();
      }
    }
  }
}

template <int D, int BN = kBN>
hipError_t launch_t(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const int smem = Smem32<D, BN>::kTotal;
  static_assert(Smem32<D, BN>::kTotal <= 160 * 1024, "LDS");
  const int pol = a.rule.policy == 0 ? 0 : (rule_is_interval(a.rule) ? 1 : 2);
  auto kern = pol == 0 ? fwd_f32_kernel<D, 0, BN> : (pol == 1 ? fwd_f32_kernel<D, 1, BN> : fwd_f32_kernel<D, 2, BN>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kThreads), smem, s, a);
  return hipGetLastError();
}

}  // namespace
}  // namespace fa
