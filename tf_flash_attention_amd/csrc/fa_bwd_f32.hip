// fa_bwd_f32.hip — fp32 fused attention backward on gfx950 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's BackwardImpl (flash_attention.cu:1079-1967) for fp32
// inputs (any d, v_d <= 128, every policy / sync mode / rule; up to 256 in fa_bwd_f32_wide.hip).  The f32-input MFMA
// is a k-ordered fmaf chain at the f32 vector rate, so numerics stay full fp32
// (the 1e-5 parity target) while the five GEMMs of the backward leave the VALU.
// Same two-pass split as the fp16 backward (fa_bwd_f16_fast.hip), no atomics:
//   prep : D = rowsum(dO∘O), lse2 = m·log2e + log2 l
//   dkdv : key-outer; lane = key; K·scale·log2e and V resident as B operands
//            S  = Qᵀ·K' (C = -lse2)  P = exp2(S)     dP = dOᵀ·V (C = -D)   dS = P∘dP
//            dV += dO·P,  dK += Q·dS      (k-step = accumulator register j: P / dS
//                                           straight from registers)
//   dq   : query-outer; lane = query; Q·scale·log2e and dO resident
//            Sᵀ = Kᵀ·Q' (C = -lse2)  dPᵀ = Vᵀ·dO (C = -D)  dQ += K·(Pᵀ∘dPᵀ)
// Channels are zero-padded to D = 32·⌈max(d, v_d)/32⌉; masks are rules (fa_rules.h).
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kThrPrep = 256;
constexpr int kThr = 256;  // 4 waves x 32 keys / queries
constexpr int kT = 32;     // queries (dkdv) / keys (dq) per streamed tile

__global__ __launch_bounds__(kThrPrep) void bwd_prep_f32_kernel(BwdArgs a) {
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t total = a.b * (int64_t)nq;
  const int64_t i = blockIdx.x * (int64_t)kThrPrep + threadIdx.x;
  if (i >= total) return;
  const int64_t bi = i / nq;
  const int q = (int)(i - bi * nq);
  const float* O = static_cast<const float*>(a.O) + bi * (int64_t)vd * nq + q;
  const float* dO = static_cast<const float*>(a.dO) + bi * (int64_t)vd * nq + q;
  float D0 = 0.f, D1 = 0.f;
  int v = 0;
  for (; v + 1 < vd; v += 2) {
    D0 = fmaf(O[(int64_t)v * nq], dO[(int64_t)v * nq], D0);
    D1 = fmaf(O[(int64_t)(v + 1) * nq], dO[(int64_t)(v + 1) * nq], D1);
  }
  if (v < vd) D0 = fmaf(O[(int64_t)v * nq], dO[(int64_t)v * nq], D0);
  const float l = static_cast<const float*>(a.l)[i];
  const float m = static_cast<const float*>(a.m)[i];
  static_cast<float*>(a.ws_D)[i] = D0 + D1;
  static_cast<float*>(a.ws_lse)[i] = (l > 0.f) ? m * kLog2e + __log2f(l) : __builtin_huge_valf();
}

// one streamed tile of two [D][32] tensors: row images [D][32] and transposed images [32][D+1]
template <int D>
struct Tile32 {
  static constexpr int kRow = D * kT;               // floats
  static constexpr int kTr = kT * (D + 1);
  static constexpr int offA = 0, offB = kRow, offAT = 2 * kRow, offBT = 2 * kRow + kTr, offC = 2 * kRow + 2 * kTr;
  static constexpr int kSlot = offC + 2 * kT;      // + two 32-float row-constant vectors (dkdv: lse2, D)
  static constexpr int kChunks = 2 * D * (kT / 4);  // float4 chunks of the two tensors
  static constexpr int kCPT = (kChunks + kThr - 1) / kThr;
};

// float4 of row[e..e+3] (zeros past n)
__device__ __forceinline__ floatx4 load4(const float* row, int e, int n, bool vec) {
  if (vec && e + 4 <= n) return *reinterpret_cast<const floatx4*>(row + e);
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (e + i < n) v[i] = row[e + i];
  return v;
}

// Streams [d_a][n] tensor A and [d_b][n] tensor B in 32-column tiles through a 2-slot LDS ring
// (register staged one tile ahead).  Chunk idx: tensor = idx / (D*8), row c, columns 4m..4m+3.
template <int D, bool kBT = true>
struct Streamer {
  const float* A;
  const float* B;
  int da, db, n;
  bool vec;
  floatx4 reg[Tile32<D>::kCPT];
  __device__ void load(int col0) {
#pragma unroll
    for (int j = 0; j < Tile32<D>::kCPT; ++j) {
      const int idx = threadIdx.x + kThr * j;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx < Tile32<D>::kChunks) {
        const bool isB = idx >= D * (kT / 4);
        const int k = isB ? idx - D * (kT / 4) : idx, c = k >> 3, m = k & 7;
        if (c < (isB ? db : da)) v = load4((isB ? B : A) + (int64_t)c * n, col0 + 4 * m, n, vec);
      }
      reg[j] = v;
    }
  }
  __device__ void store(lds_f_t* slot) const {
#pragma unroll
    for (int j = 0; j < Tile32<D>::kCPT; ++j) {
      const int idx = threadIdx.x + kThr * j;
      if (idx < Tile32<D>::kChunks) {
        const bool isB = idx >= D * (kT / 4);
        const int k = isB ? idx - D * (kT / 4) : idx, c = k >> 3, m = k & 7;
        lds_f_t* row = slot + (isB ? Tile32<D>::offB : Tile32<D>::offA);
        lds_f_t* tr = slot + (isB ? Tile32<D>::offBT : Tile32<D>::offAT);
        *reinterpret_cast<lds_f4_t*>(row + c * kT + 4 * m) = reg[j];
        if (!isB || kBT) {
#pragma unroll
          for (int i = 0; i < 4; ++i) tr[(4 * m + i) * (D + 1) + c] = reg[j][i];
        }
      }
    }
  }
};

template <int D>
constexpr int dkdv32_smem() {
  return 4 * ((2 * Tile32<D>::kSlot > 2 * D * 128) ? 2 * Tile32<D>::kSlot : 2 * D * 128);
}
template <int D>
constexpr int dq32_smem() {
  return 4 * ((2 * Tile32<D>::kSlot > 2 * D * 128) ? 2 * Tile32<D>::kSlot : 2 * D * 128);
}

// ---------------------------------------------------------------------------
// dK / dV: 4 waves x 32 keys per workgroup; query tiles of 32 stream through LDS.
//   POL 0 full, 1 interval rules, 2 any other rule (per-element order check)
template <int D, int POL>
__global__ __launch_bounds__(kThr, D >= 128 ? 1 : 2) void bwd_dkdv_f32_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_f_t* smem = (lds_f_t*)smem_raw;
  using T = Tile32<D>;
  constexpr int kBK = 128;
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const float c2 = (float)a.scale * kLog2e;
  const float* K = static_cast<const float*>(a.K) + bi * (int64_t)d * nk;
  const float* V = static_cast<const float*>(a.V) + bi * (int64_t)vd * nk;
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
  const bool kvec = ((nk & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);
  const bool qvec = ((nq & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.dO) & 15) == 0);

  // ---- resident B operands: lane (r,h) holds X[c = 2s + h][key = k0 + 32w + r]
  float kb[D / 2], vb[D / 2];
  for (int idx = tid; idx < 2 * D * (kBK / 4); idx += kThr) {
    const bool isV = idx >= D * (kBK / 4);
    const int k = isV ? idx - D * (kBK / 4) : idx, c = k / (kBK / 4), m = k % (kBK / 4);
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (c < (isV ? vd : d)) v = load4((isV ? V : K) + (int64_t)c * nk, k0 + 4 * m, nk, kvec);
    *reinterpret_cast<lds_f4_t*>(smem + (isV ? D * kBK : 0) + c * kBK + 4 * m) = v;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < D / 2; ++s) {
    kb[s] = smem[(2 * s + h) * kBK + 32 * w + r] * c2;
    vb[s] = smem[D * kBK + (2 * s + h) * kBK + 32 * w + r];
  }
  __syncthreads();

  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / kT) * kT;
  const int ntiles = (qe > qb) ? (qe - qt0 + kT - 1) / kT : 0;
  const int key = k0 + 32 * w + r;
  const int wk0 = k0 + 32 * w, wk1 = min(wk0 + 31, nk - 1);
  const bool wave_active = wk0 < nk;
  const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;
  int qlo = 0, qspan = nq;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
  }

  Streamer<D> st{static_cast<const float*>(a.Q) + bi * (int64_t)d * nq,
                 static_cast<const float*>(a.dO) + bi * (int64_t)vd * nq, d, vd, nq, qvec, {}};
  float lr = 0.f;
  auto load_tile = [&](int qa) {
    st.load(qa);
    if (tid < 64) {
      const int q = qa + (tid & 31);
      lr = (q < nq) ? ((tid < 32) ? glse[q] : gD[q]) : ((tid < 32) ? __builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot) {
    lds_f_t* base = smem + slot * T::kSlot;
    st.store(base);
    if (tid < 64) base[T::offC + tid] = lr;
  };

  floatx16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dk[u][i] = 0.f; dv[u][i] = 0.f; }

  if (ntiles > 0) { load_tile(qt0); store_tile(0); }
  if (ntiles > 1) load_tile(qt0 + kT);
  for (int it = 0; it < ntiles; ++it) {
    __syncthreads();
    const int qa = qt0 + it * kT;
    if (it + 1 < ntiles) store_tile((it + 1) & 1);
    if (it + 2 < ntiles) load_tile(qa + 2 * kT);
    int cls = 2;
    if (!wave_active) cls = 0;
    else if (POL != 0) cls = tile_class(a.rule, qa, min(qa + kT, nq) - 1, wk0, wk1);
    if (cls == 0) continue;
    const lds_f_t* base = smem + (it & 1) * T::kSlot;
    floatx16 sacc, pacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ql = (i & 3) + 8 * (i >> 2) + 4 * h;
      sacc[i] = -base[T::offC + ql];
      pacc[i] = -base[T::offC + kT + ql];
    }
#pragma unroll
    for (int s = 0; s < D / 2; ++s) {
      sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offA + (2 * s + h) * kT + r], kb[s], sacc, 0, 0, 0);
      pacc = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offB + (2 * s + h) * kT + r], vb[s], pacc, 0, 0, 0);
    }
    float p[16], ds[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (POL != 0 && cls == 1) {
        const int q = qa + (i & 3) + 8 * (i >> 2) + 4 * h;
        bool ok;
        if (POL == 1) ok = (unsigned)(q - qlo) < (unsigned)qspan;
        else ok = (q < nq) && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko);
        pv = ok ? pv : 0.f;
      }
      p[i] = pv;
      ds[i] = pv * pacc[i];
    }
    // dV += dO·P, dK += Q·dS: k-step j = queries (j&3) + 8(j>>2) + 4h (transposed images)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int ql = (j & 3) + 8 * (j >> 2) + 4 * h;
#pragma unroll
      for (int u = 0; u < D / 32; ++u) {
        dv[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offBT + ql * (D + 1) + 32 * u + r], p[j], dv[u], 0, 0, 0);
        dk[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offAT + ql * (D + 1) + 32 * u + r], ds[j], dk[u], 0, 0, 0);
      }
    }
  }

  if (!wave_active || key >= nk) return;
  float* dK = static_cast<float*>(a.dK) + bi * (int64_t)d * nk;
  float* dV = static_cast<float*>(a.dV) + bi * (int64_t)vd * nk;
  const float sc = (float)a.scale;
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dK[(int64_t)c * nk + key] = dk[u][i] * sc;
      if (c < vd) dV[(int64_t)c * nk + key] = dv[u][i];
    }
}

// ---------------------------------------------------------------------------
// dQ: 4 waves x 32 queries per workgroup; key tiles of 32 stream through LDS.
template <int D, int POL>
__global__ __launch_bounds__(kThr, D >= 128 ? 1 : 2) void bwd_dq_f32_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_f_t* smem = (lds_f_t*)smem_raw;
  using T = Tile32<D>;
  constexpr int kBM = 128;
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
  const float* dO = static_cast<const float*>(a.dO) + bi * (int64_t)vd * nq;
  const bool qvec = ((nq & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.dO) & 15) == 0);
  const bool kvec = ((nk & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);

  // ---- resident B operands: lane (r,h) holds X[c = 2s + h][q = q0 + 32w + r]
  float qf[D / 2], of[D / 2];
  for (int idx = tid; idx < 2 * D * (kBM / 4); idx += kThr) {
    const bool isO = idx >= D * (kBM / 4);
    const int k = isO ? idx - D * (kBM / 4) : idx, c = k / (kBM / 4), m = k % (kBM / 4);
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (c < (isO ? vd : d)) v = load4((isO ? dO : Q) + (int64_t)c * nq, q0 + 4 * m, nq, qvec);
    *reinterpret_cast<lds_f4_t*>(smem + (isO ? D * kBM : 0) + c * kBM + 4 * m) = v;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < D / 2; ++s) {
    qf[s] = smem[(2 * s + h) * kBM + 32 * w + r] * c2;
    of[s] = smem[D * kBM + (2 * s + h) * kBM + 32 * w + r];
  }
  __syncthreads();

  const int wq0 = q0 + 32 * w, wq1 = min(wq0 + 31, nq - 1);
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;
  floatx16 negl, negd;
  {
    const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
    const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
    const float lv = (qi < nq) ? -glse[qi] : kNegInf, dv = (qi < nq) ? -gD[qi] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) { negl[i] = lv; negd[i] = dv; }
  }
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kT) * kT;
  const int ntiles = (ke > kb) ? (ke - kt0 + kT - 1) / kT : 0;
  const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;
  int klo = 0, kspan = nk;
  if (POL == 1 && wave_active) {
    int khi;
    key_interval(a.rule, min(qi, nq - 1), &klo, &khi);
    kspan = max(khi - klo + 1, 0);
  }

  // K and V tiles: K row image [D][32] (Sᵀ A operand) + K transposed [32][D+1] (dQ A operand),
  // V row image [D][32] (dPᵀ A operand)
  Streamer<D, false> st{static_cast<const float*>(a.K) + bi * (int64_t)d * nk,
                 static_cast<const float*>(a.V) + bi * (int64_t)vd * nk, d, vd, nk, kvec, {}};

  floatx16 dq[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[u][i] = 0.f;

  if (ntiles > 0) { st.load(kt0); st.store(smem); }
  if (ntiles > 1) st.load(kt0 + kT);
  for (int it = 0; it < ntiles; ++it) {
    __syncthreads();
    const int ka = kt0 + it * kT;
    if (it + 1 < ntiles) st.store(smem + ((it + 1) & 1) * T::kSlot);
    if (it + 2 < ntiles) st.load(ka + 2 * kT);
    int cls;
    if (!wave_active) cls = 0;
    else if (POL == 0) cls = (ka + kT <= nk) ? 2 : 1;
    else {
      cls = tile_class(a.rule, wq0, wq1, ka, min(ka + kT, nk) - 1);
      if (cls == 2 && ka + kT > nk) cls = 1;
    }
    if (cls == 0) continue;
    const lds_f_t* base = smem + (it & 1) * T::kSlot;
    floatx16 sacc = negl, pacc = negd;
#pragma unroll
    for (int s = 0; s < D / 2; ++s) {
      sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offA + (2 * s + h) * kT + r], qf[s], sacc, 0, 0, 0);
      pacc = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offB + (2 * s + h) * kT + r], of[s], pacc, 0, 0, 0);
    }
    float ds[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (cls == 1) {
        const int kk = ka + (i & 3) + 8 * (i >> 2) + 4 * h;
        bool ok = kk < nk;
        if (POL == 1) ok &= (unsigned)(kk - klo) < (unsigned)kspan;
        if (POL == 2) ok &= check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1)));
        pv = ok ? pv : 0.f;
      }
      ds[i] = pv * pacc[i];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int kl = (j & 3) + 8 * (j >> 2) + 4 * h;
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
        dq[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(base[T::offAT + kl * (D + 1) + 32 * u + r], ds[j], dq[u], 0, 0, 0);
    }
  }

  if (!wave_active || qi >= nq) return;
  float* dQ = static_cast<float*>(a.dQ) + bi * (int64_t)d * nq;
  const float sc = (float)a.scale;
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dQ[(int64_t)c * nq + qi] = dq[u][i] * sc;
    }
}

template <int D>
hipError_t launch_t(const BwdArgs& a, hipStream_t s) {
  const int pol = a.rule.policy == 0 ? 0 : (rule_is_interval(a.rule) ? 1 : 2);
  auto kk = pol == 0 ? bwd_dkdv_f32_kernel<D, 0> : (pol == 1 ? bwd_dkdv_f32_kernel<D, 1> : bwd_dkdv_f32_kernel<D, 2>);
  auto kq = pol == 0 ? bwd_dq_f32_kernel<D, 0> : (pol == 1 ? bwd_dq_f32_kernel<D, 1> : bwd_dq_f32_kernel<D, 2>);
  constexpr int smk = dkdv32_smem<D>(), smq = dq32_smem<D>();
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kk), smk);
  if (e != hipSuccess) return e;
  e = set_smem_once(reinterpret_cast<const void*>(kq), smq);
  if (e != hipSuccess) return e;
  const int64_t nkb = (a.rule.k.n + 127) / 128, nqb = (a.rule.q.n + 127) / 128;
  hipLaunchKernelGGL(kk, dim3((unsigned)(a.b * nkb)), dim3(kThr), smk, s, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kq, dim3((unsigned)(a.b * nqb)), dim3(kThr), smq, s, a);
  return hipGetLastError();
}

}  // namespace

bool bwd_f32_supported(const BwdArgs& a) {
  // (128 < max(d, v_d) <= 256: fa_bwd_f32_wide.hip, 64-key / 64-query workgroups)
  return a.d >= 1 && a.v_d >= 1 && a.d <= 256 && a.v_d <= 256 &&
         a.b * ((a.rule.k.n + 63) / 64) < (1ll << 31) && a.b * ((a.rule.q.n + 63) / 64) < (1ll << 31);
}

hipError_t launch_bwd_f32(const BwdArgs& a, hipStream_t s) {
  const int64_t nrows = a.b * (int64_t)a.rule.q.n;
  hipLaunchKernelGGL(bwd_prep_f32_kernel, dim3((unsigned)((nrows + kThrPrep - 1) / kThrPrep)), dim3(kThrPrep), 0, s,
                     a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_t<32>(a, s);
  if (dm <= 64) return launch_t<64>(a, s);
  if (dm <= 128) return launch_t<128>(a, s);
  return launch_bwd_f32_wide(a, s);
}

}  // namespace fa
