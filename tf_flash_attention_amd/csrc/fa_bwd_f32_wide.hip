// fa_bwd_f32_wide.hip — fp32 fused attention backward for 128 < max(d, v_d) <= 256 on gfx950 MFMA
// (v_mfma_f32_16x16x4_f32).  The prep kernel (D, lse2) runs in fa_bwd_f32.hip; these are its two
// passes at D = 256 (channels zero-padded).
//
// fa_bwd_f32.hip's 32-row tiles hold K'·V (dK/dV pass) or Q'·dO (dQ pass) resident as B operands
// of 32x32x2 MFMAs: at 256 channels that is 256 registers a wave before any accumulator.  Here a
// wave owns 16 keys (16 queries): the 16x16x4 MFMA's B operand is one float per lane per 4-channel
// k-step, so the resident operands are 2 x 64 registers and the 256-channel accumulators of both
// gradients 2 x 64, with no output-channel chunking and no recomputed products.
//
// Register layout of v_mfma_f32_16x16x4_f32 (lane l, g = l >> 4, c = l & 15): A[row c][k g],
// B[k g][col c], D[row 4g + i][col c] in register i.  So register i of a 16 x 16 product is the B
// operand of k-step i of the next one (its k index g selects row 4g + i): P and dS feed the
// gradient MFMAs straight from the accumulators, their A operands read with the same row order.
//
//   dkdv : key-outer; D layout [query][key]:  S = Qᵀ·K' (C = -lse2)  P = exp2(S)  dP = dOᵀ·V (C = -D)
//          dS = P∘dP;  dV[c][key] += Σ_q dO[c][q] P[q][key],  dK[c][key] += Σ_q Q[c][q] dS[q][key]
//   dq   : query-outer; D layout [key][query]:  Sᵀ = Kᵀ·Q' (C = -lse2)  dPᵀ = Vᵀ·dO (C = -D)
//          dQ[c][q] += Σ_key K[c][key] dSᵀ[key][q]
// Streamed tiles (16 queries / keys of two tensors) sit in LDS as padded row images [256][17]: the
// S / dP A operands read one row per 16-lane group (consecutive columns), the gradient A operands
// one column per group (rows 17 floats apart, distinct banks), so one image serves both.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 256;
constexpr int kNW = 4;            // waves per workgroup
constexpr int kThr = kNW * 64;
constexpr int kT = 16;            // keys (queries) per wave; queries (keys) per streamed tile
constexpr int kBlk = kNW * kT;    // keys (queries) per workgroup
constexpr int kRP = kT + 1;       // padded image row, floats
constexpr int kImg = kD * kRP;    // one tensor's tile image, floats
constexpr int kSlot = 2 * kImg + 2 * kT;   // two images + two 16-float row-constant vectors (dK/dV)
constexpr int kNSlot = 2;
constexpr int kSmem = 4 * kNSlot * kSlot;  // bytes (69.9 KB)
constexpr int kChunks = 2 * kD * (kT / 4); // float4 chunks of one tile (two tensors)
constexpr int kCPT = kChunks / kThr;       // 8 a thread
static_assert(kChunks % kThr == 0, "staging");

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// float4 of row[e..e+3] (zeros past n)
__device__ __forceinline__ floatx4 ld4(const float* row, int e, int n, bool vec) {
  if (vec && e + 4 <= n) return *reinterpret_cast<const floatx4*>(row + e);
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (e + i < n) v[i] = row[e + i];
  return v;
}

// Streams the [da][n] tensor A and the [db][n] tensor B in 16-column tiles into padded LDS images
// (register staged one tile ahead).  Chunk idx: tensor idx / (D*4), row c, columns 4m..4m+3.
struct Stream16 {
  const float* A;
  const float* B;
  int da, db, n;
  bool vec;
  floatx4 reg[kCPT];
  __device__ void load(int col0) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = threadIdx.x + kThr * j;
      const bool isB = idx >= kD * (kT / 4);
      const int k = isB ? idx - kD * (kT / 4) : idx, c = k >> 2, m = k & 3;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (c < (isB ? db : da)) v = ld4((isB ? B : A) + (int64_t)c * n, col0 + 4 * m, n, vec);
      reg[j] = v;
    }
  }
  __device__ void store(lds_f_t* slot) const {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = threadIdx.x + kThr * j;
      const bool isB = idx >= kD * (kT / 4);
      const int k = isB ? idx - kD * (kT / 4) : idx, c = k >> 2, m = k & 3;
      lds_f_t* row = slot + (isB ? kImg : 0) + c * kRP + 4 * m;
#pragma unroll
      for (int i = 0; i < 4; ++i) row[i] = reg[j][i];
    }
  }
};

// ---------------------------------------------------------------------------
// dK / dV: 4 waves x 16 keys a workgroup; query tiles of 16 stream through LDS.
//   POL 0 full, 1 interval rules, 2 any other rule (per-element order check)
template <int POL>
__global__ __launch_bounds__(kThr, 1) void bwd_dkdv_f32w_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_f_t* smem = (lds_f_t*)smem_raw;
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nkb = (nk + kBlk - 1) / kBlk;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBlk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const float c2 = (float)a.scale * kLog2e;
  const float* K = static_cast<const float*>(a.K) + bi * (int64_t)d * nk;
  const float* V = static_cast<const float*>(a.V) + bi * (int64_t)vd * nk;
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
  const bool qvec = ((nq & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.dO) & 15) == 0);

  // ---- resident B operands: lane (g, c16) holds X[channel 4s + g][key k0 + 16w + c16]
  const int key = k0 + kT * w + c16;
  const bool key_ok = key < nk;
  float kb[kD / 4], vb[kD / 4];
#pragma unroll
  for (int s = 0; s < kD / 4; ++s) {
    const int c = 4 * s + g;
    kb[s] = (key_ok && c < d) ? K[(int64_t)c * nk + key] * c2 : 0.f;
    vb[s] = (key_ok && c < vd) ? V[(int64_t)c * nk + key] : 0.f;
  }

  const int klast = min(k0 + kBlk, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / kT) * kT;
  const int ntiles = (qe > qb) ? (qe - qt0 + kT - 1) / kT : 0;
  const int wk0 = k0 + kT * w, wk1 = min(wk0 + kT - 1, nk - 1);
  const bool wave_active = wk0 < nk;
  const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;
  int qlo = 0, qspan = nq;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
  }

  Stream16 st{static_cast<const float*>(a.Q) + bi * (int64_t)d * nq,
              static_cast<const float*>(a.dO) + bi * (int64_t)vd * nq, d, vd, nq, qvec, {}};
  float lr = 0.f;
  auto load_tile = [&](int qa) {
    st.load(qa);
    if (tid < 2 * kT) {
      const int q = qa + (tid & (kT - 1));
      lr = (q < nq) ? ((tid < kT) ? glse[q] : gD[q]) : ((tid < kT) ? __builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot) {
    lds_f_t* base = smem + slot * kSlot;
    st.store(base);
    if (tid < 2 * kT) base[2 * kImg + tid] = lr;
  };

  floatx4 dk[kD / 16], dv[kD / 16];
#pragma unroll
  for (int u = 0; u < kD / 16; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) { dk[u][i] = 0.f; dv[u][i] = 0.f; }

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
    const lds_f_t* base = smem + (it & 1) * kSlot;
    const lds_f_t* imQ = base;
    const lds_f_t* imO = base + kImg;
    floatx4 sacc, pacc;  // register i: query qa + 4g + i, key = this lane's
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sacc[i] = -base[2 * kImg + 4 * g + i];
      pacc[i] = -base[2 * kImg + kT + 4 * g + i];
    }
    // A = Qᵀ / dOᵀ: row = query c16, k = channel 4s + g
    // (two chains each over the even / odd k-steps: four independent MFMA chains in flight; every A
    // operand read kAh k-steps ahead into a register rotation, so no MFMA waits on its own read)
    floatx4 sacc1 = {0.f, 0.f, 0.f, 0.f}, pacc1 = {0.f, 0.f, 0.f, 0.f};
    constexpr int kAh = 4;
    float aq[kAh + 1], ao[kAh + 1];
    auto rd = [&](int n) __attribute__((always_inline)) {
      aq[n % (kAh + 1)] = imQ[(4 * n + g) * kRP + c16];
      ao[n % (kAh + 1)] = imO[(4 * n + g) * kRP + c16];
    };
#pragma unroll
    for (int n = 0; n < kAh; ++n) rd(n);
#pragma unroll
    for (int n = 0; n < kD / 4; ++n) {
      if (n + kAh < kD / 4) rd(n + kAh);
      if (n & 1) {
        sacc1 = mfma16(aq[n % (kAh + 1)], kb[n], sacc1);
        pacc1 = mfma16(ao[n % (kAh + 1)], vb[n], pacc1);
      } else {
        sacc = mfma16(aq[n % (kAh + 1)], kb[n], sacc);
        pacc = mfma16(ao[n % (kAh + 1)], vb[n], pacc);
      }
    }
    sacc += sacc1;
    pacc += pacc1;
    float p[4], ds[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (POL != 0 && cls == 1) {
        const int q = qa + 4 * g + i;
        bool ok;
        if (POL == 1) ok = (unsigned)(q - qlo) < (unsigned)qspan;
        else ok = (q < nq) && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko);
        pv = ok ? pv : 0.f;
      }
      p[i] = pv;
      ds[i] = pv * pacc[i];
    }
    // dV += dO·P, dK += Q·dS: k-step i = queries 4g' + i; A = X[channel 16u + c16][query 4g + i]
    // (read kAh products ahead, as above)
    auto rdg = [&](int m) __attribute__((always_inline)) {
      const int i = m / (kD / 16), u = m % (kD / 16), off = (16 * u + c16) * kRP + 4 * g + i;
      ao[m % (kAh + 1)] = imO[off];
      aq[m % (kAh + 1)] = imQ[off];
    };
#pragma unroll
    for (int m = 0; m < kAh; ++m) rdg(m);
#pragma unroll
    for (int m = 0; m < 4 * (kD / 16); ++m) {
      if (m + kAh < 4 * (kD / 16)) rdg(m + kAh);
      const int i = m / (kD / 16), u = m % (kD / 16);
      dv[u] = mfma16(ao[m % (kAh + 1)], p[i], dv[u]);
      dk[u] = mfma16(aq[m % (kAh + 1)], ds[i], dk[u]);
    }
  }

  if (!wave_active || !key_ok) return;
  float* dK = static_cast<float*>(a.dK) + bi * (int64_t)d * nk;
  float* dV = static_cast<float*>(a.dV) + bi * (int64_t)vd * nk;
  const float sc = (float)a.scale;
  // register i of block u: channel 16u + 4g + i, key = this lane's
#pragma unroll
  for (int u = 0; u < kD / 16; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * u + 4 * g + i;
      if (c < d) dK[(int64_t)c * nk + key] = dk[u][i] * sc;
      if (c < vd) dV[(int64_t)c * nk + key] = dv[u][i];
    }
}

// ---------------------------------------------------------------------------
// dQ: 4 waves x 16 queries a workgroup; key tiles of 16 stream through LDS.
template <int POL>
__global__ __launch_bounds__(kThr, 1) void bwd_dq_f32w_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_f_t* smem = (lds_f_t*)smem_raw;
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nqb = (nq + kBlk - 1) / kBlk;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBlk;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const float c2 = (float)a.scale * kLog2e;
  const float* Q = static_cast<const float*>(a.Q) + bi * (int64_t)d * nq;
  const float* dO = static_cast<const float*>(a.dO) + bi * (int64_t)vd * nq;
  const bool kvec = ((nk & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);

  // ---- resident B operands: lane (g, c16) holds X[channel 4s + g][query q0 + 16w + c16]
  const int qi = q0 + kT * w + c16;
  const bool q_ok = qi < nq;
  float qf[kD / 4], of[kD / 4];
#pragma unroll
  for (int s = 0; s < kD / 4; ++s) {
    const int c = 4 * s + g;
    qf[s] = (q_ok && c < d) ? Q[(int64_t)c * nq + qi] * c2 : 0.f;
    of[s] = (q_ok && c < vd) ? dO[(int64_t)c * nq + qi] : 0.f;
  }
  const int wq0 = q0 + kT * w, wq1 = min(wq0 + kT - 1, nq - 1);
  const bool wave_active = wq0 < nq;
  constexpr float kNegInf = -__builtin_huge_valf();
  float negl, negd;
  {
    const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
    const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
    negl = q_ok ? -glse[qi] : kNegInf;
    negd = q_ok ? -gD[qi] : 0.f;
  }
  const int qlast = min(q0 + kBlk, nq) - 1;
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

  Stream16 st{static_cast<const float*>(a.K) + bi * (int64_t)d * nk,
              static_cast<const float*>(a.V) + bi * (int64_t)vd * nk, d, vd, nk, kvec, {}};

  floatx4 dq[kD / 16];
#pragma unroll
  for (int u = 0; u < kD / 16; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) dq[u][i] = 0.f;

  if (ntiles > 0) { st.load(kt0); st.store(smem); }
  if (ntiles > 1) st.load(kt0 + kT);
  for (int it = 0; it < ntiles; ++it) {
    __syncthreads();
    const int ka = kt0 + it * kT;
    if (it + 1 < ntiles) st.store(smem + ((it + 1) & 1) * kSlot);
    if (it + 2 < ntiles) st.load(ka + 2 * kT);
    int cls;
    if (!wave_active) cls = 0;
    else if (POL == 0) cls = (ka + kT <= nk) ? 2 : 1;
    else {
      cls = tile_class(a.rule, wq0, wq1, ka, min(ka + kT, nk) - 1);
      if (cls == 2 && ka + kT > nk) cls = 1;
    }
    if (cls == 0) continue;
    const lds_f_t* imK = smem + (it & 1) * kSlot;
    const lds_f_t* imV = imK + kImg;
    floatx4 sacc, pacc;  // register i: key ka + 4g + i, query = this lane's
#pragma unroll
    for (int i = 0; i < 4; ++i) { sacc[i] = negl; pacc[i] = negd; }
    // A = Kᵀ / Vᵀ: row = key c16, k = channel 4s + g
    floatx4 sacc1 = {0.f, 0.f, 0.f, 0.f}, pacc1 = {0.f, 0.f, 0.f, 0.f};  // (four chains and read-ahead, as in dK/dV)
    constexpr int kAh = 4;
    float ak[kAh + 1], av[kAh + 1];
    auto rd = [&](int n) __attribute__((always_inline)) {
      ak[n % (kAh + 1)] = imK[(4 * n + g) * kRP + c16];
      av[n % (kAh + 1)] = imV[(4 * n + g) * kRP + c16];
    };
#pragma unroll
    for (int n = 0; n < kAh; ++n) rd(n);
#pragma unroll
    for (int n = 0; n < kD / 4; ++n) {
      if (n + kAh < kD / 4) rd(n + kAh);
      if (n & 1) {
        sacc1 = mfma16(ak[n % (kAh + 1)], qf[n], sacc1);
        pacc1 = mfma16(av[n % (kAh + 1)], of[n], pacc1);
      } else {
        sacc = mfma16(ak[n % (kAh + 1)], qf[n], sacc);
        pacc = mfma16(av[n % (kAh + 1)], of[n], pacc);
      }
    }
    sacc += sacc1;
    pacc += pacc1;
    float ds[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (cls == 1) {
        const int kk = ka + 4 * g + i;
        bool ok = kk < nk;
        if (POL == 1) ok &= (unsigned)(kk - klo) < (unsigned)kspan;
        if (POL == 2) ok &= check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1)));
        pv = ok ? pv : 0.f;
      }
      ds[i] = pv * pacc[i];
    }
    // dQ += K·dSᵀ: k-step i = keys 4g' + i; A = K[channel 16u + c16][key 4g + i]
    auto rdg = [&](int m) __attribute__((always_inline)) {
      const int i = m / (kD / 16), u = m % (kD / 16);
      ak[m % (kAh + 1)] = imK[(16 * u + c16) * kRP + 4 * g + i];
    };
#pragma unroll
    for (int m = 0; m < kAh; ++m) rdg(m);
#pragma unroll
    for (int m = 0; m < 4 * (kD / 16); ++m) {
      if (m + kAh < 4 * (kD / 16)) rdg(m + kAh);
      dq[m % (kD / 16)] = mfma16(ak[m % (kAh + 1)], ds[m / (kD / 16)], dq[m % (kD / 16)]);
    }
  }

  if (!wave_active || !q_ok) return;
  float* dQ = static_cast<float*>(a.dQ) + bi * (int64_t)d * nq;
  const float sc = (float)a.scale;
#pragma unroll
  for (int u = 0; u < kD / 16; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * u + 4 * g + i;
      if (c < d) dQ[(int64_t)c * nq + qi] = dq[u][i] * sc;
    }
}

}  // namespace

hipError_t launch_bwd_f32_wide(const BwdArgs& a, hipStream_t s) {
  const int pol = a.rule.policy == 0 ? 0 : (rule_is_interval(a.rule) ? 1 : 2);
  auto kk = pol == 0 ? bwd_dkdv_f32w_kernel<0> : (pol == 1 ? bwd_dkdv_f32w_kernel<1> : bwd_dkdv_f32w_kernel<2>);
  auto kq = pol == 0 ? bwd_dq_f32w_kernel<0> : (pol == 1 ? bwd_dq_f32w_kernel<1> : bwd_dq_f32w_kernel<2>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kk), kSmem);
  if (e != hipSuccess) return e;
  e = set_smem_once(reinterpret_cast<const void*>(kq), kSmem);
  if (e != hipSuccess) return e;
  const int64_t nkb = (a.rule.k.n + kBlk - 1) / kBlk, nqb = (a.rule.q.n + kBlk - 1) / kBlk;
  hipLaunchKernelGGL(kk, dim3((unsigned)(a.b * nkb)), dim3(kThr), kSmem, s, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kq, dim3((unsigned)(a.b * nqb)), dim3(kThr), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
