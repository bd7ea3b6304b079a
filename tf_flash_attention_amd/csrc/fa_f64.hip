// fa_f64.hip — fp64 fused attention forward + two-pass backward on gfx950 MFMA
// (v_mfma_f64_16x16x4_f64, 64 cycles, the only fp64 matrix instruction).
//
// Replaces the reference's ForwardImpl / BackwardImpl (flash_attention.cu:593-1967)
// for float64 inputs.  The f64 MFMA keeps IEEE double arithmetic, so the 1e-10
// parity target holds while the matrix work leaves the (equally fast on paper,
// but issue-bound) f64 VALU.  Structure follows the fp32 kernels (fa_fwd_f32.hip,
// fa_bwd_f32.hip) re-tiled for the 16x16 f64 shape:
//   A operand  lane (g = lane>>4, r = lane&15): A[row r][k g]     (one double)
//   B operand                                    B[k g][col r]
//   C/D        register i of lane (g, r):        C[row g + 4i][col r]
// so one wave owns 16 queries (forward, dq) or 16 keys (dkdv).  A 16x16 score
// tile Sᵀ (rows = keys) leaves register i of lane (g, r) holding key g + 4i:
// register i of every lane group is exactly the k-step {4i .. 4i+3} of the
// following product, so P / dS feed the PV / dV / dK / dQ MFMAs straight from
// registers.  Softmax runs in the natural-log domain with exp() from the device
// math library (full double accuracy).
//   forward : Sᵀ = Kᵀ·(scale·Q) (C = -m),  Oᵀ += V·Pᵀ,  lazy max rebase
//   prep    : D = rowsum(dO∘O), lse = m + log l (+inf for empty rows)
//   dkdv    : key-outer, K·scale and V resident; S = Qᵀ·K' (C = -lse), dP = dOᵀ·V (C = -D)
//   dq      : query-outer, Q·scale and dO resident; Sᵀ = Kᵀ·Q', dPᵀ = Vᵀ·dO, dQ += K·dSᵀ
// At 64 < D <= 128 the backward streams 16-column tiles (the two-slot ring of the Q/dO row and
// transposed images then fits LDS) and the dK/dV pass runs twice, each launch accumulating one
// half of the channels (the resident K', V operands plus all 128 channels of dK and dV would not
// fit two waves per SIMD): the S / dP products are formed in both launches.
// At 128 < D <= 256 every kernel runs four waves (one per SIMD, the whole 512-entry register file:
// the resident operands alone are 128 registers a tensor) over 64-query (key) blocks and 16-column
// tiles; the backward passes hold a quarter (dK / dV) or half (dQ) of their output channels per
// launch and stage one tile at a time (a tile's four images are 132 KB).
// Row images ([channel][32 keys|queries]) swap their 16-column halves on odd
// channel rows so the four lane groups of an A-operand read hit disjoint banks;
// transposed images ([32][D+16]) are padded for the same reason.
#include "fa_device.h"
#include "fa_kernels.h"

namespace fa {
namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef double doublex2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) double lds_d_t;
typedef __attribute__((address_space(3))) doublex2 lds_d2_t;

// NW waves a workgroup, each 16 queries (keys): 8 up to D = 128, 4 past it
template <int NW> constexpr int thr_of() { return 64 * NW; }
template <int NW> constexpr int bm_of() { return 16 * NW; }
constexpr int kT = 32;      // streamed keys (queries) per tile
constexpr int kThrPrep = 256;
constexpr double kRebase = 16.0;  // lazy max rebase threshold (natural units)

__device__ __forceinline__ doublex4 mma(double a, double b, doublex4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ doublex4 splat4(double x) { return doublex4{x, x, x, x}; }
// reductions over the four lane groups that share a column (lanes r, r+16, r+32, r+48)
__device__ __forceinline__ double grp_max(double x) {
  x = fmax(x, __shfl_xor(x, 16));
  return fmax(x, __shfl_xor(x, 32));
}
__device__ __forceinline__ double grp_sum(double x) {
  x += __shfl_xor(x, 16);
  return x + __shfl_xor(x, 32);
}
// row image index: [c][TT] — at TT = 32 with the 16-column halves swapped on odd rows (a 256-B
// row puts the four lane groups' rows of an A read on the same banks otherwise); 128-B rows
// (TT = 16) already fall in alternate bank halves
template <int TT = kT>
__device__ __forceinline__ int rimg(int c, int col) {
  return TT == 32 ? c * TT + (col ^ ((c & 1) << 4)) : c * TT + col;
}
// doubles row[e], row[e+1] (zeros past n)
__device__ __forceinline__ doublex2 load2(const double* row, int e, int n, bool vec) {
  if (vec && e + 2 <= n) return *reinterpret_cast<const doublex2*>(row + e);
  doublex2 v = {0.0, 0.0};
  if (e < n) v[0] = row[e];
  if (e + 1 < n) v[1] = row[e + 1];
  return v;
}
__device__ __forceinline__ bool vec_ok(int n, const void* p0, const void* p1) {
  return ((n & 1) == 0) && ((reinterpret_cast<uintptr_t>(p0) & 15) == 0) && ((reinterpret_cast<uintptr_t>(p1) & 15) == 0);
}

// Streams tensors A [da][n] and B [db][n] in kT-column tiles: row image of A, row image
// of B (kRB), transposed images ([kT][D+16]) of A (kTA) and B (kTB).  Register-staged
// one tile ahead.
template <int D, bool kRB, bool kTA, bool kTB, int TT = kT, int NW = 8>
struct Stream64 {
  static constexpr int kThr = thr_of<NW>();
  static constexpr int kP = D + 16;
  static constexpr int offA = 0, offB = D * TT, offAT = offB + (kRB ? D * TT : 0);
  static constexpr int offBT = offAT + (kTA ? TT * kP : 0);
  static constexpr int offC = offBT + (kTB ? TT * kP : 0);
  static constexpr int kSlot = offC + 2 * TT;         // doubles (+ two TT row-constant vectors)
  static constexpr int kCR = TT / 2;                  // double2 chunks per row
  static constexpr int kChunks = D * kCR;             // double2 chunks per tensor
  static constexpr int kCPT = (2 * kChunks + kThr - 1) / kThr;
  const double* A;
  const double* B;
  int da, db, n;
  bool vec;
  doublex2 reg[kCPT];
  __device__ void load(int col0) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = threadIdx.x + kThr * j;
      doublex2 v = {0.0, 0.0};
      if (idx < 2 * kChunks) {
        const bool isB = idx >= kChunks;
        const int k = isB ? idx - kChunks : idx, c = k / kCR, m = k % kCR;
        if (c < (isB ? db : da)) v = load2((isB ? B : A) + (int64_t)c * n, col0 + 2 * m, n, vec);
      }
      reg[j] = v;
    }
  }
  __device__ static void put(lds_d_t* slot, int idx, doublex2 v) {
    if (idx < 2 * kChunks) {
      const bool isB = idx >= kChunks;
      const int k = isB ? idx - kChunks : idx, c = k / kCR, m = k % kCR;
      if (!isB || kRB) *reinterpret_cast<lds_d2_t*>(slot + (isB ? offB : offA) + rimg<TT>(c, 2 * m)) = v;
      if (isB ? kTB : kTA) {
        lds_d_t* tr = slot + (isB ? offBT : offAT);
        tr[(2 * m) * kP + c] = v[0];
        tr[(2 * m + 1) * kP + c] = v[1];
      }
    }
  }
  __device__ void store(lds_d_t* slot) const {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) put(slot, threadIdx.x + kThr * j, reg[j]);
  }
  // the tile at col0 straight into slot, four chunks a thread at a time (no staging registers
  // live beyond the group)
  __device__ void copy(lds_d_t* slot, int col0) const {
#pragma unroll 1
    for (int j0 = 0; j0 < kCPT; j0 += 4) {
      doublex2 v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int idx = threadIdx.x + kThr * (j0 + jj);
        v[jj] = doublex2{0.0, 0.0};
        if (j0 + jj < kCPT && idx < 2 * kChunks) {
          const bool isB = idx >= kChunks;
          const int k = isB ? idx - kChunks : idx, c = k / kCR, m = k % kCR;
          if (c < (isB ? db : da)) v[jj] = load2((isB ? B : A) + (int64_t)c * n, col0 + 2 * m, n, vec);
        }
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (j0 + jj < kCPT) put(slot, threadIdx.x + kThr * (j0 + jj), v[jj]);
    }
  }
};

// ring slots of a streamed tile: up to D = 128 two (register-staged one tile ahead, stored beside
// the compute); past it one, loaded and stored between two barriers (the staging registers of a
// 256-channel tile, 64 a lane, would spill the resident operands)
constexpr int kLdsBytes = 160 * 1024;
template <int D> constexpr int slots_of() { return D <= 128 ? 2 : 1; }

// resident operand: X[c = 4s + g][col0 + 16w + r] of a [dx][n] tensor via an LDS [D][128] image
template <int D, int NW>
__device__ __forceinline__ void stage_block(lds_d_t* img, const double* X, int dx, int n, int col0, bool vec) {
  constexpr int kThr = thr_of<NW>(), kBM = bm_of<NW>();
  for (int idx = threadIdx.x; idx < D * (kBM / 2); idx += kThr) {
    const int c = idx / (kBM / 2), m = idx % (kBM / 2);
    doublex2 v = {0.0, 0.0};
    if (c < dx) v = load2(X + (int64_t)c * n, col0 + 2 * m, n, vec);
    *reinterpret_cast<lds_d2_t*>(img + c * kBM + 2 * m) = v;
  }
}

// ---------------------------------------------------------------------------
// forward: 8 waves x 16 queries; key tiles of 32 (K row image + V transposed image)
//   POL 0 full, 1 interval rules, 2 any other rule (per-element order check)
template <int D, int POL, int NW, int TT>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 2 : 1) void fwd_f64_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_d_t* smem = (lds_d_t*)smem_raw;
  constexpr int kBM = bm_of<NW>();
  constexpr int kNT = TT / 16;  // 16-key blocks per tile
  using St = Stream64<D, false, false, true, TT, NW>;
  const double kNegInf = -__builtin_huge_val();
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const double sc = a.scale;
  const double* Q = static_cast<const double*>(a.Q) + bi * (int64_t)d * nq;

  stage_block<D, NW>(smem, Q, d, nq, q0, vec_ok(nq, a.Q, a.Q));
  __syncthreads();
  double qf[D / 4];  // B operand of Sᵀ: Q[c = 4s + g][q = 16w + r] * scale
#pragma unroll
  for (int s = 0; s < D / 4; ++s) qf[s] = smem[(4 * s + g) * kBM + 16 * w + r] * sc;
  __syncthreads();

  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / TT) * TT;
  const int ntiles = (ke > kb) ? (ke - kt0 + TT - 1) / TT : 0;
  const int wq0 = q0 + 16 * w, wq1 = min(wq0 + 15, nq - 1);
  const bool wave_active = wq0 < nq;
  const int qi = wq0 + r;
  const int qo = (POL == 2 && qi < nq) ? seq_order(a.rule.q, a.rule, qi) : 0;
  int klo = 0, kspan = 0, wlo_min = 0, wlo_max = 0, whi_min = 0, whi_max = 0;
  if (POL == 1 && wave_active) {
    int khi;
    key_interval(a.rule, min(qi, nq - 1), &klo, &khi);
    kspan = max(khi - klo + 1, 0);
    const int last = min(15, nq - 1 - wq0);
    wlo_min = __builtin_amdgcn_readfirstlane(klo);
    whi_min = __builtin_amdgcn_readfirstlane(khi);
    wlo_max = __builtin_amdgcn_readlane(klo, last);
    whi_max = __builtin_amdgcn_readlane(khi, last);
  }
  St st{static_cast<const double*>(a.K) + bi * (int64_t)d * nk, static_cast<const double*>(a.V) + bi * (int64_t)vd * nk,
        d, vd, nk, vec_ok(nk, a.K, a.V), {}};

  doublex4 acc[D / 16];
#pragma unroll
  for (int u = 0; u < D / 16; ++u) acc[u] = splat4(0.0);
  double m_run = 0.0, l_run = 0.0, m_max = kNegInf;
  bool m_set = false;

  constexpr int kSlots = slots_of<D>();
  if (kSlots == 2 && ntiles > 0) st.load(kt0);
  for (int it = 0; it < ntiles; ++it) {
    const int k0 = kt0 + it * TT;
    if constexpr (kSlots == 2) {
      st.store(smem + (it & 1) * St::kSlot);
      if (it + 1 < ntiles) st.load(k0 + TT);
    } else {
      __syncthreads();
      st.copy(smem, k0);
    }
    __syncthreads();

    const int k1 = k0 + TT - 1;
    int cls;
    if (!wave_active) cls = 0;
    else if (POL == 0) cls = k1 < nk ? 2 : 1;
    else if (POL == 1) cls = (wlo_min > k1 || whi_max < k0) ? 0 : ((wlo_max <= k0 && whi_min >= k1) ? 2 : 1);
    else {
      cls = tile_class(a.rule, wq0, wq1, k0, min(k1, nk - 1));
      if (cls == 2 && k1 >= nk) cls = 1;
    }
    if (cls == 0) continue;
    const lds_d_t* base = smem + (kSlots == 2 ? (it & 1) : 0) * St::kSlot;

    // Sᵀ - m: A = Kᵀ (lane: key 16t + r, channel 4s + g)
    doublex4 s4[kNT];
#pragma unroll
    for (int t = 0; t < kNT; ++t) s4[t] = splat4(-m_run);
#pragma unroll
    for (int s = 0; s < D / 4; ++s)
#pragma unroll
      for (int t = 0; t < kNT; ++t) s4[t] = mma(base[St::offA + rimg<TT>(4 * s + g, 16 * t + r)], qf[s], s4[t]);
    if (cls == 1) {
#pragma unroll
      for (int t = 0; t < kNT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + 16 * t + g + 4 * i;
          bool ok;
          if (POL == 1) ok = (unsigned)(key - klo) < (unsigned)kspan;
          else {
            ok = key < nk;
            if (POL == 2) ok &= check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(key, nk - 1)));
          }
          s4[t][i] = ok ? s4[t][i] : kNegInf;
        }
    }
    double mt = fmax(fmax(s4[0][0], s4[0][1]), fmax(s4[0][2], s4[0][3]));
#pragma unroll
    for (int t = 1; t < kNT; ++t) mt = fmax(mt, fmax(fmax(s4[t][0], s4[t][1]), fmax(s4[t][2], s4[t][3])));
    mt = grp_max(mt);
    m_max = fmax(m_max, m_run + mt);
    const bool seed = !m_set && (mt != kNegInf);
    if (__any((mt > kRebase) | seed)) {
      const double delta = m_set ? fmax(mt, 0.0) : (seed ? mt : 0.0);
      const double alpha = m_set ? exp(-delta) : 1.0;
      m_run += delta;
      m_set = m_set || seed;
      l_run *= alpha;
#pragma unroll
      for (int u = 0; u < D / 16; ++u) acc[u] *= alpha;
#pragma unroll
      for (int t = 0; t < kNT; ++t) s4[t] -= delta;
    }
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s4[t][i] = exp(s4[t][i]);
        l_run += s4[t][i];
      }
    // Oᵀ[v][q] += Σ_key V[v][key] P[key][q]: k-step (t, i) = keys 16t + 4i + g
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const lds_d_t* vrow = base + St::offBT + (16 * t + 4 * i + g) * St::kP + r;
#pragma unroll
        for (int u = 0; u < D / 16; ++u) acc[u] = mma(vrow[16 * u], s4[t][i], acc[u]);
      }
  }

  if (!wave_active) return;
  const double l_tot = grp_sum(l_run);
  const double inv = (l_tot > 0.0) ? 1.0 / l_tot : 0.0;
  if (qi < nq) {
    double* O = static_cast<double*>(a.O) + bi * (int64_t)vd * nq;
#pragma unroll
    for (int u = 0; u < D / 16; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int v = 16 * u + g + 4 * i;
        if (v < vd) O[(int64_t)v * nq + qi] = acc[u][i] * inv;
      }
    if (g == 0) {
      double* lo = static_cast<double*>(a.l) + bi * (int64_t)nq;
      double* mo = static_cast<double*>(a.m) + bi * (int64_t)nq;
      if (l_tot > 0.0) {
        lo[qi] = l_tot * exp(m_run - m_max);
        mo[qi] = m_max;
      } else {
        lo[qi] = 0.0;
        mo[qi] = neg_inf_approx<double>();
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward prep: D = rowsum(dO∘O), lse = m + log l
__global__ __launch_bounds__(kThrPrep) void bwd_prep_f64_kernel(BwdArgs a) {
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t i = blockIdx.x * (int64_t)kThrPrep + threadIdx.x;
  if (i >= a.b * (int64_t)nq) return;
  const int64_t bi = i / nq;
  const int q = (int)(i - bi * nq);
  const double* O = static_cast<const double*>(a.O) + bi * (int64_t)vd * nq + q;
  const double* dO = static_cast<const double*>(a.dO) + bi * (int64_t)vd * nq + q;
  double D0 = 0.0, D1 = 0.0;
  int v = 0;
  for (; v + 1 < vd; v += 2) {
    D0 = fma(O[(int64_t)v * nq], dO[(int64_t)v * nq], D0);
    D1 = fma(O[(int64_t)(v + 1) * nq], dO[(int64_t)(v + 1) * nq], D1);
  }
  if (v < vd) D0 = fma(O[(int64_t)v * nq], dO[(int64_t)v * nq], D0);
  const double l = static_cast<const double*>(a.l)[i];
  const double m = static_cast<const double*>(a.m)[i];
  static_cast<double*>(a.ws_D)[i] = D0 + D1;
  static_cast<double*>(a.ws_lse)[i] = (l > 0.0) ? m + log(l) : __builtin_huge_val();
}

// D <= 64: the resident K and V (Q and dO) blocks are staged together; above one after the other
template <int D, int TT, int NW, typename St>
constexpr int bwd64_smem() {
  constexpr int s1 = slots_of<D>() * St::kSlot, s2 = (D > 64 ? 1 : 2) * D * bm_of<NW>();
  return 8 * (s1 > s2 ? s1 : s2);
}

// resident B operands X[c = 4s + g][col0 + 16w + r] (x scale) of two tensors, through LDS: both images
// at once for D <= 64, one at a time above (a [128][128] double image is 128 KB)
template <int D, int NW>
__device__ __forceinline__ void resident_pair(lds_d_t* smem, const double* X, int dx, const double* Y, int dy, int n,
                                              int col0, bool vec, double xs, double (&xf)[D / 4], double (&yf)[D / 4]) {
  constexpr int kBM = bm_of<NW>();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  if constexpr (D <= 64) {
    stage_block<D, NW>(smem, X, dx, n, col0, vec);
    stage_block<D, NW>(smem + D * kBM, Y, dy, n, col0, vec);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 4; ++s) {
      xf[s] = smem[(4 * s + g) * kBM + 16 * w + r] * xs;
      yf[s] = smem[D * kBM + (4 * s + g) * kBM + 16 * w + r];
    }
  } else {
    stage_block<D, NW>(smem, X, dx, n, col0, vec);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 4; ++s) xf[s] = smem[(4 * s + g) * kBM + 16 * w + r] * xs;
    __syncthreads();
    stage_block<D, NW>(smem, Y, dy, n, col0, vec);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 4; ++s) yf[s] = smem[(4 * s + g) * kBM + 16 * w + r];
  }
  __syncthreads();
}

// dK / dV: NW waves x 16 keys; query tiles of TT (Q, dO row + transposed images, lse, D).
// Channels [CH·D/NCH, (CH + 1)·D/NCH) of dK / dV (NCH = 1: every channel)
template <int D, int POL, int TT, int CH, int NCH, int NW>
__global__ __launch_bounds__(64 * NW, 1) void bwd_dkdv_f64_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_d_t* smem = (lds_d_t*)smem_raw;
  constexpr int kBM = bm_of<NW>();
  using St = Stream64<D, true, true, true, TT, NW>;
  constexpr int kNT = TT / 16;                      // 16-query blocks per tile
  constexpr int kNU = D / NCH / 16;                 // 16-channel blocks of dK / dV held
  constexpr int kC0 = CH * (D / NCH);               // first channel held
  constexpr int kSlots = slots_of<D>();
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nkb = (nk + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const double sc = a.scale;
  const double* K = static_cast<const double*>(a.K) + bi * (int64_t)d * nk;
  const double* V = static_cast<const double*>(a.V) + bi * (int64_t)vd * nk;
  const double* glse = static_cast<const double*>(a.ws_lse) + bi * (int64_t)nq;
  const double* gD = static_cast<const double*>(a.ws_D) + bi * (int64_t)nq;

  double kb[D / 4], vb[D / 4];  // B operands: X[c = 4s + g][key = k0 + 16w + r]
  resident_pair<D, NW>(smem, K, d, V, vd, nk, k0, vec_ok(nk, a.K, a.V), sc, kb, vb);

  const int klast = min(k0 + kBM, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / TT) * TT;
  const int ntiles = (qe > qb) ? (qe - qt0 + TT - 1) / TT : 0;
  const int wk0 = k0 + 16 * w, wk1 = min(wk0 + 15, nk - 1);
  const int key = wk0 + r;
  const bool wave_active = wk0 < nk;
  const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;
  int qlo = 0, qspan = nq;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
  }

  St st{static_cast<const double*>(a.Q) + bi * (int64_t)d * nq, static_cast<const double*>(a.dO) + bi * (int64_t)vd * nq,
        d, vd, nq, vec_ok(nq, a.Q, a.dO), {}};
  double cr = 0.0;
  auto load_tile = [&](int qa) {
    st.load(qa);
    if (tid < 2 * TT) {
      const int q = qa + (tid & (TT - 1));
      cr = (q < nq) ? ((tid < TT) ? glse[q] : gD[q]) : ((tid < TT) ? __builtin_huge_val() : 0.0);
    }
  };
  auto store_tile = [&](int slot) {
    lds_d_t* b = smem + slot * St::kSlot;
    st.store(b);
    if (tid < 2 * TT) b[St::offC + tid] = cr;
  };

  doublex4 dk[kNU], dv[kNU];
#pragma unroll
  for (int u = 0; u < kNU; ++u) dk[u] = dv[u] = splat4(0.0);

  if (kSlots == 2 && ntiles > 0) {
    load_tile(qt0);
    store_tile(0);
  }
  if (kSlots == 2 && ntiles > 1) load_tile(qt0 + TT);
  for (int it = 0; it < ntiles; ++it) {
    __syncthreads();
    const int qa = qt0 + it * TT;
    if constexpr (kSlots == 2) {
      if (it + 1 < ntiles) store_tile((it + 1) & 1);
      if (it + 2 < ntiles) load_tile(qa + 2 * TT);
    } else {  // one slot: this tile copied in between two barriers
      st.copy(smem, qa);
      if (tid < 2 * TT) {
        const int q = qa + (tid & (TT - 1));
        smem[St::offC + tid] = (q < nq) ? ((tid < TT) ? glse[q] : gD[q]) : ((tid < TT) ? __builtin_huge_val() : 0.0);
      }
      __syncthreads();
    }
    int cls = 2;
    if (!wave_active) cls = 0;
    else if (POL != 0) cls = tile_class(a.rule, qa, min(qa + TT, nq) - 1, wk0, wk1);
    if (cls == 0) continue;
    const lds_d_t* base = smem + (kSlots == 2 ? (it & 1) : 0) * St::kSlot;
    doublex4 sacc[kNT], pacc[kNT];
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ql = 16 * t + g + 4 * i;
        sacc[t][i] = -base[St::offC + ql];
        pacc[t][i] = -base[St::offC + TT + ql];
      }
    // S = Qᵀ·K', dP = dOᵀ·V: A = X[c = 4s + g][q = 16t + r] from the row images
#pragma unroll
    for (int s = 0; s < D / 4; ++s)
#pragma unroll
      for (int t = 0; t < kNT; ++t) {
        sacc[t] = mma(base[St::offA + rimg<TT>(4 * s + g, 16 * t + r)], kb[s], sacc[t]);
        pacc[t] = mma(base[St::offB + rimg<TT>(4 * s + g, 16 * t + r)], vb[s], pacc[t]);
      }
    double p[kNT][4], ds[kNT][4];
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double pv = exp(sacc[t][i]);
        if (POL != 0 && cls == 1) {
          const int q = qa + 16 * t + g + 4 * i;
          bool ok;
          if (POL == 1) ok = (unsigned)(q - qlo) < (unsigned)qspan;
          else ok = (q < nq) && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko);
          pv = ok ? pv : 0.0;
        }
        p[t][i] = pv;
        ds[t][i] = pv * pacc[t][i];
      }
    // dV += dO·P, dK += Q·dS: k-step (t, i) = queries 16t + 4i + g (transposed images)
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ql = 16 * t + 4 * i + g;
#pragma unroll
        for (int u = 0; u < kNU; ++u) {
          dv[u] = mma(base[St::offBT + ql * St::kP + kC0 + 16 * u + r], p[t][i], dv[u]);
          dk[u] = mma(base[St::offAT + ql * St::kP + kC0 + 16 * u + r], ds[t][i], dk[u]);
        }
      }
  }

  if (!wave_active || key >= nk) return;
  double* dK = static_cast<double*>(a.dK) + bi * (int64_t)d * nk;
  double* dV = static_cast<double*>(a.dV) + bi * (int64_t)vd * nk;
#pragma unroll
  for (int u = 0; u < kNU; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = kC0 + 16 * u + g + 4 * i;
      if (c < d) dK[(int64_t)c * nk + key] = dk[u][i] * sc;
      if (c < vd) dV[(int64_t)c * nk + key] = dv[u][i];
    }
}

// dQ: NW waves x 16 queries; key tiles of TT (K, V row images + K transposed image).
// Channels [CH·D/NCH, (CH + 1)·D/NCH) of dQ
template <int D, int POL, int TT, int CH, int NCH, int NW>
__global__ __launch_bounds__(64 * NW, 1) void bwd_dq_f64_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_d_t* smem = (lds_d_t*)smem_raw;
  constexpr int kBM = bm_of<NW>();
  using St = Stream64<D, true, true, false, TT, NW>;
  constexpr int kNT = TT / 16;  // 16-key blocks per tile
  constexpr int kNU = D / NCH / 16;  // 16-channel blocks of dQ held
  constexpr int kC0 = CH * (D / NCH);
  constexpr int kSlots = slots_of<D>();
  const double kNegInf = -__builtin_huge_val();
  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const double sc = a.scale;
  const double* Q = static_cast<const double*>(a.Q) + bi * (int64_t)d * nq;
  const double* dO = static_cast<const double*>(a.dO) + bi * (int64_t)vd * nq;

  double qf[D / 4], of[D / 4];  // B operands: X[c = 4s + g][q = q0 + 16w + r]
  resident_pair<D, NW>(smem, Q, d, dO, vd, nq, q0, vec_ok(nq, a.Q, a.dO), sc, qf, of);

  const int wq0 = q0 + 16 * w, wq1 = min(wq0 + 15, nq - 1);
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;
  double nl, nd;
  {
    const double* glse = static_cast<const double*>(a.ws_lse) + bi * (int64_t)nq;
    const double* gD = static_cast<const double*>(a.ws_D) + bi * (int64_t)nq;
    nl = (qi < nq) ? -glse[qi] : kNegInf;
    nd = (qi < nq) ? -gD[qi] : 0.0;
  }
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / TT) * TT;
  const int ntiles = (ke > kb) ? (ke - kt0 + TT - 1) / TT : 0;
  const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;
  int klo = 0, kspan = nk;
  if (POL == 1 && wave_active) {
    int khi;
    key_interval(a.rule, min(qi, nq - 1), &klo, &khi);
    kspan = max(khi - klo + 1, 0);
  }

  St st{static_cast<const double*>(a.K) + bi * (int64_t)d * nk, static_cast<const double*>(a.V) + bi * (int64_t)vd * nk,
        d, vd, nk, vec_ok(nk, a.K, a.V), {}};
  doublex4 dq[kNU];
#pragma unroll
  for (int u = 0; u < kNU; ++u) dq[u] = splat4(0.0);

  if (kSlots == 2 && ntiles > 0) {
    st.load(kt0);
    st.store(smem);
  }
  if (kSlots == 2 && ntiles > 1) st.load(kt0 + TT);
  for (int it = 0; it < ntiles; ++it) {
    __syncthreads();
    const int ka = kt0 + it * TT;
    if constexpr (kSlots == 2) {
      if (it + 1 < ntiles) st.store(smem + ((it + 1) & 1) * St::kSlot);
      if (it + 2 < ntiles) st.load(ka + 2 * TT);
    } else {
      st.copy(smem, ka);
      __syncthreads();
    }
    int cls;
    if (!wave_active) cls = 0;
    else if (POL == 0) cls = (ka + TT <= nk) ? 2 : 1;
    else {
      cls = tile_class(a.rule, wq0, wq1, ka, min(ka + TT, nk) - 1);
      if (cls == 2 && ka + TT > nk) cls = 1;
    }
    if (cls == 0) continue;
    const lds_d_t* base = smem + (kSlots == 2 ? (it & 1) : 0) * St::kSlot;
    doublex4 sacc[kNT], pacc[kNT];
#pragma unroll
    for (int t = 0; t < kNT; ++t) {
      sacc[t] = splat4(nl);
      pacc[t] = splat4(nd);
    }
#pragma unroll
    for (int s = 0; s < D / 4; ++s)
#pragma unroll
      for (int t = 0; t < kNT; ++t) {
        sacc[t] = mma(base[St::offA + rimg<TT>(4 * s + g, 16 * t + r)], qf[s], sacc[t]);
        pacc[t] = mma(base[St::offB + rimg<TT>(4 * s + g, 16 * t + r)], of[s], pacc[t]);
      }
    double ds[kNT][4];
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double pv = exp(sacc[t][i]);
        if (cls == 1) {
          const int kk = ka + 16 * t + g + 4 * i;
          bool ok = kk < nk;
          if (POL == 1) ok &= (unsigned)(kk - klo) < (unsigned)kspan;
          if (POL == 2) ok &= check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1)));
          pv = ok ? pv : 0.0;
        }
        ds[t][i] = pv * pacc[t][i];
      }
    // dQ[c][q] += Σ_key K[c][key] dSᵀ[key][q]: k-step (t, i) = keys 16t + 4i + g
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const lds_d_t* krow = base + St::offAT + (16 * t + 4 * i + g) * St::kP + kC0 + r;
#pragma unroll
        for (int u = 0; u < kNU; ++u) dq[u] = mma(krow[16 * u], ds[t][i], dq[u]);
      }
  }

  if (!wave_active || qi >= nq) return;
  double* dQ = static_cast<double*>(a.dQ) + bi * (int64_t)d * nq;
#pragma unroll
  for (int u = 0; u < kNU; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = kC0 + 16 * u + g + 4 * i;
      if (c < d) dQ[(int64_t)c * nq + qi] = dq[u][i] * sc;
    }
}

int policy_class(const Rule& r) { return r.policy == 0 ? 0 : (rule_is_interval(r) ? 1 : 2); }

// NW = 8 waves and 32-column tiles up to D = 64, 16-column tiles at D = 128; 4 waves past it
template <int D> constexpr int nw_of() { return D > 128 ? 4 : 8; }
template <int D> constexpr int tt_of() { return D > 64 ? 16 : kT; }

template <int D>
hipError_t launch_fwd_t(const FwdArgs& a, hipStream_t s) {
  constexpr int NW = nw_of<D>(), TT = D > 128 ? 16 : kT;
  using St = Stream64<D, false, false, true, TT, NW>;
  constexpr int sm1 = slots_of<D>() * St::kSlot, sm2 = D * bm_of<NW>();
  constexpr int smem = 8 * (sm1 > sm2 ? sm1 : sm2);
  static_assert(smem <= kLdsBytes, "fp64 forward: LDS");
  const int pol = policy_class(a.rule);
  auto kern = pol == 0 ? fwd_f64_kernel<D, 0, NW, TT>
                       : (pol == 1 ? fwd_f64_kernel<D, 1, NW, TT> : fwd_f64_kernel<D, 2, NW, TT>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  const int64_t nqb = (a.rule.q.n + bm_of<NW>() - 1) / bm_of<NW>();
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(thr_of<NW>()), smem, s, a);
  return hipGetLastError();
}

template <int D, int CH, int NCH>
hipError_t launch_dkdv_f64(const BwdArgs& a, hipStream_t s) {
  constexpr int NW = nw_of<D>(), TT = tt_of<D>();
  const int pol = policy_class(a.rule);
  auto kk = pol == 0 ? bwd_dkdv_f64_kernel<D, 0, TT, CH, NCH, NW>
                     : (pol == 1 ? bwd_dkdv_f64_kernel<D, 1, TT, CH, NCH, NW> : bwd_dkdv_f64_kernel<D, 2, TT, CH, NCH, NW>);
  constexpr int smem = bwd64_smem<D, TT, NW, Stream64<D, true, true, true, TT, NW>>();
  static_assert(smem <= kLdsBytes, "fp64 dK/dV: LDS");
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kk), smem);
  if (e != hipSuccess) return e;
  const int64_t nkb = (a.rule.k.n + bm_of<NW>() - 1) / bm_of<NW>();
  hipLaunchKernelGGL(kk, dim3((unsigned)(a.b * nkb)), dim3(thr_of<NW>()), smem, s, a);
  return hipGetLastError();
}

template <int D, int CH, int NCH>
hipError_t launch_dq_f64(const BwdArgs& a, hipStream_t s) {
  constexpr int NW = nw_of<D>(), TT = tt_of<D>();
  const int pol = policy_class(a.rule);
  auto kq = pol == 0 ? bwd_dq_f64_kernel<D, 0, TT, CH, NCH, NW>
                     : (pol == 1 ? bwd_dq_f64_kernel<D, 1, TT, CH, NCH, NW> : bwd_dq_f64_kernel<D, 2, TT, CH, NCH, NW>);
  constexpr int smem = bwd64_smem<D, TT, NW, Stream64<D, true, true, false, TT, NW>>();
  static_assert(smem <= kLdsBytes, "fp64 dQ: LDS");
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kq), smem);
  if (e != hipSuccess) return e;
  const int64_t nqb = (a.rule.q.n + bm_of<NW>() - 1) / bm_of<NW>();
  hipLaunchKernelGGL(kq, dim3((unsigned)(a.b * nqb)), dim3(thr_of<NW>()), smem, s, a);
  return hipGetLastError();
}

// channel chunks a launch holds: dK / dV all up to D = 64, halves at 128, quarters at 256 (the
// resident K', V operands take 2·D/4 doubles a lane); dQ all up to 128, halves at 256
template <int D>
hipError_t launch_bwd_t(const BwdArgs& a, hipStream_t s) {
  constexpr int NKV = D <= 64 ? 1 : (D <= 128 ? 2 : 4), NQ = D <= 128 ? 1 : 2;
  hipError_t e = launch_dkdv_f64<D, 0, NKV>(a, s);
  if constexpr (NKV > 1) {
    if (e == hipSuccess) e = launch_dkdv_f64<D, 1, NKV>(a, s);
  }
  if constexpr (NKV > 2) {
    if (e == hipSuccess) e = launch_dkdv_f64<D, 2, NKV>(a, s);
    if (e == hipSuccess) e = launch_dkdv_f64<D, 3, NKV>(a, s);
  }
  if (e == hipSuccess) e = launch_dq_f64<D, 0, NQ>(a, s);
  if constexpr (NQ > 1) {
    if (e == hipSuccess) e = launch_dq_f64<D, 1, NQ>(a, s);
  }
  return e;
}

}  // namespace

bool fwd_f64_supported(const FwdArgs& a) {
  return a.d >= 1 && a.v_d >= 1 && a.d <= 256 && a.v_d <= 256 && a.b * ((a.rule.q.n + 63) / 64) < (1ll << 31);
}

hipError_t launch_fwd_f64(const FwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_fwd_t<32>(a, s);
  if (dm <= 64) return launch_fwd_t<64>(a, s);
  if (dm <= 128) return launch_fwd_t<128>(a, s);
  return launch_fwd_t<256>(a, s);
}

// backward keeps K·scale, V (dkdv) or Q·scale, dO (dq) plus the dK/dV (dQ) accumulators in
// registers: 2·D/4 + 2·D/16·4 doubles per lane up to D = 64; past it the passes hold a channel chunk
// of their outputs per launch (launch_bwd_t)
bool bwd_f64_supported(const BwdArgs& a) {
  return a.d >= 1 && a.v_d >= 1 && a.d <= 256 && a.v_d <= 256 && a.b * ((a.rule.k.n + 63) / 64) < (1ll << 31) &&
         a.b * ((a.rule.q.n + 63) / 64) < (1ll << 31);
}

hipError_t launch_bwd_f64(const BwdArgs& a, hipStream_t s) {
  const int64_t nrows = a.b * (int64_t)a.rule.q.n;
  hipLaunchKernelGGL(bwd_prep_f64_kernel, dim3((unsigned)((nrows + kThrPrep - 1) / kThrPrep)), dim3(kThrPrep), 0, s,
                     a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_bwd_t<32>(a, s);
  if (dm <= 64) return launch_bwd_t<64>(a, s);
  if (dm <= 128) return launch_bwd_t<128>(a, s);
  return launch_bwd_t<256>(a, s);
}

}  // namespace fa
