// fa_generic.hip — dtype-generic fused attention kernels (fp16 / fp32 / fp64).
//
// These are the portable path: LDS-tiled, FMA-based, any policy / seq rank / sync
// mode, any channel count.  Up to MAXD channels (256 for fp16/fp32, 128 for fp64)
// Q / K / V stay resident in LDS per tile; past that the channel-chunked kernels
// below stream the channels in 32-row chunks (the reference sizes its key tile from
// shared memory instead and has no fixed channel cap, flash_attention.cu:1977-2067).
// They serve only shapes no MFMA kernel takes (d or v_d past 128, fp64 past 128).
//
// Algorithm (FA2 style, replacing the reference's FA1-style lock-serialised
// ForwardImpl/BackwardImpl, flash_attention.cu:425-1077 / 1079-1967):
//   forward : one workgroup per (batch slice, 32-query block); the key range is
//             bounded arithmetically by the rule (fa_rules.h), O/l/m live in
//             registers and are written exactly once — no inter-workgroup locks.
//   backward: prep kernel (D = rowsum(dO*O), lse = m + log l), one workgroup per
//             (batch slice, 32-key block) accumulating dK/dV in registers and dQ
//             through fp32/fp64 atomics into a workspace, then a cast kernel.
#include "fa_device.h"
#include "fa_kernels.h"

namespace fa {

namespace {

constexpr int kGBQ = 32;   // query rows per workgroup
constexpr int kGBK = 32;   // keys per tile
constexpr int kThreads = 256;

template <typename T, int MAXD>
__global__ __launch_bounds__(kThreads) void fwd_generic_kernel(FwdArgs a) {
  using A = typename AccOf<T>::type;
  using LT = typename LOf<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = a.d, vd = a.v_d;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  A* Qs = reinterpret_cast<A*>(smem);        // [d][BQ]
  A* Ks = Qs + d * kGBQ;                      // [d][BK]
  A* Vs = Ks + d * kGBK;                      // [vd][BK]
  A* Ps = Vs + vd * kGBK;                     // [BQ][BK+1]

  const uint32_t nqb = (nq + kGBQ - 1) / kGBQ;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (bid % nqb) * kGBQ;
  const int tid = threadIdx.x, r = tid >> 3, sub = tid & 7;

  const T* Q = static_cast<const T*>(a.Q) + bi * (int64_t)d * nq;
  const T* K = static_cast<const T*>(a.K) + bi * (int64_t)d * nk;
  const T* V = static_cast<const T*>(a.V) + bi * (int64_t)vd * nk;

  for (int idx = tid; idx < d * kGBQ; idx += kThreads) {
    const int c = idx / kGBQ, qq = idx % kGBQ;
    Qs[idx] = (q0 + qq < nq) ? to_acc<A>(Q[(int64_t)c * nq + q0 + qq]) : A(0);
  }

  const int qlast = min(q0 + kGBQ, nq) - 1;
  int kb, ke;
  k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);

  const int q = q0 + r;
  const bool qvalid = q < nq;
  const int qo = qvalid ? seq_order(a.rule.q, a.rule, q) : 0;
  const A scale = static_cast<A>(a.scale);

  A m_i = neg_inf<A>(), l_i = A(0);
  A o[MAXD / 8];
#pragma unroll
  for (int i = 0; i < MAXD / 8; ++i) o[i] = A(0);

  for (int k0 = kb; k0 < ke; k0 += kGBK) {
    __syncthreads();
    for (int idx = tid; idx < d * kGBK; idx += kThreads) {
      const int c = idx / kGBK, kk = idx % kGBK;
      Ks[idx] = (k0 + kk < ke) ? to_acc<A>(K[(int64_t)c * nk + k0 + kk]) : A(0);
    }
    for (int idx = tid; idx < vd * kGBK; idx += kThreads) {
      const int c = idx / kGBK, kk = idx % kGBK;
      Vs[idx] = (k0 + kk < ke) ? to_acc<A>(V[(int64_t)c * nk + k0 + kk]) : A(0);
    }
    __syncthreads();

    A s[4];
    A mt = neg_inf<A>();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kk = sub + 8 * j, k = k0 + kk;
      A acc = A(0);
      for (int c = 0; c < d; ++c) acc += Qs[c * kGBQ + r] * Ks[c * kGBK + kk];
      bool ok = qvalid && k < ke;
      if (ok && a.rule.policy != 0) ok = check_orders(a.rule, qo, seq_order(a.rule.k, a.rule, k));
      s[j] = ok ? acc * scale : neg_inf<A>();
      mt = max(mt, s[j]);
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) mt = max(mt, __shfl_xor(mt, off));
    const A m_new = max(m_i, mt);
    const A m_use = (m_new == neg_inf<A>()) ? A(0) : m_new;
    const A alpha = fa_exp(m_i - m_use);
    A ls = A(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const A p = fa_exp(s[j] - m_use);
      Ps[r * (kGBK + 1) + sub + 8 * j] = p;
      ls += p;
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) ls += __shfl_xor(ls, off);
    l_i = l_i * alpha + ls;
    m_i = m_new;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXD / 8; ++i) {
      const int v = sub + 8 * i;
      if (v < vd) {
        A acc = o[i] * alpha;
        for (int kk = 0; kk < kGBK; ++kk) acc += Ps[r * (kGBK + 1) + kk] * Vs[v * kGBK + kk];
        o[i] = acc;
      }
    }
  }

  if (!qvalid) return;
  T* O = static_cast<T*>(a.O) + bi * (int64_t)vd * nq;
  const bool any = l_i > A(0);
  const A inv = any ? A(1) / l_i : A(0);
#pragma unroll
  for (int i = 0; i < MAXD / 8; ++i) {
    const int v = sub + 8 * i;
    if (v < vd) O[(int64_t)v * nq + q] = from_acc<T>(o[i] * inv);
  }
  if (sub == 0) {
    LT* lo = static_cast<LT*>(a.l) + bi * (int64_t)nq;
    T* mo = static_cast<T*>(a.m) + bi * (int64_t)nq;
    if (any) {
      const T mt = from_acc<T>(m_i);
      // l is stored relative to the ROUNDED m so that exp(s - m)/l is exact
      // for the backward (SURVEY.md §7 hard part 4)
      lo[q] = static_cast<LT>(l_i * fa_exp(m_i - to_acc<A>(mt)));
      mo[q] = mt;
    } else {
      lo[q] = LT(0);
      mo[q] = neg_inf_approx<T>();
    }
  }
}

// D[q] = sum_v dO[v][q]*O[v][q];  lse[q] = m + log(l)  (+inf for rows attending nothing)
template <typename T>
__global__ __launch_bounds__(kThreads) void bwd_prep_kernel(BwdArgs a) {
  using A = typename AccOf<T>::type;
  using LT = typename LOf<T>::type;
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t total = a.b * (int64_t)nq;
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= total) return;
  const int64_t bi = i / nq;
  const int q = i % nq;
  const T* O = static_cast<const T*>(a.O) + bi * (int64_t)vd * nq + q;
  const T* dO = static_cast<const T*>(a.dO) + bi * (int64_t)vd * nq + q;
  A D = A(0);
  for (int v = 0; v < vd; ++v) D += to_acc<A>(O[(int64_t)v * nq]) * to_acc<A>(dO[(int64_t)v * nq]);
  const A l = static_cast<A>(static_cast<const LT*>(a.l)[i]);
  const A m = to_acc<A>(static_cast<const T*>(a.m)[i]);
  A* ws_D = static_cast<A*>(a.ws_D);
  A* ws_lse = static_cast<A*>(a.ws_lse);
  ws_D[i] = D;
  ws_lse[i] = (l > A(0)) ? m + fa_log(l) : pos_inf<A>();
}

template <typename T, int MAXD>
__global__ __launch_bounds__(kThreads) void bwd_generic_kernel(BwdArgs a) {
  using A = typename AccOf<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = a.d, vd = a.v_d;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  A* Ks = reinterpret_cast<A*>(smem);   // [d][32]
  A* Vs = Ks + d * kGBK;                // [vd][32]
  A* Qs = Vs + vd * kGBK;               // [d][32]
  A* dOs = Qs + d * kGBQ;               // [vd][32]
  A* Ps = dOs + vd * kGBQ;              // [32][33]
  A* dSs = Ps + kGBQ * (kGBK + 1);      // [32][33]
  A* lse_s = dSs + kGBQ * (kGBK + 1);   // [32]
  A* D_s = lse_s + kGBQ;                // [32]

  const uint32_t nkb = (nk + kGBK - 1) / kGBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (bid % nkb) * kGBK;
  const int tid = threadIdx.x, j = tid & 31, g = tid >> 5;

  const T* Q = static_cast<const T*>(a.Q) + bi * (int64_t)d * nq;
  const T* K = static_cast<const T*>(a.K) + bi * (int64_t)d * nk;
  const T* V = static_cast<const T*>(a.V) + bi * (int64_t)vd * nk;
  const T* dO = static_cast<const T*>(a.dO) + bi * (int64_t)vd * nq;
  const A* gD = static_cast<const A*>(a.ws_D) + bi * (int64_t)nq;
  const A* glse = static_cast<const A*>(a.ws_lse) + bi * (int64_t)nq;
  A* dQacc = static_cast<A*>(a.ws_dQ) + bi * (int64_t)d * nq;

  for (int idx = tid; idx < d * kGBK; idx += kThreads) {
    const int c = idx / kGBK, kk = idx % kGBK;
    Ks[idx] = (k0 + kk < nk) ? to_acc<A>(K[(int64_t)c * nk + k0 + kk]) : A(0);
  }
  for (int idx = tid; idx < vd * kGBK; idx += kThreads) {
    const int c = idx / kGBK, kk = idx % kGBK;
    Vs[idx] = (k0 + kk < nk) ? to_acc<A>(V[(int64_t)c * nk + k0 + kk]) : A(0);
  }
  const int klast = min(k0 + kGBK, nk) - 1;
  int qb, qe;
  q_range_for_k_block(a.rule, k0, klast, &qb, &qe);

  const int k = k0 + j;
  const bool kvalid = k < nk;
  const int ko = kvalid ? seq_order(a.rule.k, a.rule, k) : 0;
  const A scale = static_cast<A>(a.scale);

  A dk[MAXD / 8], dv[MAXD / 8];
#pragma unroll
  for (int i = 0; i < MAXD / 8; ++i) { dk[i] = A(0); dv[i] = A(0); }

  for (int q0 = qb; q0 < qe; q0 += kGBQ) {
    __syncthreads();
    for (int idx = tid; idx < d * kGBQ; idx += kThreads) {
      const int c = idx / kGBQ, qq = idx % kGBQ;
      Qs[idx] = (q0 + qq < qe) ? to_acc<A>(Q[(int64_t)c * nq + q0 + qq]) : A(0);
    }
    for (int idx = tid; idx < vd * kGBQ; idx += kThreads) {
      const int c = idx / kGBQ, qq = idx % kGBQ;
      dOs[idx] = (q0 + qq < qe) ? to_acc<A>(dO[(int64_t)c * nq + q0 + qq]) : A(0);
    }
    if (tid < kGBQ) {
      const bool v = q0 + tid < qe;
      lse_s[tid] = v ? glse[q0 + tid] : pos_inf<A>();
      D_s[tid] = v ? gD[q0 + tid] : A(0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qq = g + 8 * i, q = q0 + qq;
      A s = A(0), dp = A(0);
      for (int c = 0; c < d; ++c) s += Qs[c * kGBQ + qq] * Ks[c * kGBK + j];
      for (int v = 0; v < vd; ++v) dp += dOs[v * kGBQ + qq] * Vs[v * kGBK + j];
      bool ok = kvalid && q < qe;
      if (ok && a.rule.policy != 0) ok = check_orders(a.rule, seq_order(a.rule.q, a.rule, q), ko);
      const A p = ok ? fa_exp(s * scale - lse_s[qq]) : A(0);
      Ps[qq * (kGBK + 1) + j] = p;
      dSs[qq * (kGBK + 1) + j] = p * (dp - D_s[qq]) * scale;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXD / 8; ++i) {
      const int c = g + 8 * i;
      if (c < vd) {
        A acc = dv[i];
        for (int qq = 0; qq < kGBQ; ++qq) acc += Ps[qq * (kGBK + 1) + j] * dOs[c * kGBQ + qq];
        dv[i] = acc;
      }
      if (c < d) {
        A acc = dk[i];
        for (int qq = 0; qq < kGBQ; ++qq) acc += dSs[qq * (kGBK + 1) + j] * Qs[c * kGBQ + qq];
        dk[i] = acc;
      }
    }
    // dQ[c][q] += sum_j dS[q][j] * K[c][j]
    {
      const int qq = tid & 31, cg = tid >> 5, q = q0 + qq;
      if (q < qe) {
        for (int c = cg; c < d; c += 8) {
          A acc = A(0);
#pragma unroll 8
          for (int jj = 0; jj < kGBK; ++jj) acc += dSs[qq * (kGBK + 1) + jj] * Ks[c * kGBK + jj];
          atomicAdd(&dQacc[(int64_t)c * nq + q], acc);
        }
      }
    }
  }

  if (!kvalid) return;
  T* dK = static_cast<T*>(a.dK) + bi * (int64_t)d * nk;
  T* dV = static_cast<T*>(a.dV) + bi * (int64_t)vd * nk;
#pragma unroll
  for (int i = 0; i < MAXD / 8; ++i) {
    const int c = g + 8 * i;
    if (c < d) dK[(int64_t)c * nk + k] = from_acc<T>(dk[i]);
    if (c < vd) dV[(int64_t)c * nk + k] = from_acc<T>(dv[i]);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void cast_dq_kernel(const typename AccOf<T>::type* src, T* dst, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i < n) dst[i] = from_acc<T>(src[i]);
}

template <typename T, int MAXD>
hipError_t launch_fwd_generic_t(const FwdArgs& a, hipStream_t stream) {
  using A = typename AccOf<T>::type;
  const int nq = a.rule.q.n;
  const int64_t nqb = (nq + kGBQ - 1) / kGBQ;
  const size_t smem = sizeof(A) * ((size_t)a.d * kGBQ + (size_t)a.d * kGBK + (size_t)a.v_d * kGBK + kGBQ * (kGBK + 1));
  auto kern = fwd_generic_kernel<T, MAXD>;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kThreads), smem, stream, a);
  return hipGetLastError();
}

template <typename T, int MAXD>
hipError_t launch_bwd_generic_t(const BwdArgs& a, hipStream_t stream) {
  using A = typename AccOf<T>::type;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  hipError_t e = hipMemsetAsync(a.ws_dQ, 0, sizeof(A) * (size_t)a.b * a.d * nq, stream);
  if (e != hipSuccess) return e;
  const int64_t nrows = a.b * (int64_t)nq;
  hipLaunchKernelGGL(bwd_prep_kernel<T>, dim3((unsigned)((nrows + kThreads - 1) / kThreads)), dim3(kThreads), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t nkb = (nk + kGBK - 1) / kGBK;
  const size_t smem = sizeof(A) * ((size_t)(a.d + a.v_d) * kGBK + (size_t)(a.d + a.v_d) * kGBQ + 2 * kGBQ * (kGBK + 1) + 2 * kGBQ);
  auto kern = bwd_generic_kernel<T, MAXD>;
  e = set_smem_once(reinterpret_cast<const void*>(kern), (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(kThreads), smem, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = a.b * (int64_t)a.d * nq;
  hipLaunchKernelGGL(cast_dq_kernel<T>, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, stream,
                     static_cast<const A*>(a.ws_dQ), static_cast<T*>(a.dQ), n);
  return hipGetLastError();
}

// ---- channel-chunked kernels: any d, v_d (d or v_d past MAXD) ----
//
// forward: one workgroup per (slice, 32-query block, chunk of kVC output channels); the scores of
// a key tile are summed over 32-channel chunks of Q and K staged through LDS, so LDS use does not
// depend on d; every chunk's workgroup recomputes the scores (only for v_d past kVC), and the
// chunk-0 workgroup writes l and m.
constexpr int kDC = 32;  // channels per staged chunk
static_assert(kGBQ == kGBK, "the chunk loaders stage Q and K rows in one loop");

template <typename T> struct ChunkOf { static constexpr int kVC = 256; };
template <> struct ChunkOf<double> { static constexpr int kVC = 128; };

template <typename T>
__global__ __launch_bounds__(kThreads) void fwd_generic_ch_kernel(FwdArgs a, int nvc) {
  using A = typename AccOf<T>::type;
  using LT = typename LOf<T>::type;
  constexpr int kVC = ChunkOf<T>::kVC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = a.d, vd = a.v_d;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  A* Qc = reinterpret_cast<A*>(smem);  // [kDC][BQ]
  A* Kc = Qc + kDC * kGBQ;             // [kDC][BK]
  A* Vs = Kc + kDC * kGBK;             // [kVC][BK]
  A* Ps = Vs + kVC * kGBK;             // [BQ][BK+1]

  const uint32_t nqb = (nq + kGBQ - 1) / kGBQ;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int vc = bid % nvc;
  const int64_t bi = (bid / nvc) / nqb;
  const int q0 = ((bid / nvc) % nqb) * kGBQ;
  const int v0 = vc * kVC, v1 = min(vd, v0 + kVC);
  const int tid = threadIdx.x, r = tid >> 3, sub = tid & 7;

  const T* Q = static_cast<const T*>(a.Q) + bi * (int64_t)d * nq;
  const T* K = static_cast<const T*>(a.K) + bi * (int64_t)d * nk;
  const T* V = static_cast<const T*>(a.V) + bi * (int64_t)vd * nk;

  const int qlast = min(q0 + kGBQ, nq) - 1;
  int kb, ke;
  k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int q = q0 + r;
  const bool qvalid = q < nq;
  const int qo = qvalid ? seq_order(a.rule.q, a.rule, q) : 0;
  const A scale = static_cast<A>(a.scale);

  A m_i = neg_inf<A>(), l_i = A(0);
  A o[kVC / 8];
#pragma unroll
  for (int i = 0; i < kVC / 8; ++i) o[i] = A(0);

  for (int k0 = kb; k0 < ke; k0 += kGBK) {
    A acc[4] = {A(0), A(0), A(0), A(0)};
    for (int c0 = 0; c0 < d; c0 += kDC) {
      __syncthreads();
      for (int idx = tid; idx < kDC * kGBQ; idx += kThreads) {
        const int c = c0 + idx / kGBQ, qq = idx % kGBQ;
        Qc[idx] = (c < d && q0 + qq < nq) ? to_acc<A>(Q[(int64_t)c * nq + q0 + qq]) : A(0);
        const int kk = idx % kGBK;
        Kc[idx] = (c < d && k0 + kk < ke) ? to_acc<A>(K[(int64_t)c * nk + k0 + kk]) : A(0);
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = sub + 8 * j;
#pragma unroll 8
        for (int c = 0; c < kDC; ++c) acc[j] += Qc[c * kGBQ + r] * Kc[c * kGBK + kk];
      }
    }
    for (int idx = tid; idx < kVC * kGBK; idx += kThreads) {
      const int v = v0 + idx / kGBK, kk = idx % kGBK;
      Vs[idx] = (v < v1 && k0 + kk < ke) ? to_acc<A>(V[(int64_t)v * nk + k0 + kk]) : A(0);
    }
    A s[4];
    A mt = neg_inf<A>();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + sub + 8 * j;
      bool ok = qvalid && k < ke;
      if (ok && a.rule.policy != 0) ok = check_orders(a.rule, qo, seq_order(a.rule.k, a.rule, k));
      s[j] = ok ? acc[j] * scale : neg_inf<A>();
      mt = max(mt, s[j]);
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) mt = max(mt, __shfl_xor(mt, off));
    const A m_new = max(m_i, mt);
    const A m_use = (m_new == neg_inf<A>()) ? A(0) : m_new;
    const A alpha = fa_exp(m_i - m_use);
    A ls = A(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const A p = fa_exp(s[j] - m_use);
      Ps[r * (kGBK + 1) + sub + 8 * j] = p;
      ls += p;
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) ls += __shfl_xor(ls, off);
    l_i = l_i * alpha + ls;
    m_i = m_new;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kVC / 8; ++i) {
      const int v = v0 + sub + 8 * i;
      if (v < v1) {
        A acc2 = o[i] * alpha;
        for (int kk = 0; kk < kGBK; ++kk) acc2 += Ps[r * (kGBK + 1) + kk] * Vs[(v - v0) * kGBK + kk];
        o[i] = acc2;
      }
    }
  }

  if (!qvalid) return;
  T* O = static_cast<T*>(a.O) + bi * (int64_t)vd * nq;
  const bool any = l_i > A(0);
  const A inv = any ? A(1) / l_i : A(0);
#pragma unroll
  for (int i = 0; i < kVC / 8; ++i) {
    const int v = v0 + sub + 8 * i;
    if (v < v1) O[(int64_t)v * nq + q] = from_acc<T>(o[i] * inv);
  }
  if (sub == 0 && vc == 0) {
    LT* lo = static_cast<LT*>(a.l) + bi * (int64_t)nq;
    T* mo = static_cast<T*>(a.m) + bi * (int64_t)nq;
    if (any) {
      const T mt = from_acc<T>(m_i);
      lo[q] = static_cast<LT>(l_i * fa_exp(m_i - to_acc<A>(mt)));
      mo[q] = mt;
    } else {
      lo[q] = LT(0);
      mo[q] = neg_inf_approx<T>();
    }
  }
}

// backward: one workgroup per (slice, 32-key block, chunk of kVC output channels): S and dP of a
// query tile are summed over 32-channel chunks of Q / K and dO / V; the workgroup then
// accumulates dK and dV for its channel chunk and adds its chunk of dQ through atomics (the
// resident kernel's scheme, bwd_generic_kernel)
template <typename T>
__global__ __launch_bounds__(kThreads) void bwd_generic_ch_kernel(BwdArgs a, int noc) {
  using A = typename AccOf<T>::type;
  constexpr int kOC = ChunkOf<T>::kVC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = a.d, vd = a.v_d;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  A* Xq = reinterpret_cast<A*>(smem);  // [kDC][BQ] chunk of Q or dO
  A* Xk = Xq + kDC * kGBQ;             // [kDC][BK] chunk of K or V
  A* Qo = Xk + kDC * kGBK;             // [kOC][BQ] the output chunk's Q rows
  A* dOo = Qo + kOC * kGBQ;            // [kOC][BQ] ... dO rows
  A* Ko = dOo + kOC * kGBQ;            // [kOC][BK] ... K rows (for dQ; fixed per workgroup)
  A* Ps = Ko + kOC * kGBK;             // [BQ][BK+1]
  A* dSs = Ps + kGBQ * (kGBK + 1);     // [BQ][BK+1]
  A* lse_s = dSs + kGBQ * (kGBK + 1);  // [BQ]
  A* D_s = lse_s + kGBQ;               // [BQ]

  const uint32_t nkb = (nk + kGBK - 1) / kGBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int oc = bid % noc;
  const int64_t bi = (bid / noc) / nkb;
  const int k0 = ((bid / noc) % nkb) * kGBK;
  const int c0 = oc * kOC;
  const int tid = threadIdx.x, j = tid & 31, g = tid >> 5;

  const T* Q = static_cast<const T*>(a.Q) + bi * (int64_t)d * nq;
  const T* K = static_cast<const T*>(a.K) + bi * (int64_t)d * nk;
  const T* V = static_cast<const T*>(a.V) + bi * (int64_t)vd * nk;
  const T* dO = static_cast<const T*>(a.dO) + bi * (int64_t)vd * nq;
  const A* gD = static_cast<const A*>(a.ws_D) + bi * (int64_t)nq;
  const A* glse = static_cast<const A*>(a.ws_lse) + bi * (int64_t)nq;
  A* dQacc = static_cast<A*>(a.ws_dQ) + bi * (int64_t)d * nq;

  for (int idx = tid; idx < kOC * kGBK; idx += kThreads) {
    const int c = c0 + idx / kGBK, kk = idx % kGBK;
    Ko[idx] = (c < d && k0 + kk < nk) ? to_acc<A>(K[(int64_t)c * nk + k0 + kk]) : A(0);
  }
  const int klast = min(k0 + kGBK, nk) - 1;
  int qb, qe;
  q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int k = k0 + j;
  const bool kvalid = k < nk;
  const int ko = kvalid ? seq_order(a.rule.k, a.rule, k) : 0;
  const A scale = static_cast<A>(a.scale);

  A dk[kOC / 8], dv[kOC / 8];
#pragma unroll
  for (int i = 0; i < kOC / 8; ++i) { dk[i] = A(0); dv[i] = A(0); }

  for (int q0 = qb; q0 < qe; q0 += kGBQ) {
    // S = Q^T K and dP = dO^T V over channel chunks (thread: queries g + 8i, key j)
    A sacc[4] = {A(0), A(0), A(0), A(0)}, pacc[4] = {A(0), A(0), A(0), A(0)};
    for (int pass = 0; pass < 2; ++pass) {
      const int cn = pass == 0 ? d : vd;
      const T* Xg = pass == 0 ? Q : dO;
      const T* Yg = pass == 0 ? K : V;
      for (int cc = 0; cc < cn; cc += kDC) {
        __syncthreads();
        for (int idx = tid; idx < kDC * kGBQ; idx += kThreads) {
          const int c = cc + idx / kGBQ, qq = idx % kGBQ;
          Xq[idx] = (c < cn && q0 + qq < qe) ? to_acc<A>(Xg[(int64_t)c * nq + q0 + qq]) : A(0);
          const int kk = idx % kGBK;
          Xk[idx] = (c < cn && k0 + kk < nk) ? to_acc<A>(Yg[(int64_t)c * nk + k0 + kk]) : A(0);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = g + 8 * i;
          A t = A(0);
#pragma unroll 8
          for (int c = 0; c < kDC; ++c) t += Xq[c * kGBQ + qq] * Xk[c * kGBK + j];
          if (pass == 0) sacc[i] += t; else pacc[i] += t;
        }
      }
    }
    // the output chunk's Q / dO rows, the row constants
    for (int idx = tid; idx < kOC * kGBQ; idx += kThreads) {
      const int c = c0 + idx / kGBQ, qq = idx % kGBQ;
      const bool qin = q0 + qq < qe;
      Qo[idx] = (c < d && qin) ? to_acc<A>(Q[(int64_t)c * nq + q0 + qq]) : A(0);
      dOo[idx] = (c < vd && qin) ? to_acc<A>(dO[(int64_t)c * nq + q0 + qq]) : A(0);
    }
    if (tid < kGBQ) {
      const bool v = q0 + tid < qe;
      lse_s[tid] = v ? glse[q0 + tid] : pos_inf<A>();
      D_s[tid] = v ? gD[q0 + tid] : A(0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qq = g + 8 * i, q = q0 + qq;
      bool ok = kvalid && q < qe;
      if (ok && a.rule.policy != 0) ok = check_orders(a.rule, seq_order(a.rule.q, a.rule, q), ko);
      const A p = ok ? fa_exp(sacc[i] * scale - lse_s[qq]) : A(0);
      Ps[qq * (kGBK + 1) + j] = p;
      dSs[qq * (kGBK + 1) + j] = p * (pacc[i] - D_s[qq]) * scale;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kOC / 8; ++i) {
      const int cl = g + 8 * i, c = c0 + cl;
      if (c < vd) {
        A acc = dv[i];
        for (int qq = 0; qq < kGBQ; ++qq) acc += Ps[qq * (kGBK + 1) + j] * dOo[cl * kGBQ + qq];
        dv[i] = acc;
      }
      if (c < d) {
        A acc = dk[i];
        for (int qq = 0; qq < kGBQ; ++qq) acc += dSs[qq * (kGBK + 1) + j] * Qo[cl * kGBQ + qq];
        dk[i] = acc;
      }
    }
    {  // dQ[c][q] += sum_j dS[q][j] * K[c][j] for this chunk's channels
      const int qq = tid & 31, cg = tid >> 5, q = q0 + qq;
      if (q < qe) {
        for (int cl = cg; cl < kOC && c0 + cl < d; cl += 8) {
          A acc = A(0);
#pragma unroll 8
          for (int jj = 0; jj < kGBK; ++jj) acc += dSs[qq * (kGBK + 1) + jj] * Ko[cl * kGBK + jj];
          atomicAdd(&dQacc[(int64_t)(c0 + cl) * nq + q], acc);
        }
      }
    }
  }

  if (!kvalid) return;
  T* dK = static_cast<T*>(a.dK) + bi * (int64_t)d * nk;
  T* dV = static_cast<T*>(a.dV) + bi * (int64_t)vd * nk;
#pragma unroll
  for (int i = 0; i < kOC / 8; ++i) {
    const int c = c0 + g + 8 * i;
    if (c < d) dK[(int64_t)c * nk + k] = from_acc<T>(dk[i]);
    if (c < vd) dV[(int64_t)c * nk + k] = from_acc<T>(dv[i]);
  }
}

template <typename T>
hipError_t launch_fwd_generic_ch(const FwdArgs& a, hipStream_t stream) {
  using A = typename AccOf<T>::type;
  constexpr int kVC = ChunkOf<T>::kVC;
  const int64_t nqb = (a.rule.q.n + kGBQ - 1) / kGBQ;
  const int nvc = (a.v_d + kVC - 1) / kVC;
  const size_t smem = sizeof(A) * ((size_t)kDC * kGBQ + (size_t)kDC * kGBK + (size_t)kVC * kGBK + kGBQ * (kGBK + 1));
  if (a.b * nqb * nvc >= (int64_t(1) << 31)) return hipErrorInvalidConfiguration;  // grid.x range
  auto kern = fwd_generic_ch_kernel<T>;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb * nvc)), dim3(kThreads), smem, stream, a, nvc);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_bwd_generic_ch(const BwdArgs& a, hipStream_t stream) {
  using A = typename AccOf<T>::type;
  constexpr int kOC = ChunkOf<T>::kVC;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  hipError_t e = hipMemsetAsync(a.ws_dQ, 0, sizeof(A) * (size_t)a.b * a.d * nq, stream);
  if (e != hipSuccess) return e;
  const int64_t nrows = a.b * (int64_t)nq;
  hipLaunchKernelGGL(bwd_prep_kernel<T>, dim3((unsigned)((nrows + kThreads - 1) / kThreads)), dim3(kThreads), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t nkb = (nk + kGBK - 1) / kGBK;
  const int noc = (max(a.d, a.v_d) + kOC - 1) / kOC;
  if (a.b * nkb * noc >= (int64_t(1) << 31)) return hipErrorInvalidConfiguration;  // grid.x range
  const size_t smem = sizeof(A) * ((size_t)kDC * (kGBQ + kGBK) + (size_t)kOC * (2 * kGBQ + kGBK) + 2 * kGBQ * (kGBK + 1) +
                                   2 * kGBQ);
  auto kern = bwd_generic_ch_kernel<T>;
  e = set_smem_once(reinterpret_cast<const void*>(kern), (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb * noc)), dim3(kThreads), smem, stream, a, noc);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = a.b * (int64_t)a.d * nq;
  hipLaunchKernelGGL(cast_dq_kernel<T>, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, stream,
                     static_cast<const A*>(a.ws_dQ), static_cast<T*>(a.dQ), n);
  return hipGetLastError();
}

template <typename T>
hipError_t dispatch_fwd(const FwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_fwd_generic_t<T, 32>(a, s);
  if (dm <= 64) return launch_fwd_generic_t<T, 64>(a, s);
  if (dm <= 128) return launch_fwd_generic_t<T, 128>(a, s);
  if (dm <= ChunkOf<T>::kVC) return launch_fwd_generic_t<T, ChunkOf<T>::kVC>(a, s);
  return launch_fwd_generic_ch<T>(a, s);
}

template <typename T>
hipError_t dispatch_bwd(const BwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_bwd_generic_t<T, 32>(a, s);
  if (dm <= 64) return launch_bwd_generic_t<T, 64>(a, s);
  if (dm <= 128) return launch_bwd_generic_t<T, 128>(a, s);
  if (dm <= ChunkOf<T>::kVC) return launch_bwd_generic_t<T, ChunkOf<T>::kVC>(a, s);
  return launch_bwd_generic_ch<T>(a, s);
}

}  // namespace

hipError_t launch_fwd_generic(int dtype, const FwdArgs& a, hipStream_t s) {
  switch (dtype) {
    case 0: return dispatch_fwd<__half>(a, s);
    case 1: return dispatch_fwd<float>(a, s);
    default: return dispatch_fwd<double>(a, s);
  }
}

hipError_t launch_bwd_generic(int dtype, const BwdArgs& a, hipStream_t s) {
  switch (dtype) {
    case 0: return dispatch_bwd<__half>(a, s);
    case 1: return dispatch_bwd<float>(a, s);
    default: return dispatch_bwd<double>(a, s);
  }
}

// the channel-chunked kernels take any count; the cap only keeps a slice's channel rows (and the
// dQ workspace index) well inside the int32 / int64 ranges the kernels use.  Their work grows as
// d * max(d, v_d) / 256 (each chunk of output channels recomputes the full-d scores), so very wide
// shapes are correct but slow; a grid past 2^31 blocks is refused (hipErrorInvalidConfiguration)
// before the launch.
int generic_max_channels(int dtype) { return (void)dtype, 65536; }

}  // namespace fa
