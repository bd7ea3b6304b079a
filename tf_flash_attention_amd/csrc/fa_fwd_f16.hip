// fa_fwd_f16.hip — fp16 fused attention forward on gfx950 MFMA.
//
// Replaces the reference's ForwardImpl (flash_attention.cu:425-1077), which ran
// QKᵀ and PV as scalar SIMT FMAs with fp16 accumulation and serialised the
// O/l/m read-modify-write of every (query block, key block) pair through a
// global spin lock.  Here:
//   * one workgroup = 4 waves = 128 query rows of one (batch, head) slice;
//     the key loop runs inside the workgroup (FA2 order) so O, l, m live in
//     registers and are written exactly once — no locks, no memsets;
//   * Sᵀ = Kᵀ·Q and Oᵀ = V·Pᵀ on v_mfma_f32_32x32x16_f16 with fp32 accumulation.
//     Computing the TRANSPOSED scores puts the key index in the MFMA rows, so
//     (a) each lane owns one query column — the softmax row reductions are
//     in-register plus one cross-half exchange, and (b) the Sᵀ accumulator
//     is already the B operand of Oᵀ = V·Pᵀ (no LDS round trip for P), and
//     Oᵀ[v][q] comes out channel-first exactly as O is stored in HBM;
//   * the channel-first [c][n] tiles of Q and K are staged in LDS as stored
//     and read as k-contiguous MFMA operands with ds_read_b64_tr_b16
//     (hardware transpose); V goes to LDS as [key/4][v][4] slabs so its
//     operand reads are plain conflict-free ds_read_b64;
//   * masks are rules: per (wave, key tile) the tile is classified from the
//     order bounds (none / all / mixed) and only mixed tiles evaluate the
//     per-element rule (fa_rules.h); the key range of the block is bounded
//     arithmetically, so skipped tiles cost nothing (causal, local bands).
// Online softmax in the log2 domain (exp2 on v_exp_f32), fp32 statistics.
#include "fa_device.h"
#include "fa_kernels.h"

namespace fa {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((__vector_size__(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16_t;
typedef __attribute__((address_space(3))) char lds_char_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2_t;

constexpr int kBM = 128;     // query rows per workgroup (4 waves x 32)
constexpr int kBN = 64;      // keys per tile
constexpr int kVPad = 2;     // V slab row padding, in 8-byte rows
constexpr int kThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <int D>
struct Smem {
  static constexpr int kQ = D * kBM * 2;            // Q [D][128] halfs, 256-B rows
  static constexpr int kK = D * kBN * 2;            // K [D][64]  halfs, 128-B rows
  static constexpr int kV = 16 * (D + kVPad) * 8;   // V [16][D+pad][4] halfs
  static constexpr int kBuf = kK + kV;
  static constexpr int kTotal = (2 * kBuf > kQ) ? 2 * kBuf : kQ;  // Q aliases the K/V buffers
};

__device__ __forceinline__ half4 tr_read(const lds_char_t* base, uint32_t off) {
  const v4i16 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(base + off));
  return __builtin_bit_cast(half4, t);
}

__device__ __forceinline__ half4 read_b64(const lds_char_t* base, uint32_t off) {
  return *reinterpret_cast<const __attribute__((address_space(3))) half4*>(base + off);
}

__device__ __forceinline__ u32x4 load16(const __half* p) { return *reinterpret_cast<const u32x4*>(p); }

// 8 consecutive halfs starting at element `e` of a row of length n (zero past n).
__device__ __forceinline__ u32x4 load_chunk(const __half* row, int e, int n, bool vec) {
  if (vec) return (e < n) ? load16(row + e) : u32x4{0, 0, 0, 0};
  unsigned short h[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (e + j < n) ? __half_as_ushort(row[e + j]) : (unsigned short)0;
  return u32x4{h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16), h[4] | (uint32_t(h[5]) << 16),
               h[6] | (uint32_t(h[7]) << 16)};
}

// D=128 needs the whole 512-entry register file (one wave per SIMD)
template <int D>
__global__ __launch_bounds__(kThreads, (D >= 128 ? 1 : 2)) void fwd_f16_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = Smem<D>;

  const int nq = a.rule.q.n, nk = a.rule.k.n, d = a.d, vd = a.v_d;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;  // tr-read lane roles

  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const bool kvec = ((nk & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.K) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.V) & 15) == 0);

  // ---- Q tile [D][128] -> LDS (row c at c*256 B, 64-B blocks XOR-swizzled by c&3)
  for (int idx = tid; idx < D * 16; idx += kThreads) {
    const int c = idx >> 4, m = idx & 15;
    u32x4 v = {0, 0, 0, 0};
    if (c < d) v = load_chunk(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec);
    *reinterpret_cast<lds_u32x4_t*>(smem + c * 256 + ((m * 16) ^ ((c & 3) << 6))) = v;
  }
  __syncthreads();
  // Q as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + j][q = 32w + r]
  half8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
      const int col = 32 * w + 16 * (g & 1) + 4 * tp;
      const half4 t = tr_read(smem, crow * 256 + ((col * 2) ^ ((crow & 3) << 6)));
      if (e == 0) qf[s].lo = t; else qf[s].hi = t;
    }
  }
  __syncthreads();  // Q region is reused by the K/V buffers

  // ---- key range of this query block (rule-bounded) and per-lane query order
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb, ke;
  k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;
  const int wq0 = q0 + 32 * w;
  const int wq1 = min(wq0 + 31, nq - 1);
  const bool wave_active = wq0 < nq;
  const int qi = wq0 + r;
  const int qo = (qi < nq) ? seq_order(a.rule.q, a.rule, qi) : 0;
  const float scale2 = (float)a.scale * kLog2e;

  // ---- register staging of one K/V tile: D/32 16-byte chunks of each per thread
  u32x4 kreg[D / 32], vreg[D / 32];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int j = 0; j < D / 32; ++j) {
      const int idx = tid + kThreads * j, c = idx >> 3, m = idx & 7;
      kreg[j] = (c < d) ? load_chunk(K + (int64_t)c * nk, k0 + 8 * m, nk, kvec) : u32x4{0, 0, 0, 0};
      vreg[j] = (c < vd) ? load_chunk(V + (int64_t)c * nk, k0 + 8 * m, nk, kvec) : u32x4{0, 0, 0, 0};
    }
  };
  auto store_tile = [&](int buf) {
    lds_char_t* kbuf = smem + buf * S::kBuf;
    lds_char_t* vbuf = kbuf + S::kK;
#pragma unroll
    for (int j = 0; j < D / 32; ++j) {
      const int idx = tid + kThreads * j, c = idx >> 3, m = idx & 7;
      *reinterpret_cast<lds_u32x4_t*>(kbuf + c * 128 + ((m * 16) ^ ((c & 2) << 5))) = kreg[j];
      *reinterpret_cast<lds_u32x2_t*>(vbuf + ((2 * m) * (D + kVPad) + c) * 8) = vreg[j].xy;
      *reinterpret_cast<lds_u32x2_t*>(vbuf + ((2 * m + 1) * (D + kVPad) + c) * 8) = vreg[j].zw;
    }
  };

  floatx16 acc_o[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_o[u][i] = 0.f;
  float m_run = -__builtin_huge_valf(), l_run = 0.f;

  if (ntiles > 0) load_tile(kt0);
  for (int it = 0; it < ntiles; ++it) {
    const int k0 = kt0 + it * kBN;
    store_tile(it & 1);
    if (it + 1 < ntiles) load_tile(k0 + kBN);
    __syncthreads();

    int cls = 0;
    if (wave_active) cls = tile_class(a.rule, wq0, wq1, k0, min(k0 + kBN, nk) - 1);
    if (cls == 0) continue;
    const bool tail = k0 + kBN > nk;
    const lds_char_t* kbuf = smem + (it & 1) * S::kBuf;
    const lds_char_t* vbuf = kbuf + S::kK;

    // Sᵀ[key][q] for the two 32-key halves of the tile
    floatx16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) st[t][i] = 0.f;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        half8 kf;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
          const int col = 32 * t + 16 * (g & 1) + 4 * tp;
          const half4 x = tr_read(kbuf, crow * 128 + ((col * 2) ^ ((crow & 2) << 5)));
          if (e == 0) kf.lo = x; else kf.hi = x;
        }
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], st[t], 0, 0, 0);
      }
    }

    // scale to the log2 domain; rule mask on mixed / tail tiles
    float mt = -__builtin_huge_valf();
    if (cls == 1 || tail) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
          bool ok = key < nk && qi < nq;
          if (ok && cls == 1) ok = check_orders(a.rule, qo, seq_order(a.rule.k, a.rule, key));
          const float x = ok ? st[t][i] * scale2 : -__builtin_huge_valf();
          st[t][i] = x;
          mt = fmaxf(mt, x);
        }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float x = st[t][i] * scale2;
          st[t][i] = x;
          mt = fmaxf(mt, x);
        }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32));
    const float m_new = fmaxf(m_run, mt);
    const float m_use = (m_new == -__builtin_huge_valf()) ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc_o[u][i] *= alpha;

    // P (fp16) as the B operand of Oᵀ = V·Pᵀ: k-step s = registers 8(s&1).. of tile s>>1
    half8 pf[4];
    float ls = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(st[s >> 1][8 * (s & 1) + j] - m_use);
        ls += p;
        pf[s][j] = (_Float16)p;
      }
    l_run += ls;

    // Oᵀ[v][q] += V[v][key] Pᵀ[key][q]; V operand element j <- key 16s + 8(j>>2) + 4h + (j&3)
#pragma unroll
    for (int u = 0; u < D / 32; ++u) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        half8 vf;
        vf.lo = read_b64(vbuf, ((4 * s + h) * (D + kVPad) + 32 * u + r) * 8);
        vf.hi = read_b64(vbuf, ((4 * s + 2 + h) * (D + kVPad) + 32 * u + r) * 8);
        acc_o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[s], acc_o[u], 0, 0, 0);
      }
    }
  }

  if (!wave_active) return;
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi < nq) {
    __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (v < vd) O[(int64_t)v * nq + qi] = __float2half(acc_o[u][i] * inv);
      }
    if (h == 0) {
      float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
      __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
      if (l_tot > 0.f) {
        const __half mT = __float2half(m_run * kLn2);
        // l relative to the STORED (rounded) m, so exp(s - m)/l is exact downstream
        lo[qi] = l_tot * __builtin_amdgcn_exp2f(m_run - __half2float(mT) * kLog2e);
        mo[qi] = mT;
      } else {
        lo[qi] = 0.f;
        mo[qi] = neg_inf_approx<__half>();
      }
    }
  }
}

template <int D>
hipError_t launch_t(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const int smem = Smem<D>::kTotal;
  auto kern = fwd_f16_kernel<D>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kThreads), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool fwd_f16_supported(const FwdArgs& a) {
  return a.d >= 1 && a.v_d >= 1 && a.d <= 128 && a.v_d <= 128 && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16(const FwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  if (dm <= 32) return launch_t<32>(a, s);
  if (dm <= 64) return launch_t<64>(a, s);
  return launch_t<128>(a, s);
}

}  // namespace fa
