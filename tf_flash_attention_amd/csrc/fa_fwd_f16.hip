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

#include <stdlib.h>

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

constexpr int kBN = 64;      // keys per tile
constexpr int kVPad = 2;     // V slab row padding, in 8-byte rows
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.f;  // log2 units (cdna_hip_programming.md T13)

// value of lane l^32 (v_permlane32_swap instead of an LDS bpermute)
__device__ __forceinline__ float xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// Structure flags (FA_FWD_VARIANT overrides the default for A/B timing runs)
constexpr int kFOcc3 = 4;        // ask for 3 waves/SIMD (VGPR <= 168)
constexpr int kFDot2 = 8;        // row sums of the fp16 P by v_dot2_f32_f16 (half the VALU ops)
constexpr int kFOcc1 = 16;       // one wave per SIMD: the whole 512-entry register file
constexpr int kFSched = 32;      // force a 1-MFMA/5-VALU interleave (sched_group_barrier)
// row sums on the matrix pipe: one more MFMA per PV k-step with an all-ones A operand (every row of
// its accumulator is the query's running sum), instead of v_dot2c on the VALU.  At d <= 32 a tile's
// 8 MFMAs leave the pipe idle two thirds of the time beside the softmax issue, so the 4 extra
// MFMAs are free and the 16 dot2c they replace are not
constexpr int kFMfmaSum = 64;

template <int D, int NW>
struct Smem {
  static constexpr int kBM = 32 * NW;               // query rows per workgroup
  static constexpr int kQRow = 2 * kBM;              // bytes per Q row
  static constexpr int kQ = D * kQRow;               // Q [D][BM] halfs
  static constexpr int kK = D * kBN * 2;             // K [D][64]  halfs, 128-B rows
  static constexpr int kV = 16 * (D + kVPad) * 8;    // V [16][D+pad][4] halfs
  static constexpr int kBuf = kK + kV;
  static constexpr int kNBuf = 3;                    // K/V ring: tile t (V), t+1 (K), t+2 (being written)
  static constexpr int kTotal = (kNBuf * kBuf > kQ) ? kNBuf * kBuf : kQ;  // Q aliases the ring
};

constexpr int waves_per_eu(int D, int F) { return (D >= 128 || (F & kFOcc1)) ? 1 : ((F & kFOcc3) ? 3 : 2); }

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

// One workgroup = NW waves = 32*NW query rows of one (batch, head) slice.
//   POL  0: full policy (no rule mask; only the nk tail is masked)
//        1: interval rules (causal, 1d unit-stride local): each query's allowed keys
//           are an index interval [klo, khi]; the tile class is two scalar compares
//           against the wave's bounds and the mixed-tile mask one unsigned compare
//        2: other local rules (2d, strided): tile_class + per-element rule check
//   Tiles with no allowed pair for a wave are skipped by that wave (no MFMAs).
//   FAST d == v_d == D and K/V rows 16-byte aligned (nk % 8 == 0): unguarded
//        dwordx4 staging.
// Scores are produced directly as exp2 arguments: Q is pre-scaled by
// scale*log2(e) once (fp16), and the running max enters each Sᵀ MFMA chain as
// its C operand (-m broadcast), so P = exp2(acc) needs no per-element FMA.
// Software pipeline (one barrier per key tile, 3-slot LDS ring): while the
// softmax of tile j runs on the VALU, the Sᵀ MFMAs of tile j+1 are already in
// the matrix pipe, and the PV MFMAs of tile j follow (cdna_hip_programming.md
// T15); the K/V tile j+2 is written to LDS after the barrier and tile j+3 is
// loaded into registers (T14).
template <int D, int NW, int POL, bool FAST, int F>
__global__ __launch_bounds__(NW * 64, waves_per_eu(D, F)) void fwd_f16_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = Smem<D, NW>;
  constexpr int kThr = NW * 64;
  constexpr int kBM = S::kBM;
  constexpr int kChunks = D * 8;                                   // 16-B chunks per K (or V) tile
  constexpr int kCPT = (kChunks + kThr - 1) / kThr;                // chunks per thread
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n, d = FAST ? D : a.d, vd = FAST ? D : a.v_d;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;  // tr-read lane roles

  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;

  // ---- key range of this query block (rule-bounded)
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;

  // ---- register staging of one K/V tile (16-B chunks; chunk = 8 keys of one channel row)
  auto load_into = [&](u32x4 (&kr)[kCPT], u32x4 (&vr)[kCPT], int k0) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = tid + kThr * j, c = idx >> 3, m = idx & 7;
      const bool in = (kChunks % kThr == 0) || idx < kChunks;
      const int e = k0 + 8 * m;
      if (FAST && (kChunks % kThr == 0) && k0 + kBN <= nk) {  // whole tile in range: unguarded
        kr[j] = load16(K + (int64_t)c * nk + e);
        vr[j] = load16(V + (int64_t)c * nk + e);
      } else if (FAST) {
        kr[j] = (in && e < nk) ? load16(K + (int64_t)c * nk + e) : u32x4{0, 0, 0, 0};
        vr[j] = (in && e < nk) ? load16(V + (int64_t)c * nk + e) : u32x4{0, 0, 0, 0};
      } else {
        kr[j] = (in && c < d) ? load_chunk(K + (int64_t)c * nk, e, nk, false) : u32x4{0, 0, 0, 0};
        vr[j] = (in && c < vd) ? load_chunk(V + (int64_t)c * nk, e, nk, false) : u32x4{0, 0, 0, 0};
      }
    }
  };
  auto store_from = [&](const u32x4 (&kr)[kCPT], const u32x4 (&vr)[kCPT], int buf) {
    lds_char_t* kbuf = smem + buf * S::kBuf;
    lds_char_t* vbuf = kbuf + S::kK;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const int idx = tid + kThr * j, c = idx >> 3, m = idx & 7;
      if ((kChunks % kThr == 0) || idx < kChunks) {
        // K: [c][64 keys], 64-B halves swapped on rows with c&2 (conflict-free tr reads)
        *reinterpret_cast<lds_u32x4_t*>(kbuf + c * 128 + ((m * 16) ^ ((c & 2) << 5))) = kr[j];
        // V: [key/4][v][4] slabs -> the PV operand is a plain conflict-free ds_read_b64
        *reinterpret_cast<lds_u32x2_t*>(vbuf + ((2 * m) * (D + kVPad) + c) * 8) = vr[j].xy;
        *reinterpret_cast<lds_u32x2_t*>(vbuf + ((2 * m + 1) * (D + kVPad) + c) * 8) = vr[j].zw;
      }
    }
  };
  // prologue loads of tiles 0 and 1 are in flight together with the Q tile
  u32x4 kreg[kCPT], vreg[kCPT], kreg1[kCPT], vreg1[kCPT];
  if (ntiles > 0) load_into(kreg, vreg, kt0);
  if (ntiles > 1) load_into(kreg1, vreg1, kt0 + kBN);

  // ---- Q tile [D][BM] -> LDS (64-B blocks XOR-swizzled by c&3: conflict-free tr reads)
  for (int idx = tid; idx < D * (kBM / 8); idx += kThr) {
    const int c = idx / (kBM / 8), m = idx % (kBM / 8);
    u32x4 v = {0, 0, 0, 0};
    if (c < d) v = load_chunk(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec);
    *reinterpret_cast<lds_u32x4_t*>(smem + c * S::kQRow + ((m * 16) ^ ((c & 3) << 6))) = v;
  }
  __syncthreads();
  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + j][q = 32w + r]
  half8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
      const int col = 32 * w + 16 * (g & 1) + 4 * tp;
      const half4 t = tr_read(smem, crow * S::kQRow + ((col * 2) ^ ((crow & 3) << 6)));
      if (e == 0) qf[s].lo = t; else qf[s].hi = t;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = (_Float16)((float)qf[s][j] * c2);
  }
  __syncthreads();  // the Q region is reused by the K/V ring

  const int wq0 = q0 + 32 * w;
  const int wq1 = min(wq0 + 31, nq - 1);
  const bool wave_active = wq0 < nq;
  const int qi = wq0 + r;
  const int qo = (POL == 2 && qi < nq) ? seq_order(a.rule.q, a.rule, qi) : 0;
  // POL 1 (interval rules): this lane's allowed keys [klo, klo + kspan) and the wave's
  // bounds on them (both ends are non-decreasing in the query, so lanes 0 / last bound them)
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
  // tile class for this wave: 0 no allowed pair (skipped), 1 mixed (per-element mask), 2 all
  auto tcls = [&](int k0) -> int {
    const int k1 = k0 + kBN - 1;
    if (!wave_active) return 0;
    if (POL == 0) return k1 < nk ? 2 : 1;
    if (POL == 1) {
      if (wlo_min > k1 || whi_max < k0) return 0;
      return (wlo_max <= k0 && whi_min >= k1) ? 2 : 1;
    }
    const int c = tile_class(a.rule, wq0, wq1, k0, min(k1, nk - 1));
    return (c == 2 && k1 >= nk) ? 1 : c;
  };

  auto load_tile = [&](int k0) { load_into(kreg, vreg, k0); };
  auto store_tile = [&](int buf) { store_from(kreg, vreg, buf); };

  floatx16 acc_o[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_o[u][i] = 0.f;
  // m_run: lazily updated softmax reference (log2 units) that l_run / acc_o are relative
  // to; negm = -m_run broadcast (the C operand of every Sᵀ chain); m_max: exact row max.
  float m_run = 0.f, l_run = 0.f, m_max = kNegInf;
  bool m_set = false;
  constexpr bool MSUM = (F & kFMfmaSum) != 0;
  floatx16 acc_l;  // MSUM: the running row sum in every register (rows are identical)
#pragma unroll
  for (int i = 0; i < 16; ++i) acc_l[i] = 0.f;
  floatx16 negm;
#pragma unroll
  for (int i = 0; i < 16; ++i) negm[i] = 0.f;

  // Sᵀ - m of one tile (both 32-key halves), K fragments streamed from ring slot `buf`
  auto qk = [&](int buf, floatx16 (&st)[2]) {
    const lds_char_t* kbuf = smem + buf * S::kBuf;
#pragma unroll
    for (int t = 0; t < 2; ++t)
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
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], s == 0 ? negm : st[t], 0, 0, 0);
      }
  };

  // Rule/tail mask, row max and (lazy) rebase of the scores of tile `it` (after
  // this, exp2(st) are the tile's probabilities relative to m_run).
  auto prepare = [&](int it, int cls, floatx16 (&st)[2], floatx16 (&nxt)[2], bool has_next) {
    const int k0 = kt0 + it * kBN;
    if (cls == 1) {  // mixed / tail tile: per-element mask
      const int base = k0 + 4 * h - klo;
#pragma unroll
      for (int t = 0; t < 2; ++t)
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
    {  // v_max3 chains (2 new values per instruction), two independent chains
      float mx0 = fmaxf(st[0][0], st[0][1]), mx1 = fmaxf(st[1][0], st[1][1]);
#pragma unroll
      for (int i = 2; i < 16; i += 2) {
        mx0 = fmaxf(fmaxf(mx0, st[0][i]), st[0][i + 1]);
        mx1 = fmaxf(fmaxf(mx1, st[1][i]), st[1][i + 1]);
      }
      mt = fmaxf(mx0, mx1);
      mt = fmaxf(mt, xor32(mt));  // tile row max relative to m_run
    }
    m_max = fmaxf(m_max, m_run + mt);
    // lazy rescale (cdna_hip_programming.md T13): move m_run only when the tile max
    // exceeds it by more than kRescaleThr (P <= 2^kRescaleThr), or to seed it
    const bool seed = !m_set && (mt != kNegInf);
    if (__any((mt > kRescaleThr) | seed)) {
      const float delta = m_set ? fmaxf(mt, 0.f) : (seed ? mt : 0.f);
      const float alpha = m_set ? __builtin_amdgcn_exp2f(-delta) : 1.f;
      m_run += delta;
      m_set = m_set || seed;
      l_run *= alpha;
      if constexpr (MSUM) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc_l[i] *= alpha;
      }
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc_o[u][i] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[0][i] -= delta;
        st[1][i] -= delta;
        negm[i] = -m_run;
      }
      if (has_next) {  // the next tile's in-flight scores were formed against the old m_run
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          nxt[0][i] -= delta;
          nxt[1][i] -= delta;
        }
      }
    }
  };

  // P = exp2(st) (fp16) as the B operand of Oᵀ = V·Pᵀ (k-step s = registers 8(s&1).. of
  // half s>>1), row sums, and the PV MFMAs
  auto exp_pv = [&](floatx16 (&st)[2], int buf) {
    const lds_char_t* vbuf = smem + buf * S::kBuf + S::kK;
    typedef _Float16 half2v __attribute__((ext_vector_type(2)));
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = (_Float16)__builtin_amdgcn_exp2f(st[s >> 1][8 * (s & 1) + j]);
      if constexpr (MSUM) {
        half8 ones;
#pragma unroll
        for (int j = 0; j < 8; ++j) ones[j] = (_Float16)1.f;
        acc_l = __builtin_amdgcn_mfma_f32_32x32x16_f16(ones, pf, acc_l, 0, 0, 0);
      } else if (F & kFDot2) {
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          ls0 = __builtin_amdgcn_fdot2(half2v{pf[j], pf[j + 1]}, one2, ls0, false);
          ls1 = __builtin_amdgcn_fdot2(half2v{pf[j + 2], pf[j + 3]}, one2, ls1, false);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          ls0 += (float)pf[j];
          ls1 += (float)pf[j + 1];
        }
      }
#pragma unroll
      for (int u = 0; u < D / 32; ++u) {
        half8 vf;
        vf.lo = read_b64(vbuf, ((4 * s + h) * (D + kVPad) + 32 * u + r) * 8);
        vf.hi = read_b64(vbuf, ((4 * s + 2 + h) * (D + kVPad) + 32 * u + r) * 8);
        acc_o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf, acc_o[u], 0, 0, 0);
      }
    }
    l_run += ls0 + ls1;
  };

  // ---- prologue: tiles 0, 1 in the ring, tile 2 in registers, tile 0 scored
  floatx16 stA[2], stB[2];
  if (ntiles > 0) {
    store_tile(0);
    if (ntiles > 1) store_from(kreg1, vreg1, 1);
    if (ntiles > 2) load_tile(kt0 + 2 * kBN);
    __syncthreads();
    if (tcls(kt0) != 0) qk(0, stA);
  }
  // iteration it: ring slot it%3 holds tile it (V read now), slot (it+1)%3 tile it+1
  // (K read now), slot (it+2)%3 receives tile it+2.  One branch-free region per
  // iteration interleaves the Sᵀ MFMAs of tile it+1 and the PV MFMAs of tile it
  // with the exp/convert/row-sum VALU of tile it.
  int slot = 0;
  auto step = [&](int it, floatx16 (&cur)[2], floatx16 (&nxt)[2]) {
    const int s1 = (slot == 2) ? 0 : slot + 1;
    const int s2 = (s1 == 2) ? 0 : s1 + 1;
    if (it > 0) __syncthreads();  // tile it+1 complete; slot s2 (tile it-1) free
    if (it + 2 < ntiles) {
      store_tile(s2);
      if (it + 3 < ntiles) load_tile(kt0 + (it + 3) * kBN);
    }
    const int ccur = tcls(kt0 + it * kBN);
    const int cnxt = it + 1 < ntiles ? tcls(kt0 + (it + 1) * kBN) : 0;
    if (cnxt != 0) qk(s1, nxt);   // Sᵀ MFMAs of tile it+1 enter the matrix pipe first
    if (ccur != 0) {              // tiles without an allowed pair for this wave are skipped
      prepare(it, ccur, cur, nxt, cnxt != 0);
      exp_pv(cur, slot);
    }
    if (F & kFSched) {  // MFMA / VALU interleave for the region (cdna_hip_programming.md T19)
#pragma unroll
      for (int i = 0; i < 2 * (D / 16) + 4 * (D / 32); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x2, 5, 0);   // then up to 5 VALU
      }
    }
    slot = s1;
  };
  for (int it = 0; it < ntiles; it += 2) {
    step(it, stA, stB);
    if (it + 1 < ntiles) step(it + 1, stB, stA);
  }

  if (!wave_active) return;
  const float l_tot = MSUM ? acc_l[0] : l_run + xor32(l_run);
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi < nq) {
    __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (FAST || v < vd) O[(int64_t)v * nq + qi] = __float2half(acc_o[u][i] * inv);
      }
    if (h == 0) {
      float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
      __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
      if (l_tot > 0.f) {
        const __half mT = __float2half(m_max * kLn2);
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

template <int D, int NW, int F>
hipError_t launch_t(const FwdArgs& a, hipStream_t s) {
  using S = Smem<D, NW>;
  const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
  const int smem = S::kTotal;
  const bool fast = a.d == D && a.v_d == D && (a.rule.k.n % 8 == 0) &&
                    (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.V) % 16 == 0);
  const int pol = a.rule.policy == 0 ? 0 : (rule_is_interval(a.rule) ? 1 : 2);
  auto kern = pol == 0 ? (fast ? fwd_f16_kernel<D, NW, 0, true, F> : fwd_f16_kernel<D, NW, 0, false, F>)
            : pol == 1 ? (fast ? fwd_f16_kernel<D, NW, 1, true, F> : fwd_f16_kernel<D, NW, 1, false, F>)
                       : (fast ? fwd_f16_kernel<D, NW, 2, true, F> : fwd_f16_kernel<D, NW, 2, false, F>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(NW * 64), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool fwd_f16_supported(const FwdArgs& a) {
  if (fwd_f16_wide_supported(a)) return true;
  return a.d >= 1 && a.v_d >= 1 && a.d <= 128 && a.v_d <= 128 && a.b * ((a.rule.q.n + 127) / 128) < (1ll << 31);
}

hipError_t launch_fwd_f16(const FwdArgs& a, hipStream_t s) {
  const int dm = max(a.d, a.v_d);
  // 128 < max(d, v_d) <= 256, every rule and alignment: 256-channel MFMA tiles (fa_fwd_f16_wide.hip)
  if (dm > 128) return launch_fwd_f16_wide(a, s);
#ifdef FA_DIAG
  // FA_FWD_VARIANT = <NW><F> below 1000 pins this general kernel (A/B runs), e.g. 408
  const int v = diag_variant("FA_FWD_VARIANT");
  if (v >= 0 && v < 1000 && dm <= 32) {  // d <= 32: 308 dot2c row sums (the round-3 default), 372 MFMA row sums
    if (v == 308) return launch_t<32, 4, 8>(a, s);
    if (v == 372) return launch_t<32, 4, 8 | kFMfmaSum>(a, s);
    if (v == 808) return launch_t<32, 8, 8>(a, s);
    if (v == 872) return launch_t<32, 8, 8 | kFMfmaSum>(a, s);
  }
  if (v >= 0 && v < 1000 && dm > 32 && dm <= 64) {
    switch (v) {
      case 400: return launch_t<64, 4, 0>(a, s);
      case 408: return launch_t<64, 4, 8>(a, s);
      case 424: return launch_t<64, 4, 24>(a, s);
      case 456: return launch_t<64, 4, 56>(a, s);
      case 800: return launch_t<64, 8, 0>(a, s);
      case 808: return launch_t<64, 8, 8>(a, s);
      case 840: return launch_t<64, 8, 40>(a, s);
      default: break;
    }
  }
  const bool pinned = v >= 0 && v < 1000;
#else
  constexpr bool pinned = false;
#endif
  if (!pinned && fwd_f16_fast_supported(a)) return launch_fwd_f16_fast(a, s);
  if (dm <= 32) return launch_t<32, 4, 8>(a, s);
  if (dm <= 64) {
    // local bands: ~10 key tiles per block, so block prologue/epilogue matter;
    // 4-wave blocks let two blocks per CU cover each other's (c4: 5.2 vs 5.9 ms)
    if (a.rule.policy == 2) return launch_t<64, 4, 8>(a, s);
    return launch_t<64, 8, 8>(a, s);
  }
  return launch_t<128, 4, 8>(a, s);
}

}  // namespace fa
