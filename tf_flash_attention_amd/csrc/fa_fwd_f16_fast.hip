// fa_fwd_f16_fast.hip — fp16 fused attention forward, streamlined main loop for
// the common shapes (d == v_d ∈ {64, 128}, K/V rows 16-byte aligned, nk % 8 == 0)
// under the full policy and the interval rules (causal, 1d unit-stride local).
//
// Same algorithm and operand layouts as fa_fwd_f16.hip (which remains the path
// for every other shape and for strided / 2d local rules); what differs is how
// the key loop is laid out for the gfx950 issue port:
//   * K and V have separate 2-slot LDS rings.  Iteration `it` reads K(it+1) (for
//     the Sᵀ MFMAs of the next tile) and V(it) (for this tile's PV MFMAs), and
//     writes K(it+2) / V(it+1) into the slots the previous iteration finished
//     with — one barrier per key tile, and the loop unrolled by two so every
//     LDS address is a lane constant plus an immediate;
//   * K/V tiles are fetched with buffer loads (one SGPR descriptor per slice,
//     the tile offset in soffset): no per-tile address VALU;
//   * all K and V fragment reads of a tile are issued together right after the
//     barrier, before any of the tile's VALU, so LDS latency overlaps the
//     softmax instead of serialising the MFMAs behind it;
//   * full tiles take a branch-free path; only mixed tiles (rule edge / nk tail)
//     evaluate a per-element mask.
// Replaces the reference's ForwardImpl (flash_attention.cu:425-1077) for these
// shapes; numerics (fp32 accumulation, lazy log2-domain rescale, l relative to
// the stored fp16 m) are identical to fa_fwd_f16.hip.
#include "fa_device.h"
#include "fa_kernels.h"

#include <stdlib.h>

namespace fa {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef short v4i16 __attribute__((__vector_size__(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16_t;
typedef __attribute__((address_space(3))) char lds_char_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2_t;

constexpr int kBN = 64;      // keys per tile
constexpr int kVPad = 1;     // V group row padding, in 16-byte rows
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.f;  // log2 units (cdna_hip_programming.md T13)

// structure flags (FA_FWD_VARIANT selects them for A/B timing; the launcher's default is tuned)
constexpr int kFSumAdd = 1;  // row sums by f32 adds of the exponentials (else v_dot2 on packed P)
constexpr int kFPrio = 2;    // s_setprio 1 for the second half of the waves (guide T5, static form)
constexpr int kFLateV = 4;   // read the V fragments after the rebase decision (shorter live range)
constexpr int kFOcc3 = 8;    // three waves per SIMD (<= 168 VGPRs)
constexpr int kFDeep = 16;   // two register sets for the K/V staging: global loads two tiles ahead
// ablation bits: timing-only diagnostic builds (outputs are WRONG), FA_FWD_VARIANT=1899 + FA_FWD_ABL
// kDiag: per-wave s_memtime sums of the loop phases written over the l output (diagnostic only)
constexpr int kDiag = 4096;
constexpr int kANoBar = 64, kANoExp = 128, kANoLoad = 256, kANoMax = 512, kANoQK = 1024, kANoPV = 2048;

template <int D, int NW>
struct FastSmem {
  static constexpr int kBM = 32 * NW;               // query rows per workgroup
  static constexpr int kQRow = 2 * kBM;             // bytes per Q row
  static constexpr int kQ = D * kQRow;              // Q [D][BM] halfs
  static constexpr int kK = D * kBN * 2;            // K tile [D][64] halfs, 128-B rows
  static constexpr int kV = 8 * (D + kVPad) * 16;   // V tile [8 groups][D+pad][8] halfs
  static constexpr int offK = kQ;                   // K slots 0, 1
  static constexpr int offV = kQ + 2 * kK;          // V slots 0, 1
  static constexpr int kTotal = kQ + 2 * kK + 2 * kV;
};

// max / sum of x over lanes l and l^32: after the half swap one result holds the
// lower half twice and the other the upper half twice, so a symmetric op of the
// two needs no lane select.
__device__ __forceinline__ float max_pair32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_pair32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ half4 tr_read(const lds_char_t* p) {
  const v4i16 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)p);
  return __builtin_bit_cast(half4, t);
}

__device__ __forceinline__ u32x4 load_chunk_q(const __half* row, int e, int n, bool vec) {
  if (vec) return (e < n) ? *reinterpret_cast<const u32x4*>(row + e) : u32x4{0, 0, 0, 0};
  unsigned short hh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) hh[j] = (e + j < n) ? __half_as_ushort(row[e + j]) : (unsigned short)0;
  return u32x4{hh[0] | (uint32_t(hh[1]) << 16), hh[2] | (uint32_t(hh[3]) << 16), hh[4] | (uint32_t(hh[5]) << 16),
               hh[6] | (uint32_t(hh[7]) << 16)};
}

// Buffer descriptor over `bytes` bytes at `p`, built from provably wave-uniform
// values (guide T20: no waterfall loops around the buffer ops).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int V>
struct IC {
  static constexpr int value = V;
};

// One workgroup = NW waves; each wave owns QB blocks of 32 queries of one (batch,
// head) slice and sweeps the key tiles its rule allows.  With QB = 2 a wave has
// two independent softmax streams sharing every K/V fragment read, and runs
// alone on its SIMD (the whole 512-entry register file), so the matrix work of
// one tile overlaps the vector work of the same wave instead of relying on a
// partner wave that reaches the same phase at the same time.
//   POL 0: full policy (only the nk tail tile is masked)
//       1: interval rules (causal, 1d unit-stride local): per-lane key interval,
//          tile class from the wave's bounds, skipped tiles cost nothing.
constexpr int fast_waves_per_eu(int D, int QB, int F) { return (D >= 128 || QB > 1) ? 1 : ((F & kFOcc3) ? 3 : 2); }

template <int D, int NW, int QB, int POL, int F>
__global__ __launch_bounds__(NW * 64, fast_waves_per_eu(D, QB, F)) void fwd_f16_fast_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = FastSmem<D, NW * QB>;
  constexpr int kThr = NW * 64;
  constexpr int kBM = S::kBM;
  constexpr int kChunks = D * 8;  // 16-B chunks per K (or V) tile
  static_assert(kChunks % kThr == 0, "tile chunks must divide over the workgroup");
  constexpr int kCPT = kChunks / kThr;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  if ((F & kFPrio) && w >= NW / 2) __builtin_amdgcn_s_setprio(1);

  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)D * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)D * nk, 2u * D * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)D * nk, 2u * D * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;

  // ---- key range of this query block (rule-bounded)
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;

  // ---- staging: chunk j of this thread = 8 keys of channel row c
  uint32_t voff[kCPT];
  uint32_t kwo[kCPT], vwo[kCPT];
  const int cm = tid & 7;  // chunk index within the 64-key row (same for every j)
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int c = (tid + kThr * j) >> 3;
    voff[j] = (uint32_t)c * (uint32_t)nk * 2u + 16u * cm;
    kwo[j] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));          // K: 64-B halves swapped on rows with c&2
    // V: group (s, h) = keys {16s + 4h + 0..3, 16s + 8 + 4h + 0..3}, [v][8 keys] rows, so one
    // ds_read_b128 is a PV A operand; chunk cm = keys 8cm..8cm+7 -> groups (cm/2, 0) and (cm/2, 1)
    vwo[j] = ((2 * (cm >> 1)) * (D + kVPad) + c) * 16 + (cm & 1) * 8;
  }
  constexpr int NSET = (F & kFDeep) ? 2 : 1;
  u32x4 kr[NSET][kCPT], vr[NSET][kCPT];
  auto load_into = [&](u32x4 (&dst)[kCPT], __amdgpu_buffer_rsrc_t rs, int k0) {
    if (k0 + kBN <= nk) {
#pragma unroll
      for (int j = 0; j < kCPT; ++j) dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[j], 2 * k0, 0);
    } else {  // nk tail: chunks past nk read as zeros (offset beyond the descriptor's range)
      const bool out = k0 + 8 * cm >= nk;
#pragma unroll
      for (int j = 0; j < kCPT; ++j)
        dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, out ? 0x80000000u : voff[j], 2 * k0, 0);
    }
  };
  auto store_k = [&](int slot, const u32x4 (&src)[kCPT]) {
    lds_char_t* kb_ = smem + S::offK + slot * S::kK;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) *reinterpret_cast<lds_u32x4_t*>(kb_ + kwo[j]) = src[j];
  };
  auto store_v = [&](int slot, const u32x4 (&src)[kCPT]) {
    lds_char_t* vb_ = smem + S::offV + slot * S::kV;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      *reinterpret_cast<lds_u32x2_t*>(vb_ + vwo[j]) = src[j].xy;
      *reinterpret_cast<lds_u32x2_t*>(vb_ + vwo[j] + (D + kVPad) * 16) = src[j].zw;
    }
  };

  // ---- prologue loads: K(0), V(0), K(1) in flight together with the Q tile
  u32x4 kr1[kCPT];
  if (ntiles > 0) { load_into(kr[0], krs, kt0); load_into(vr[0], vrs, kt0); }
  if (ntiles > 1) load_into(kr1, krs, kt0 + kBN);
  for (int idx = tid; idx < D * (kBM / 8); idx += kThr) {  // Q [D][BM], 64-B blocks XOR-swizzled by c&3
    const int c = idx / (kBM / 8), m = idx % (kBM / 8);
    const u32x4 v = load_chunk_q(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec);
    *reinterpret_cast<lds_u32x4_t*>(smem + c * S::kQRow + ((m * 16) ^ ((c & 3) << 6))) = v;
  }
  if (ntiles > 0) { store_k(0, kr[0]); store_v(0, vr[0]); }
  if (ntiles > 1) store_k(1, kr1);
  // register set x feeds the stores of iterations with parity x: K(it+2), V(it+1)
#pragma unroll
  for (int x = 0; x < NSET; ++x) {
    if (ntiles > 2 + x) load_into(kr[x], krs, kt0 + (2 + x) * kBN);
    if (ntiles > 1 + x) load_into(vr[x], vrs, kt0 + (1 + x) * kBN);
  }
  __syncthreads();

  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) of block j holds
  // Q[c = 16s + 8h + e][q = 32(QB*w + j) + r]
  half8 qf[QB][D / 16];
#pragma unroll
  for (int j = 0; j < QB; ++j)
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * (QB * w + j) + 16 * (g & 1) + 4 * tp;
        const half4 t = tr_read(smem + crow * S::kQRow + ((col * 2) ^ ((crow & 3) << 6)));
        if (e == 0) qf[j][s].lo = t; else qf[j][s].hi = t;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[j][s][e] = (_Float16)((float)qf[j][s][e] * c2);
    }

  const int wq0 = q0 + 32 * QB * w;
  const bool wave_active = wq0 < nq;
  // POL 1: each lane's allowed keys [klo, klo + kspan) per block, and the wave's bounds on them
  // (both interval ends are non-decreasing in the query, so the first / last valid lane bound them)
  int klo[QB], kspan[QB];
  int wlo_min = 0, wlo_max = 0, whi_min = 0, whi_max = 0;
#pragma unroll
  for (int j = 0; j < QB; ++j) { klo[j] = 0; kspan[j] = 0; }
  if (POL == 1 && wave_active) {
    int khi[QB];
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      key_interval(a.rule, min(wq0 + 32 * j + r, nq - 1), &klo[j], &khi[j]);
      kspan[j] = max(khi[j] - klo[j] + 1, 0);
    }
    const int last = min(32 * QB - 1, nq - 1 - wq0);  // last valid query of the wave
    wlo_min = __builtin_amdgcn_readfirstlane(klo[0]);
    whi_min = __builtin_amdgcn_readfirstlane(khi[0]);
    int lo_last = klo[0], hi_last = khi[0];
#pragma unroll
    for (int j = 1; j < QB; ++j)
      if (last >= 32 * j) { lo_last = klo[j]; hi_last = khi[j]; }
    wlo_max = __builtin_amdgcn_readlane(lo_last, last & 31);
    whi_max = __builtin_amdgcn_readlane(hi_last, last & 31);
  }
  // tile class for this wave: 0 no allowed pair (skipped), 1 mixed (per-element mask), 2 all
  auto tcls = [&](int k0) -> int {
    const int k1 = k0 + kBN - 1;
    if (!wave_active) return 0;
    if (POL == 0) return (k1 < nk && wq0 + 32 * QB <= nq) ? 2 : 1;
    if (wlo_min > k1 || whi_max < k0) return 0;
    return (wlo_max <= k0 && whi_min >= k1 && k1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants; every read is base + immediate)
  //   K: element (crow, col) of [D][64] at crow*128 + ((2*col) ^ ((crow & 2) << 5)); crow&2 == tq&2
  const uint32_t kbase0 = (8 * (g >> 1) + tq) * 128 + (((16 * (g & 1) + 4 * tp) * 2) ^ ((tq & 2) << 5));
  const uint32_t kbase1 = (8 * (g >> 1) + tq) * 128 + (((32 + 16 * (g & 1) + 4 * tp) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r,h) reads group (s, h), channel row 32u + r
  const uint32_t vbase = (h * (D + kVPad) + r) * 16;

  floatx16 acc_o[QB][D / 32];
#pragma unroll
  for (int j = 0; j < QB; ++j)
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc_o[j][u][i] = 0.f;
  // m_run: lazily moved softmax reference (log2 units) that l_run / acc_o are relative to;
  // negm = -m_run broadcast (the C operand of every Sᵀ chain); m_max: exact row max.
  // thr: rescale trigger — -FLT_MAX until the lane's first allowed key seeds m_run, then
  // kRescaleThr, so the per-tile test is one compare.
  // pend: a rebase of tile it moved m_run after the Sᵀ MFMAs of tile it+1 were issued against
  // the old value; tile it+1 subtracts it when it becomes current (rare, keeps the in-flight
  // accumulators out of the rebase branch)
  float m_run[QB], l_run[QB], l_run2[QB], m_max[QB], thr[QB], pend[QB];
  floatx16 negm[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    m_run[j] = 0.f; l_run[j] = 0.f; l_run2[j] = 0.f; m_max[j] = kNegInf; thr[j] = -__FLT_MAX__; pend[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) negm[j][i] = 0.f;
  }

  auto read_k = [&](int slot, half8 (&kf)[2][D / 16]) {
    const lds_char_t* kb_ = smem + S::offK + slot * S::kK;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        kf[t][s].lo = tr_read(kb_ + (t ? kbase1 : kbase0) + (16 * s) * 128);
        kf[t][s].hi = tr_read(kb_ + (t ? kbase1 : kbase0) + (16 * s + 4) * 128);
      }
  };
  auto read_v = [&](int slot, half8 (&vf)[4][D / 32]) {
    const lds_char_t* vb_ = smem + S::offV + slot * S::kV + vbase;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
        vf[s][u] = *reinterpret_cast<const __attribute__((address_space(3))) half8*>(
            vb_ + ((2 * s) * (D + kVPad) + 32 * u) * 16);
  };
  auto qk = [&](const half8 (&kf)[2][D / 16], floatx16 (&st)[QB][2]) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int j = 0; j < QB; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          st[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qf[j][s], s == 0 ? negm[j] : st[j][t], 0, 0, 0);
  };
  // per-element rule / tail mask of a mixed tile
  auto mask = [&](int k0, floatx16 (&st)[QB][2]) {
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      const int base = k0 + 4 * h - klo[j];
      const bool qok = wq0 + 32 * j + r < nq;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = 32 * t + (i & 3) + 8 * (i >> 2);
          const bool ok = (POL == 1) ? ((unsigned)(base + off) < (unsigned)kspan[j]) : (qok && (k0 + off + 4 * h < nk));
          st[j][t][i] = ok ? st[j][t][i] : kNegInf;
        }
    }
  };
  // row max of tile `st` (lanes l and l^32 together) -> mt
  auto rowmax = [&](floatx16 (&st)[QB][2], float (&mt)[QB]) {
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      float mx0 = fmaxf(st[j][0][0], st[j][0][1]), mx1 = fmaxf(st[j][1][0], st[j][1][1]);
#pragma unroll
      for (int i = 2; i < 16; i += 2) {
        mx0 = fmaxf(fmaxf(mx0, st[j][0][i]), st[j][0][i + 1]);
        mx1 = fmaxf(fmaxf(mx1, st[j][1][i]), st[j][1][i + 1]);
      }
      mt[j] = (F & kANoMax) ? st[j][0][0] * 0.f : max_pair32(fmaxf(mx0, mx1));
      m_max[j] = fmaxf(m_max[j], m_run[j] + mt[j]);
    }
  };
  // lazy rebase (rare): after it exp2(st) are the tile's probabilities relative to m_run
  auto rebase = [&](const float (&mt)[QB], floatx16 (&st)[QB][2], bool has_next) {
    bool fire = false;
#pragma unroll
    for (int j = 0; j < QB; ++j) fire |= mt[j] > thr[j];
    if (__any(fire)) {  // rare: seed, or a tile max moved past the threshold
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const bool unset = thr[j] < 0.f;
        const bool seed = unset && (mt[j] > thr[j]);
        const float delta = unset ? (seed ? mt[j] : 0.f) : fmaxf(mt[j], 0.f);
        const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
        m_run[j] += delta;
        thr[j] = (unset && !seed) ? thr[j] : kRescaleThr;
        l_run[j] *= alpha;
        l_run2[j] *= alpha;
#pragma unroll
        for (int u = 0; u < D / 32; ++u)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc_o[j][u][i] *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          st[j][0][i] -= delta;
          st[j][1][i] -= delta;
          negm[j][i] = -m_run[j];
        }
        pend[j] = has_next ? delta : 0.f;  // the next tile's in-flight scores used the old m_run
      }
    }
  };
  // P = exp2(st) (fp16) as the B operand of Oᵀ = V·Pᵀ; row sums; PV MFMAs
  auto exp_pv = [&](floatx16 (&st)[QB][2], const half8 (&vf)[4][D / 32]) {
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        half8 pf;
        if (F & kFSumAdd) {
          float e[8];
#pragma unroll
          for (int x = 0; x < 8; ++x) e[x] = __builtin_amdgcn_exp2f(st[j][s >> 1][8 * (s & 1) + x]);
#pragma unroll
          for (int x = 0; x < 8; x += 2) {
            l_run[j] += e[x];
            l_run2[j] += e[x + 1];
          }
#pragma unroll
          for (int x = 0; x < 8; ++x) pf[x] = (_Float16)e[x];
        } else {
#pragma unroll
          for (int x = 0; x < 8; ++x) {
            const float sv = st[j][s >> 1][8 * (s & 1) + x];
            pf[x] = (_Float16)((F & kANoExp) ? sv : __builtin_amdgcn_exp2f(sv));
          }
#pragma unroll
          for (int x = 0; x < 8; x += 4) {
            l_run[j] = __builtin_amdgcn_fdot2(half2v{pf[x], pf[x + 1]}, one2, l_run[j], false);
            l_run2[j] = __builtin_amdgcn_fdot2(half2v{pf[x + 2], pf[x + 3]}, one2, l_run2[j], false);
          }
        }
#pragma unroll
        for (int u = 0; u < D / 32; ++u) {
          if (F & kANoPV) acc_o[j][u][0] += (float)pf[u] + (float)vf[s][u][0];
          else acc_o[j][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], pf, acc_o[j][u], 0, 0, 0);
        }
      }
  };

  // ---- S(0)
  floatx16 stA[QB][2], stB[QB][2];
  if (ntiles > 0 && tcls(kt0) != 0) {
    half8 kf[2][D / 16];
    read_k(0, kf);
    qk(kf, stA);
  }

  // iteration it: K(it+1) in slot (it+1)&1, V(it) in slot it&1 (both complete after the barrier);
  // K(it+2) -> slot it&1 and V(it+1) -> slot (it+1)&1 (both finished with in iteration it-1).
  // Order: [mask(it) if mixed] [Sᵀ MFMAs of it+1 beside the row max of it] [rare rebase]
  //        [exp2 / convert / row sums of it beside its PV MFMAs]
  uint64_t dsum[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = 0;
  auto stamp = [&]() -> uint64_t {
    uint64_t t = 0;
    if (F & kDiag) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    return t;
  };
  auto step = [&](auto P_, int it, floatx16 (&cur)[QB][2], floatx16 (&nxt)[QB][2]) {
    constexpr int p = decltype(P_)::value;  // it & 1
    const uint64_t t0 = stamp();
    if (!(F & kANoBar)) __syncthreads();
    const uint64_t t1 = stamp();
    const int k0 = kt0 + it * kBN;
    const int ccur = tcls(k0);
    const bool has_next = it + 1 < ntiles;
    const int cnxt = has_next ? tcls(k0 + kBN) : 0;
    half8 kf[2][D / 16];
    half8 vf[4][D / 32];
    if (cnxt != 0) read_k(p ^ 1, kf);
    if (ccur != 0 && !(F & kFLateV)) read_v(p, vf);
    const uint64_t ta = stamp();
    constexpr int rs = (NSET == 2) ? p : 0;
    if (it + 2 < ntiles) store_k(p, kr[rs]);
    if (has_next) store_v(p ^ 1, vr[rs]);
    const uint64_t tb = stamp();
    if (!(F & kANoLoad)) {
      if (it + 2 + NSET < ntiles) load_into(kr[rs], krs, k0 + (2 + NSET) * kBN);
      if (it + 1 + NSET < ntiles) load_into(vr[rs], vrs, k0 + (1 + NSET) * kBN);
    }
    bool adj = false;
#pragma unroll
    for (int j = 0; j < QB; ++j) adj |= pend[j] != 0.f;
    if (__any(adj)) {  // rare: this tile's scores predate the last rebase
#pragma unroll
      for (int j = 0; j < QB; ++j) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          cur[j][0][i] -= pend[j];
          cur[j][1][i] -= pend[j];
        }
        pend[j] = 0.f;
      }
    }
    if (ccur == 1) mask(k0, cur);
    const uint64_t t2 = stamp();
    float mt[QB];
    if (cnxt != 0 && ccur != 0) {  // one basic block: next tile's MFMAs beside this tile's max
      if (!(F & kANoQK)) qk(kf, nxt);
      rowmax(cur, mt);
    } else {
      if (cnxt != 0 && !(F & kANoQK)) qk(kf, nxt);
      if (ccur != 0) rowmax(cur, mt);
    }
    const uint64_t t3 = stamp();
    if (ccur != 0) {
      rebase(mt, cur, cnxt != 0);
      if (F & kFLateV) read_v(p, vf);
      exp_pv(cur, vf);
    }
    const uint64_t t4 = stamp();
    if (F & kDiag) {
      dsum[0] += t1 - t0; dsum[1] += t2 - tb; dsum[5] += ta - t1; dsum[6] += tb - ta; dsum[2] += t3 - t2; dsum[3] += t4 - t3;
      if (tprev) dsum[4] += t0 - tprev;
      tprev = t4;
    }
  };
  for (int it = 0; it < ntiles; it += 2) {
    step(IC<0>{}, it, stA, stB);
    if (it + 1 < ntiles) step(IC<1>{}, it + 1, stB, stA);
  }

  if (F & kDiag) {  // barrier, reads+stores+loads+mask, QK+max, rebase+exp+PV, loop overhead
    if (lane == 0 && wave_active)
      for (int x = 0; x < 7; ++x) static_cast<float*>(a.l)[bi * (int64_t)nq + wq0 + x] = (float)dsum[x];
    return;
  }
  if (!wave_active) return;
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int qi = wq0 + 32 * j + r;
    const float l_tot = sum_pair32(l_run[j] + l_run2[j]);
    const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
    if (qi < nq) {
      __half* O = static_cast<__half*>(a.O) + bi * (int64_t)D * nq;
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          O[(int64_t)v * nq + qi] = __float2half(acc_o[j][u][i] * inv);
        }
      if (h == 0) {
        float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
        __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
        if (l_tot > 0.f) {
          const __half mT = __float2half(m_max[j] * kLn2);
          // l relative to the STORED (rounded) m, so exp(s - m)/l is exact downstream
          lo[qi] = l_tot * __builtin_amdgcn_exp2f(m_run[j] - __half2float(mT) * kLog2e);
          mo[qi] = mT;
        } else {
          lo[qi] = 0.f;
          mo[qi] = neg_inf_approx<__half>();
        }
      }
    }
  }
}

template <int D, int NW, int QB, int F>
hipError_t launch_fast_t(const FwdArgs& a, hipStream_t s) {
  using S = FastSmem<D, NW * QB>;
  const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
  const int smem = S::kTotal;
  auto kern = a.rule.policy == 0 ? fwd_f16_fast_kernel<D, NW, QB, 0, F> : fwd_f16_fast_kernel<D, NW, QB, 1, F>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(NW * 64), smem, s, a);
  return hipGetLastError();
}

int fast_variant() {
  const char* e = getenv("FA_FWD_VARIANT");
  return e ? atoi(e) : -1;
}

}  // namespace

bool fwd_f16_fast_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  return a.d == a.v_d && (a.d == 64 || a.d == 128) && (nk % 8 == 0) && nk > 0 &&
         (int64_t)a.d * nk * 2 < (1ll << 31) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) && rule_is_interval(a.rule) &&
         a.b * ((a.rule.q.n + 127) / 128) < (1ll << 31);
}

hipError_t launch_fwd_f16_fast(const FwdArgs& a, hipStream_t s) {
  // FA_FWD_VARIANT = 1<NW><QB><F>: e.g. 1420 = 4 waves x 2 query blocks, flags 0
  const int v = fast_variant();
  if (a.d == 64 && v == 1899) {  // ablations (timing only)
    const char* e = getenv("FA_FWD_ABL");
    switch (e ? atoi(e) : 0) {
      case 64: return launch_fast_t<64, 4, 2, 4 | 64>(a, s);
      case 128: return launch_fast_t<64, 4, 2, 4 | 128>(a, s);
      case 256: return launch_fast_t<64, 4, 2, 4 | 256>(a, s);
      case 512: return launch_fast_t<64, 4, 2, 4 | 512>(a, s);
      case 1024: return launch_fast_t<64, 4, 2, 4 | 1024>(a, s);
      case 2048: return launch_fast_t<64, 4, 2, 4 | 2048>(a, s);
      case 640: return launch_fast_t<64, 4, 2, 4 | 128 | 512>(a, s);
      case 3072: return launch_fast_t<64, 4, 2, 4 | 1024 | 2048>(a, s);
      case 4096: return launch_fast_t<64, 8, 1, 2 | 4096>(a, s);
      case 4100: return launch_fast_t<64, 8, 1, 6 | 4096>(a, s);
      case 4116: return launch_fast_t<64, 8, 1, 22 | 4096>(a, s);
      default: return launch_fast_t<64, 4, 2, 4>(a, s);
    }
  }
  if (a.d == 64) {
    switch (v) {
      case 1810: return launch_fast_t<64, 8, 1, 0>(a, s);
      case 1812: return launch_fast_t<64, 8, 1, 2>(a, s);
      case 1410: return launch_fast_t<64, 4, 1, 0>(a, s);
      case 1418: return launch_fast_t<64, 4, 1, 8>(a, s);
      case 1412: return launch_fast_t<64, 4, 1, 2>(a, s);
      case 1414: return launch_fast_t<64, 4, 1, 4>(a, s);
      case 1416: return launch_fast_t<64, 4, 1, 6>(a, s);
      case 1814: return launch_fast_t<64, 8, 1, 4>(a, s);
      case 1830: return launch_fast_t<64, 8, 1, 20>(a, s);
      case 1832: return launch_fast_t<64, 8, 1, 22>(a, s);
      case 1430: return launch_fast_t<64, 4, 1, 20>(a, s);
      case 1816: return launch_fast_t<64, 8, 1, 6>(a, s);
      case 1419: return launch_fast_t<64, 4, 1, 12>(a, s);
      case 14110: return launch_fast_t<64, 4, 1, 10>(a, s);
      case 1420: return launch_fast_t<64, 4, 2, 0>(a, s);
      case 1421: return launch_fast_t<64, 4, 2, 1>(a, s);
      case 1220: return launch_fast_t<64, 2, 2, 0>(a, s);
      case 1820: return launch_fast_t<64, 8, 2, 4>(a, s);
      case 1425: return launch_fast_t<64, 4, 2, 5>(a, s);
      case 1426: return launch_fast_t<64, 4, 2, 6>(a, s);
      case 1424: return launch_fast_t<64, 4, 2, 4>(a, s);
      // tuned (c2, MI355X): 8 waves x 32 queries, static priority for waves 4-7, late V reads
      default: return launch_fast_t<64, 8, 1, kFPrio | kFLateV>(a, s);
    }
  }
  switch (v) {
    case 1411: return launch_fast_t<128, 4, 1, 1>(a, s);
    case 1412: return launch_fast_t<128, 4, 1, 2>(a, s);
    case 1414: return launch_fast_t<128, 4, 1, 4>(a, s);
    case 1416: return launch_fast_t<128, 4, 1, 6>(a, s);
    case 1810: return launch_fast_t<128, 8, 1, 0>(a, s);
    case 1814: return launch_fast_t<128, 8, 1, 4>(a, s);
    case 1410: return launch_fast_t<128, 4, 1, 0>(a, s);
    // tuned (c3 forward, MI355X): 4 waves (one per SIMD), static priority, late V reads
    default: return launch_fast_t<128, 4, 1, kFPrio | kFLateV>(a, s);
  }
}

}  // namespace fa
