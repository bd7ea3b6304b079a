// fa_bwd_f16_fast.hip — fp16 fused attention backward on gfx950 MFMA for every rule
// (full, causal, local in 1d/2d with any stride) and max(d, v_d) <= 128 (channels
// zero-padded to D ∈ {64, 128}).  Rows whose 16-B chunks are aligned (16-B aligned
// tensors, nq % 8 == nk % 8 == 0) stage with one 16-B buffer load per chunk; any other
// length or alignment (ALN = false) loads the same chunks element by element.
//
// Replaces the reference's BackwardImpl (flash_attention.cu:1079-1967), which ran
// every (key block, query block) pair as scalar SIMT GEMMs and serialised the dQ
// read-modify-write through a global spin lock.  Here the pass is split the way
// the data wants to flow on this chip — no atomics, no locks, no dQ workspace:
//   prep : -D = -rowsum(dO∘O), -lse2 = -(m·log2e + log2 l)            (per query, negated:
//          the C operands of the S / dP chains)
//   dkdv : key-outer.  A wave owns 32 keys; K·scale·log2e and V stay in registers
//          as MFMA B operands, dK and dV accumulate in registers, and the query
//          tiles (Q, dO, lse2, D) stream through a 2-slot LDS ring:
//              S  = Qᵀ·K'  (C = -lse2)   P  = exp2(S)
//              dP = dOᵀ·V  (C = -D)      dS = P∘dP
//              dV += dO·P,  dK += Q·dS   (P, dS straight from the accumulators)
//   dq   : query-outer, the forward's structure.  A wave owns 32 queries; Q' and
//          dO stay in registers as B operands and the key tiles stream through LDS:
//              Sᵀ = Kᵀ·Q' (C = -lse2)    dPᵀ = Vᵀ·dO (C = -D)
//              dQ += K·(Pᵀ∘dPᵀ)
// The dq pass recomputes Sᵀ and dPᵀ (4d of the 14d MFMA FLOPs per allowed pair
// against the algorithmic 10d) in exchange for writing dQ exactly once; the
// single-kernel alternative (fa_bwd_f16.hip) spends that in fp32 atomics, which
// cap it at ≈ 1.3 TB/s of added bytes (MI355X_MICROARCH.md 'Global float atomics').
// Masks are rules (fa_rules.h): per-lane index intervals (POL 1: full windows of an
// interval rule) or the per-element order check (POL 2: strided / 2d local windows), and
// per-wave tile classes; tiles with no allowed pair are skipped.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

#include <stdlib.h>

namespace fa {
namespace {

using namespace mf;

constexpr int kThrPrep = 256;

// ---------------------------------------------------------------------------
// prep: -D = -rowsum(dO∘O) (fp32), -lse2 = -(m*log2e + log2(l)) (-inf if the row attends nothing),
// stored negated: both passes start their S / dP accumulator chains from them
__global__ __launch_bounds__(kThrPrep) void bwd_prep_kernel(BwdArgs a) {
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t total = a.b * (int64_t)nq;
  const int64_t i = blockIdx.x * (int64_t)kThrPrep + threadIdx.x;
  if (i >= total) return;
  const int64_t bi = i / nq;
  const int q = (int)(i - bi * nq);
  const __half* O = static_cast<const __half*>(a.O) + bi * (int64_t)vd * nq + q;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq + q;
  float D0 = 0.f, D1 = 0.f;
  int v = 0;
  for (; v + 1 < vd; v += 2) {
    D0 += __half2float(O[(int64_t)v * nq]) * __half2float(dO[(int64_t)v * nq]);
    D1 += __half2float(O[(int64_t)(v + 1) * nq]) * __half2float(dO[(int64_t)(v + 1) * nq]);
  }
  if (v < vd) D0 += __half2float(O[(int64_t)v * nq]) * __half2float(dO[(int64_t)v * nq]);
  const float l = static_cast<const float*>(a.l)[i];
  const float m = __half2float(static_cast<const __half*>(a.m)[i]);
  static_cast<float*>(a.ws_D)[i] = -(D0 + D1);
  static_cast<float*>(a.ws_lse)[i] = (l > 0.f) ? -(m * kLog2e + __log2f(l)) : -__builtin_huge_valf();
}

// the same per query, eight consecutive queries a thread: one 16-B load per channel row and tensor
// instead of eight 2-B ones (O, dO 16-B aligned, nq % 8 == 0; the workspace is the library's own,
// 16-B aligned).  Each query's sums run in the same order as above, so -D and -lse2 are bitwise equal.
__global__ __launch_bounds__(kThrPrep) void bwd_prep8_kernel(BwdArgs a) {
  const int nq = a.rule.q.n, vd = a.v_d;
  const int64_t i0 = 8 * (blockIdx.x * (int64_t)kThrPrep + threadIdx.x);
  if (i0 >= a.b * (int64_t)nq) return;
  const int64_t bi = i0 / nq;
  const int q = (int)(i0 - bi * nq);
  const __half* O = static_cast<const __half*>(a.O) + bi * (int64_t)vd * nq + q;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq + q;
  float D0[8], D1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) D0[j] = D1[j] = 0.f;
  auto row = [&](const __half* p, int v) __attribute__((always_inline)) {
    return *reinterpret_cast<const half8*>(p + (int64_t)v * nq);
  };
  int v = 0;
#pragma unroll 2
  for (; v + 1 < vd; v += 2) {
    const half8 o0 = row(O, v), g0 = row(dO, v), o1 = row(O, v + 1), g1 = row(dO, v + 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      D0[j] += (float)o0[j] * (float)g0[j];
      D1[j] += (float)o1[j] * (float)g1[j];
    }
  }
  if (v < vd) {
    const half8 o0 = row(O, v), g0 = row(dO, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) D0[j] += (float)o0[j] * (float)g0[j];
  }
  const float* L = static_cast<const float*>(a.l) + i0;
  const __half* M = static_cast<const __half*>(a.m) + i0;
  floatx4 d[2], s[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float l = L[j], m = __half2float(M[j]);
    d[j >> 2][j & 3] = -(D0[j] + D1[j]);
    s[j >> 2][j & 3] = (l > 0.f) ? -(m * kLog2e + __log2f(l)) : -__builtin_huge_valf();
  }
  floatx4* wd = reinterpret_cast<floatx4*>(static_cast<float*>(a.ws_D) + i0);
  floatx4* ws = reinterpret_cast<floatx4*>(static_cast<float*>(a.ws_lse) + i0);
  wd[0] = d[0];
  wd[1] = d[1];
  ws[0] = s[0];
  ws[1] = s[1];
}

// ---------------------------------------------------------------------------
// LDS images
//   "row image"  [D][W] fp16, W = 32*NW columns, 16-B chunks XOR-swizzled by (row & 3) << 6
//                (B-operand transposed reads conflict-free; the forward's Q tile)
// "Q16 image" [D][32] fp16, 64-B rows, 16-B units XOR-swizzled by (row >> 2) & 3: one ds_write_b128
// per staged chunk; conflict-free transposed reads (rows q = 0..3 of a 4-row block fill the four
// 64-B quarters of the bank window) and conflict-free b128 row reads (16 lanes = 16 rows).
// Byte offset of the 8-B half `half8` of unit u (8 queries 8u..8u+7) of row `row`.
__device__ __forceinline__ uint32_t q16_off(int row, int u, int half8 = 0) {
  return row * 64 + 16 * (u ^ ((row >> 2) & 3)) + 8 * half8;
}
// "K2 image" [D][64] fp16, 128-B rows, 16-B chunk j at position j ^ (4·bit1(row) + bits2..3(row)):
// conflict-free for the σ-permuted transposed reads (a 4-row block's rows 0/2 and 1/3 land in
// opposite 64-B halves) AND for b128 row reads (16 consecutive rows hit 16 distinct 16-B slots),
// so one image serves as Kᵀ (Sᵀ = Kᵀ·Q') and as K (dQ += K·dSᵀ).
__device__ __forceinline__ uint32_t k2_off(int row, int j, int half8 = 0) {
  return row * 128 + 16 * (j ^ (4 * ((row >> 1) & 1) + ((row >> 2) & 3))) + 8 * half8;
}
template <int D, int NW, int NS = 2>
struct DkdvSmem {
  static constexpr int kBK = 32 * NW;                 // keys per workgroup
  static constexpr int kRow = D * kBK * 2;            // K (or V) row image
  static constexpr int kQT = D * 64;                  // one [D][32] QT image
  static constexpr int offQT = 0, offOT = kQT, offLse = 2 * kQT;
  static constexpr int kSlot = offLse + 2 * 32 * 4;   // + lse2[32], D[32]
  static constexpr int kRing = NS * kSlot;
  static constexpr int kTotal = (kRing > 2 * kRow) ? kRing : 2 * kRow;  // the K/V images alias the ring
};

// ---------------------------------------------------------------------------
// dK / dV: key-outer.  One workgroup = NW waves x 32 keys of one (batch, head) slice (the d <= 64
// pass, two waves per SIMD; d = 128 runs the producer / consumer pass below).
// OC > 1 (128 < d <= 256): the workgroup accumulates dK / dV for one of OC chunks of D / OC output
// channels (chunk = block index mod OC), forming S and dP over all D channels as before: the 256-channel
// accumulators of both gradients would not fit one wave beside the resident K' and V (round 4's D = 256
// pass; the four-role pass below replaces it, FA_BWD_VARIANT=1421 keeps it for A/B).
template <int D, int NW, int WPE, int POL, bool ALN, int OC = 1>
__global__ __launch_bounds__(NW * 64, WPE) void bwd_dkdv_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = DkdvSmem<D, NW>;
  constexpr int kThr = NW * 64;
  constexpr int kBK = S::kBK;
  constexpr int kQChunks = D * 4;                     // 16-B chunks of one [D][32] tile
  static_assert((2 * kQChunks) % kThr == 0, "tile chunks must divide over the workgroup");
  constexpr int kCPT = 2 * kQChunks / kThr;           // Q and dO chunks per thread

  constexpr int kDO = D / OC;                         // output channels of this workgroup
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bidc = xcd_remap(blockIdx.x, gridDim.x);
  const int oc = (int)(bidc % OC), ou0 = oc * (kDO / 32);  // the chunk: channel blocks ou0 .. ou0 + kDO/32 - 1
  const uint32_t bid = bidc / OC;
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;  // earliest (heaviest under causal) key blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  // transposed reads of the Q16 images supply query columns 4σ(p)..4σ(p)+3 (σ swaps 1 and 2), so
  // register i of S / dP holds query 16(i>>3) + 8h + (i&7): k-step s of P / dS is queries
  // 16s + 8h + 0..7, and the dV / dK A operands are plain 16-B row reads of the same images
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  const float c2 = (float)a.scale * kLog2e;

  // channels d (Q/K) and v_d (V/O) may be smaller than D: rows past them are staged as zeros
  const int d = a.d, vd = a.v_d;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq, 2u * d * nq);
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq, 2u * vd * nq);
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;

  // ---- resident B operands: lane (r,h) holds X[c = 16s + 8h + j][key = k0 + 32w + r]
  half8 kb[D / 16], vb[D / 16];
  {
    // every chunk of a thread loaded before any is stored, branch-free (chunks past the channel
    // count or nk read as zeros): a rolled load-store loop here serialised 2D/16 memory
    // latencies in every block's prologue
    constexpr int kRPT = 2 * D * (kBK / 8) / kThr, kHalf = D * (kBK / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBK / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t krs2 = make_rsrc(K, 2u * d * nk), vrs2 = make_rsrc(V, 2u * vd * nk);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      const bool in = c < (which ? vd : d) && k0 + 8 * m < nk;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? vrs2 : krs2,
                                                       in ? (uint32_t)c * (uint32_t)nk * 2u + 16u * m : 0x80000000u, 2 * k0, 0);
      else
        rv[jj] = buf_load8h(which ? vrs2 : krs2, (uint32_t)c * (uint32_t)nk * 2u, k0 + 8 * m, nk, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBK) + ((m * 16) ^ ((c & 3) << 6))) = rv[jj];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * w + 16 * (g & 1) + 4 * tp;
        const uint32_t off = crow * (2 * kBK) + ((col * 2) ^ ((crow & 3) << 6));
        const half4 x = tr_read(smem + off), y = tr_read(smem + S::kRow + off);
        if (e == 0) { kb[s].lo = x; vb[s].lo = y; } else { kb[s].hi = x; vb[s].hi = y; }
      }
#pragma unroll
    for (int s = 0; s < D / 16; ++s) kb[s] = scale8(kb[s], c2);  // S in log2 units straight out of the MFMA
    __syncthreads();  // the K/V images are reused by the ring
  }

  // ---- query range of this key block and the per-lane / per-wave query intervals
  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / 32) * 32;
  const int ntiles = (qe > qb) ? (qe - qt0 + 31) / 32 : 0;
  const int key = k0 + 32 * w + r;
  const int wk0 = k0 + 32 * w;
  const bool wave_active = wk0 < nk;
  const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;  // this lane's key order
  int qlo = 0, qspan = nq, wlo_min = 0, wlo_max = 0, whi_min = nq - 1, whi_max = nq - 1;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
    const int last = min(31, nk - 1 - wk0);
    wlo_min = __builtin_amdgcn_readfirstlane(qlo);
    whi_min = __builtin_amdgcn_readfirstlane(qhi);
    wlo_max = __builtin_amdgcn_readlane(qlo, last);
    whi_max = __builtin_amdgcn_readlane(qhi, last);
  }
  // 0: no allowed pair for this wave, 1: mixed (per-element mask), 2: all allowed
  auto tcls = [&](int qa) -> int {
    const int qz = qa + 31;
    if (!wave_active) return 0;
    if (POL == 0) return 2;  // q >= nq rows carry -lse2 = -inf -> P = 0; keys >= nk are never stored
    if (POL == 2) return qa < nq ? tile_class(a.rule, qa, min(qz, nq - 1), wk0, min(wk0 + 31, nk - 1)) : 0;
    if (wlo_min > qz || whi_max < qa) return 0;
    return (wlo_max <= qa && whi_min >= qz) ? 2 : 1;
  };

  // ---- query-tile staging (Q, dO chunks: 8 queries of one channel row)
  uint32_t voff[kCPT];
  int crow_[kCPT], cm_[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int idx = (tid + kThr * j) % kQChunks;
    crow_[j] = idx >> 2;
    cm_[j] = idx & 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nq * 2u + (ALN ? 16u * cm_[j] : 0u);  // (ALN: the chunk's; else the row's)
  }
  // two staging sets (tile t in set t&1): a tile is loaded two steps before it is stored
  u32x4 qr[2][kCPT];
  float lr[2] = {0.f, 0.f};
  // chunk j holds dO (else Q); compile-time when the chunks divide evenly over the threads
  auto is_o = [&](int j) -> bool {
    return (kQChunks % kThr == 0) ? (j >= kQChunks / kThr) : ((tid + kThr * j) >= kQChunks);
  };
  auto load_tile = [&](int qa, int set) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      if constexpr (ALN) {
        const bool out = qa + 8 * cm_[j] >= nq || crow_[j] >= (isO ? vd : d);
        qr[set][j] = buf_load16(isO ? ors : qrs, voff[j], 2 * qa, out);
      } else {
        qr[set][j] = buf_load8h(isO ? ors : qrs, voff[j], qa + 8 * cm_[j], nq, crow_[j] < (isO ? vd : d));
      }
    }
    if (w == 0) {  // lanes 0..31: lse2, 32..63: D (wave-uniform branch; clamped load, select past nq)
      const int q = qa + (lane & 31);
      const float v = (lane < 32 ? glse : gD)[min(q, nq - 1)];
      lr[set] = (q < nq) ? v : ((lane < 32) ? -__builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot, int set) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      lds_char_t* t = base + (isO ? S::offOT : S::offQT);
      *reinterpret_cast<lds_u32x4_t*>(t + q16_off(crow_[j], cm_[j])) = qr[set][j];
    }
    if (w == 0) reinterpret_cast<lds_f_t*>(base + S::offLse)[lane] = lr[set];
  };

  floatx16 dk[kDO / 32], dv[kDO / 32];
#pragma unroll
  for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dk[u][i] = 0.f; dv[u][i] = 0.f; }

  // row constants of the tile in `base` (stored negated) as initial accumulators: S: -lse2[q], dP: -D[q]
  auto init_acc = [&](const lds_char_t* base, floatx16& sacc, floatx16& pacc) {
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {  // registers 4gq..4gq+3 = queries 16(gq>>1) + 8h + 4(gq&1) + 0..3
      const int q4 = 16 * (gq >> 1) + 8 * h + 4 * (gq & 1);
      const floatx4 l4 = *reinterpret_cast<const lds_f4_t*>(base + S::offLse + 4 * q4);
      const floatx4 d4 = *reinterpret_cast<const lds_f4_t*>(base + S::offLse + 128 + 4 * q4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sacc[4 * gq + j] = l4[j];
        pacc[4 * gq + j] = d4[j];
      }
    }
  };
  // S = Qᵀ·K', dP = dOᵀ·V: A operands (row q, k = channel) by transposed reads
  auto sdp = [&](const lds_char_t* base, floatx16& sacc, floatx16& pacc) {
    constexpr int kAh = 0;
    half8 qa8[kAh + 1], oa8[kAh + 1];
    auto rd = [&](int s) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint32_t off = q16_off(16 * s + 8 * (g >> 1) + 4 * e + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
        const half4 x = tr_read(base + S::offQT + off), y = tr_read(base + S::offOT + off);
        if (e == 0) { qa8[s % (kAh + 1)].lo = x; oa8[s % (kAh + 1)].lo = y; }
        else { qa8[s % (kAh + 1)].hi = x; oa8[s % (kAh + 1)].hi = y; }
      }
    };
#pragma unroll
    for (int s = 0; s < kAh; ++s) rd(s);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      if (s + kAh < D / 16) rd(s + kAh);
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa8[s % (kAh + 1)], kb[s], sacc, 0, 0, 0);
      pacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa8[s % (kAh + 1)], vb[s], pacc, 0, 0, 0);
    }
  };
  // P = exp2(S), dS = P∘dP; k-step s of the dV / dK products = registers 8s..8s+7
  auto softmax_m = [&](const floatx16& sacc, const floatx16& pacc, int qa, bool masked, half8 (&pf)[2], half8 (&sf)[2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (POL == 1 && masked) {
        const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
        pv = ((unsigned)(q - qlo) < (unsigned)qspan) ? pv : 0.f;
      }
      if (POL == 2 && masked) {
        const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
        pv = (q < nq && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko)) ? pv : 0.f;
      }
      pf[i >> 3][i & 7] = (_Float16)pv;
      sf[i >> 3][i & 7] = (_Float16)(pv * pacc[i]);
    }
  };
  // the edge-tile mask as a real branch (see the producer / consumer pass)
  auto softmax = [&](const floatx16& sacc, const floatx16& pacc, int qa, int cls, half8 (&pf)[2], half8 (&sf)[2]) {
    if constexpr (POL == 0) {
      softmax_m(sacc, pacc, qa, cls == 1, pf, sf);
    } else if (cls == 1) {
      asm volatile("; edge tile" ::: );
      softmax_m(sacc, pacc, qa, true, pf, sf);
    } else {
      asm volatile("; interior tile" ::: );
      softmax_m(sacc, pacc, qa, false, pf, sf);
    }
  };
  // dV += dO·P, dK += Q·dS: A = X[row 32u + r][queries 16s + 8h + 0..7] (b128 reads of the Q16 images)
  auto dvdk = [&](const lds_char_t* base, const half8 (&pf)[2], const half8 (&sf)[2]) {
    constexpr int kU = kDO / 32, kN = 2 * kU, kAh = 0;
    half8 oa[kAh + 1], qa[kAh + 1];
    auto rd = [&](int n) __attribute__((always_inline)) {  // product n = kU·s + u
      const int s = n / kU, u = n % kU;
      oa[n % (kAh + 1)] = read_b128(base + S::offOT + q16_off(32 * (ou0 + u) + r, 2 * s + h));
      qa[n % (kAh + 1)] = read_b128(base + S::offQT + q16_off(32 * (ou0 + u) + r, 2 * s + h));
    };
#pragma unroll
    for (int n = 0; n < kAh; ++n) rd(n);
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      if (n + kAh < kN) rd(n + kAh);
      const int s = n / kU, u = n % kU;
      dv[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa[n % (kAh + 1)], pf[s], dv[u], 0, 0, 0);
      dk[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa[n % (kAh + 1)], sf[s], dk[u], 0, 0, 0);
    }
  };

  load_tile(qt0, 0);  // unconditional, as in the dQ pass
  store_tile(0, 0);
  load_tile(qt0 + 32, 1);
  load_tile(qt0 + 64, 0);

  // iteration it: tile it in slot it&1 (complete after the barrier); tile it+1 -> slot (it+1)&1
  // (read in iteration it-1, finished before this barrier) from staging set (it+1)&1, which then
  // takes tile it+3.  Loads and stores are unconditional (past the end they move zeros into
  // a slot nobody reads), so hipcc's vmcnt waits stay exact: a store waits only for the load
  // issued two steps earlier.
  auto step = [&](auto P_, int it) {
    constexpr int p = decltype(P_)::value;
    __syncthreads();
    const int qa = qt0 + 32 * it;
    store_tile(p ^ 1, p ^ 1);
    load_tile(qa + 96, p ^ 1);
    const int cls = it < ntiles ? tcls(qa) : 0;  // (the loop's last pair may end on a phantom step)
    if (cls == 0) return;
    const lds_char_t* base = smem + p * S::kSlot;
    floatx16 sacc, pacc;
    init_acc(base, sacc, pacc);
    sdp(base, sacc, pacc);
    half8 pf[2], sf[2];
    softmax(sacc, pacc, qa, cls, pf, sf);
    dvdk(base, pf, sf);
  };
  // whole pairs of steps: a conditional second step (it loads) made hipcc's vmcnt waits before the
  // staging stores drain every load in flight, the one issued a step earlier included
  for (int it = 0; it < ntiles; it += 2) {
    step(IC<0>{}, it);
    step(IC<1>{}, it + 1);
  }

  // ---- dK = scale·Σ dS·Q, dV: rows c = 32u + (i&3) + 8(i>>2) + 4h, column = this lane's key
  if (!wave_active || key >= nk) return;
  __half* dK = static_cast<__half*>(a.dK) + bi * (int64_t)d * nk;
  __half* dV = static_cast<__half*>(a.dV) + bi * (int64_t)vd * nk;
  const float sc = (float)a.scale;
  if (d == D && vd == D) {  // one buffer store per value, the row's offset in an SGPR (no per-store
                            // 64-bit address, compare or exec branch)
    const __amdgpu_buffer_rsrc_t krs_ = make_rsrc(dK, 2u * d * nk), vrs_ = make_rsrc(dV, 2u * vd * nk);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nk + (uint32_t)key);
#pragma unroll
    for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t so = 2u * (32u * (ou0 + u) + (i & 3) + 8u * (i >> 2)) * (uint32_t)nk;
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(dk[u][i] * sc)), krs_, vlane, so, 0);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)dv[u][i]), vrs_, vlane, so, 0);
      }
    return;
  }
#pragma unroll
  for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * (ou0 + u) + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dK[(int64_t)c * nk + key] = __float2half(dk[u][i] * sc);
      if (c < vd) dV[(int64_t)c * nk + key] = __float2half(dv[u][i]);
    }
}

// ---------------------------------------------------------------------------
// dK / dV, producer / consumer (two waves per SIMD).  Waves w and w+4 share a SIMD and the same
// 32 keys.  Wave w (producer) forms S = Qᵀ·K' and dP = dOᵀ·V for query tile i, P = exp2(S) and
// dS = P∘dP, and hands P and dS to wave w+4 through LDS; wave w+4 (consumer) accumulates
// dV += dO·P and dK += Q·dS for tile i-1.  The producer's softmax VALU runs beside the
// consumer's MFMAs on the shared SIMD (the one-wave-per-SIMD kernel above serialises them), and
// the register file splits along the data: K', V and the S / dP accumulators live in the
// producer, the dK / dV accumulators in the consumer, each role inside its own loop so neither
// carries the other's registers (under 256 each at D = 128).  Every step: one barrier, the
// staging of tile i+1 into the ring, the load of tile i+3.
template <int D>
struct PcSmem {
  static constexpr int kBK = 128;            // keys per workgroup: four producer waves x 32
  static constexpr int kRow = D * kBK * 2;   // K (or V) row image (prologue only)
  static constexpr int kQT = D * 64;         // one [D][32] Q16 image
  static constexpr int offQT = 0, offOT = kQT, offLse = 2 * kQT, offD = offLse + 256;
  static constexpr int kSlot = offLse + 2 * 64 * 4;  // + -lse2[32], -D[32] (64-float vectors: LDS-DMA lanes)
  static constexpr int kNS = 4;              // query-tile ring
  static constexpr int offX = kNS * kSlot;   // P / dS hand-over: 2 slots x 4 waves x 4 KB
  static constexpr int kXWave = 4096;
  static constexpr int kXSlot = 4 * kXWave;
  static constexpr int kUsed = offX + 2 * kXSlot;
  static constexpr int kTotal = kUsed > 2 * kRow ? kUsed : 2 * kRow;  // the K/V images alias the ring
};

template <int D, int POL, bool ALN>
__global__ __launch_bounds__(512, 1) void bwd_dkdv_pc_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = PcSmem<D>;
  constexpr int kThr = 512;
  constexpr int kBK = S::kBK;
  constexpr int kQChunks = D * 4;                 // 16-B chunks of one [D][32] tile
  static_assert((2 * kQChunks) % kThr == 0, "tile chunks must divide over the workgroup");
  constexpr int kCPT = 2 * kQChunks / kThr;       // Q and dO chunks per thread
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;  // earliest (heaviest under causal) key blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wl = w & 3;  // group 0 produces, group 1 consumes; wl: the key slice
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int sig = ((tp & 1) << 1) | (tp >> 1);  // (see the dK/dV kernel above: σ-permuted transposed reads)
  const float c2 = (float)a.scale * kLog2e;

  const int d = a.d, vd = a.v_d;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq, 2u * d * nq);
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq, 2u * vd * nq);
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;

  // ---- K, V blocks into LDS (every thread); the producers read their resident B operands below
  {
    constexpr int kRPT = 2 * D * (kBK / 8) / kThr, kHalf = D * (kBK / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBK / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t krs2 = make_rsrc(K, 2u * d * nk), vrs2 = make_rsrc(V, 2u * vd * nk);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      const bool in = c < (which ? vd : d) && k0 + 8 * m < nk;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? vrs2 : krs2,
                                                       in ? (uint32_t)c * (uint32_t)nk * 2u + 16u * m : 0x80000000u, 2 * k0, 0);
      else
        rv[jj] = buf_load8h(which ? vrs2 : krs2, (uint32_t)c * (uint32_t)nk * 2u, k0 + 8 * m, nk, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBK) + ((m * 16) ^ ((c & 3) << 6))) = rv[jj];
    }
  }
  __syncthreads();

  // ---- query range of this key block and the per-lane / per-wave query intervals (both roles)
  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / 32) * 32;
  const int ntiles = (qe > qb) ? (qe - qt0 + 31) / 32 : 0;
  const int key = k0 + 32 * wl + r;
  const int wk0 = k0 + 32 * wl;
  const bool wave_active = wk0 < nk;
  int qlo = 0, qspan = nq, wlo_min = 0, wlo_max = 0, whi_min = nq - 1, whi_max = nq - 1;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
    const int last = min(31, nk - 1 - wk0);
    wlo_min = __builtin_amdgcn_readfirstlane(qlo);
    whi_min = __builtin_amdgcn_readfirstlane(qhi);
    wlo_max = __builtin_amdgcn_readlane(qlo, last);
    whi_max = __builtin_amdgcn_readlane(qhi, last);
  }
  auto tcls = [&](int qa) -> int {
    const int qz = qa + 31;
    if (!wave_active) return 0;
    if (POL == 0) return 2;  // q >= nq rows carry -lse2 = -inf -> P = 0; keys >= nk are never stored
    if (POL == 2) return qa < nq ? tile_class(a.rule, qa, min(qz, nq - 1), wk0, min(wk0 + 31, nk - 1)) : 0;
    if (wlo_min > qz || whi_max < qa) return 0;
    return (wlo_max <= qa && whi_min >= qz) ? 2 : 1;
  };

  // ---- query-tile staging, every thread (Q, dO chunks: 8 queries of one channel row)
  uint32_t voff[kCPT];
  int crow_[kCPT], cm_[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int idx = (tid + kThr * j) % kQChunks;
    crow_[j] = idx >> 2;
    cm_[j] = idx & 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nq * 2u + (ALN ? 16u * cm_[j] : 0u);
  }
  u32x4 qr[2][kCPT];  // two staging sets: tile t in set t&1, loaded two steps before it is stored
  float lr[2] = {0.f, 0.f};
  auto is_o = [&](int j) -> bool {
    return (kQChunks % kThr == 0) ? (j >= kQChunks / kThr) : ((tid + kThr * j) >= kQChunks);
  };
  auto load_tile = [&](int qa, int set) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      if constexpr (ALN) {
        const bool out = qa + 8 * cm_[j] >= nq || crow_[j] >= (isO ? vd : d);
        qr[set][j] = buf_load16(isO ? ors : qrs, voff[j], 2 * min(qa, nq), out);
      } else {
        qr[set][j] = buf_load8h(isO ? ors : qrs, voff[j], qa + 8 * cm_[j], nq, crow_[j] < (isO ? vd : d));
      }
    }
    if (w == 0) {  // lanes 0..31: -lse2, 32..63: -D (a wave-uniform scalar branch; the load itself is
                   // unconditional, clamped into the row, and the select replaces rows past nq)
      const int q = qa + (lane & 31);
      const float v = (lane < 32 ? glse : gD)[min(q, nq - 1)];
      lr[set] = (q < nq) ? v : ((lane < 32) ? -__builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot, int set) __attribute__((always_inline)) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      *reinterpret_cast<lds_u32x4_t*>(base + (isO ? S::offOT : S::offQT) + q16_off(crow_[j], cm_[j])) = qr[set][j];
    }
    if (w == 0) reinterpret_cast<lds_f_t*>(base + (lane < 32 ? S::offLse : S::offD - 128))[lane] = lr[set];
  };
  // hand-over slot of this wave pair: four b128 per lane (P k-steps 0/1, dS k-steps 0/1), lane-linear
  auto xoff = [&](int xs, int j) -> uint32_t { return S::offX + xs * S::kXSlot + wl * S::kXWave + j * 1024 + lane * 16; };

  // Steps it = 0 .. ntiles: the producer handles tile it (it < ntiles), the consumer tile it-1 (it >= 1).
  // Whole groups of four steps (ring slot it % 4, staging set (it+1) % 2, hand-over slot it % 2 are
  // compile-time); loads and stores are unconditional (phantom tiles move zeros), so hipcc's vmcnt
  // waits stay exact.
  const int nsteps = ntiles + 1;
  auto stage = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    __syncthreads();
    store_tile((c + 1) % 4, (c + 1) % 2);         // tile it+1 (loaded in step it-2)
    load_tile(qt0 + 32 * (it + 3), (c + 1) % 2);  // tile it+3 into the set just stored
  };
  // first tiles: tile 0's loads issued now, its store after the barrier that retires the K/V images
  load_tile(qt0, 0);
  auto stage0 = [&]() __attribute__((always_inline)) {
    __syncthreads();
    store_tile(0, 0);
    load_tile(qt0 + 32, 1);
    load_tile(qt0 + 64, 0);
  };

  if (grp == 0) {
    // ================= producer
    half8 kb[D / 16], vb[D / 16];  // resident B operands: lane (r,h) holds X[c = 16s + 8h + j][key]
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * wl + 16 * (g & 1) + 4 * tp;
        const uint32_t off = crow * (2 * kBK) + ((col * 2) ^ ((crow & 3) << 6));
        const half4 x = tr_read(smem + off), y = tr_read(smem + S::kRow + off);
        if (e == 0) { kb[s].lo = x; vb[s].lo = y; } else { kb[s].hi = x; vb[s].hi = y; }
      }
#pragma unroll
    for (int s = 0; s < D / 16; ++s) kb[s] = scale8(kb[s], c2);  // S in log2 units straight out of the MFMA
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every image read done before the ring reuses it
    stage0();
    const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;
    // row constants (-lse2, -D) of a tile: registers 4gq..4gq+3 = queries 16(gq>>1) + 8h + 4(gq&1) + 0..3
    auto read_rowc = [&](const lds_char_t* base, floatx16& sa, floatx16& pa) __attribute__((always_inline)) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int q4 = 16 * (gq >> 1) + 8 * h + 4 * (gq & 1);
        const floatx4 l4 = *reinterpret_cast<const lds_f4_t*>(base + S::offLse + 4 * q4);
        const floatx4 d4 = *reinterpret_cast<const lds_f4_t*>(base + S::offD + 4 * q4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sa[4 * gq + j] = l4[j];
          pa[4 * gq + j] = d4[j];
        }
      }
    };
    // the S / dP A operands of k-step s_ (transposed reads of the Q16 images)
    auto read_ops = [&](const lds_char_t* base, int s_, half8& q8, half8& o8) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint32_t off = q16_off(16 * s_ + 8 * (g >> 1) + 4 * e + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
        const half4 x = tr_read(base + S::offQT + off), y = tr_read(base + S::offOT + off);
        if (e == 0) { q8.lo = x; o8.lo = y; } else { q8.hi = x; o8.hi = y; }
      }
    };
    auto pstep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, it);
      const int qa = qt0 + 32 * it;
      const int cls = it < ntiles ? tcls(qa) : 0;
      const lds_char_t* base = smem + c * S::kSlot;
      floatx16 sacc, pacc;
      if (cls != 0) {
        // S = Qᵀ·K', dP = dOᵀ·V: A operands by transposed reads, two k-steps ahead of their MFMAs
        constexpr int kS = D / 16, kAh = 2;
        half8 qa8[kAh + 1], oa8[kAh + 1];
        auto rd = [&](int s_) __attribute__((always_inline)) {
          read_ops(base, s_, qa8[s_ % (kAh + 1)], oa8[s_ % (kAh + 1)]);
        };
        read_rowc(base, sacc, pacc);
#pragma unroll
        for (int s_ = 0; s_ < kAh; ++s_) rd(s_);
#pragma unroll
        for (int s_ = 0; s_ < kS; ++s_) {
          if (s_ + kAh < kS) rd(s_ + kAh);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa8[s_ % (kAh + 1)], kb[s_], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa8[s_ % (kAh + 1)], vb[s_], pacc, 0, 0, 0);
        }
      }
      if (cls == 0) return;
      // P = exp2(S), dS = P∘dP; register i = query 16(i>>3) + 8h + (i&7) = k-step i>>3 of the consumer
      half8 pf[2], sf[2];
      auto softmax = [&](bool masked) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float pv = __builtin_amdgcn_exp2f(sacc[i]);
          if (POL == 1 && masked) {
            const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
            pv = ((unsigned)(q - qlo) < (unsigned)qspan) ? pv : 0.f;
          }
          if (POL == 2 && masked) {
            const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
            pv = (q < nq && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko)) ? pv : 0.f;
          }
          pf[i >> 3][i & 7] = (_Float16)pv;
          sf[i >> 3][i & 7] = (_Float16)(pv * pacc[i]);
        }
      };
      // the edge-tile mask as a real branch: in one basic block hipcc if-converts it into an index add,
      // a compare and two selects per score on every tile (c3 backward 8.35 -> 7.72 ms)
      if (POL != 0 && cls == 1) {
        asm volatile("; edge tile" ::: );
        softmax(true);
      } else {
        asm volatile("; interior tile" ::: );
        softmax(false);
      }
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) {
        *reinterpret_cast<lds_half8_t*>(smem + xoff(c % 2, s_)) = pf[s_];
        *reinterpret_cast<lds_half8_t*>(smem + xoff(c % 2, 2 + s_)) = sf[s_];
      }
    };
    for (int it = 0; it < nsteps; it += 4) {
      pstep(IC<0>{}, it);
      pstep(IC<1>{}, it + 1);
      pstep(IC<2>{}, it + 2);
      pstep(IC<3>{}, it + 3);
    }
    return;
  }

  // ================= consumer
  stage0();
  floatx16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dk[u][i] = 0.f; dv[u][i] = 0.f; }
  auto cstep = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    stage(C_, it);
    const int qa = qt0 + 32 * (it - 1);
    const int cls = (it >= 1 && it - 1 < ntiles) ? tcls(qa) : 0;
    const lds_char_t* base = smem + ((c + 3) % 4) * S::kSlot;
    // dV += dO·P, dK += Q·dS: A = X[row 32u + r][queries 16s + 8h + 0..7] (b128 reads, two ahead)
    constexpr int kU = D / 32, kN = 2 * kU, kAh = 2;
    half8 pf[2], sf[2], oa[kAh + 1], qa_[kAh + 1];
    auto rd = [&](int n) __attribute__((always_inline)) {
      const int s_ = n / kU, u = n % kU;
      oa[n % (kAh + 1)] = read_b128(base + S::offOT + q16_off(32 * u + r, 2 * s_ + h));
      qa_[n % (kAh + 1)] = read_b128(base + S::offQT + q16_off(32 * u + r, 2 * s_ + h));
    };
    if (cls != 0) {
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) {
        pf[s_] = read_b128(smem + xoff((c + 1) % 2, s_));
        sf[s_] = read_b128(smem + xoff((c + 1) % 2, 2 + s_));
      }
#pragma unroll
      for (int n = 0; n < kAh; ++n) rd(n);
    }
    if (cls == 0) return;
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      if (n + kAh < kN) rd(n + kAh);
      const int s_ = n / kU, u = n % kU;
      dv[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa[n % (kAh + 1)], pf[s_], dv[u], 0, 0, 0);
      dk[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa_[n % (kAh + 1)], sf[s_], dk[u], 0, 0, 0);
    }
  };
  for (int it = 0; it < nsteps; it += 4) {
    cstep(IC<0>{}, it);
    cstep(IC<1>{}, it + 1);
    cstep(IC<2>{}, it + 2);
    cstep(IC<3>{}, it + 3);
  }

  // ---- dK = scale·Σ dS·Q, dV: rows c = 32u + (i&3) + 8(i>>2) + 4h, column = this lane's key
  if (!wave_active || key >= nk) return;
  __half* dK = static_cast<__half*>(a.dK) + bi * (int64_t)d * nk;
  __half* dV = static_cast<__half*>(a.dV) + bi * (int64_t)vd * nk;
  const float sc = (float)a.scale;
  if (d == D && vd == D) {
    const __amdgpu_buffer_rsrc_t krs_ = make_rsrc(dK, 2u * d * nk), vrs_ = make_rsrc(dV, 2u * vd * nk);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nk + (uint32_t)key);
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t so = 2u * (32u * u + (i & 3) + 8u * (i >> 2)) * (uint32_t)nk;
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(dk[u][i] * sc)), krs_, vlane, so, 0);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)dv[u][i]), vrs_, vlane, so, 0);
      }
    return;
  }
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dK[(int64_t)c * nk + key] = __float2half(dk[u][i] * sc);
      if (c < vd) dV[(int64_t)c * nk + key] = __float2half(dv[u][i]);
    }
}

// ---------------------------------------------------------------------------
// dK / dV at D = 256 without the recomputed products: four roles a 32-key slice, each holding one
// 64-register resident operand or one 128-register accumulator at two waves per SIMD
//   A  (S):   S = Qᵀ·K' (C = -lse2), P = exp2(S) (masked)          -> P   hand-over
//   B  (dP):  dP = dOᵀ·V (C = -D) of the tile before, dS = P∘dP      -> dS  hand-over
//   C  (dV):  dV += dO·P of the tile before
//   Dk (dK):  dK += Q·dS of the tile two before
// so S and dP are formed once per (key block, query tile) instead of once per 128-channel output
// chunk (the one-wave pass with OC = 2 issued 96 MFMAs a 32 x 32 pair; this pass 64, 16 a role).
// A workgroup = two slices (64 keys); waves 0-3 = A0, B0, A1, B1 and 4-7 = C0, Dk0, C1, Dk1, so every
// SIMD pairs a softmax role with an accumulating one.  Every step: one barrier, the staging of tile
// it+1 into the four-slot ring (Q, dO Q16 images, -lse2, -D), the load of tile it+3.
struct W4Smem {
  static constexpr int D = 256;
  static constexpr int kBK = 64;              // keys per workgroup: two slices of 32
  static constexpr int kRow = D * kBK * 2;    // K (or V) row image (prologue only): 32 KB
  static constexpr int kQT = D * 64;          // one [D][32] Q16 image: 16 KB
  static constexpr int offQT = 0, offOT = kQT, offLse = 2 * kQT, offD = offLse + 128;
  static constexpr int kSlot = offLse + 256;  // + -lse2[32], -D[32]
  static constexpr int kNS = 4;               // query-tile ring
  static constexpr int kXW = 2048;            // one slice's P (or dS) of a tile: 32 x 32 fp16, lane-linear
  static constexpr int offP = kNS * kSlot;    // P hand-over: 2 slots x 2 slices
  static constexpr int offS = offP + 4 * kXW; // dS hand-over: 2 slots x 2 slices
  static constexpr int kUsed = offS + 4 * kXW;
  static constexpr int kTotal = kUsed > 2 * kRow ? kUsed : 2 * kRow;
};

template <int POL, bool ALN>
__global__ __launch_bounds__(512, 1) void bwd_dkdv_w4_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = W4Smem;
  constexpr int D = S::D;
  constexpr int kThr = 512;
  constexpr int kBK = S::kBK;
  constexpr int kQChunks = D * 4;                 // 16-B chunks of one [D][32] tile
  constexpr int kCPT = 2 * kQChunks / kThr;       // Q and dO chunks per thread
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sl = (w >> 1) & 1;                    // key slice
  const int role = (w & 1) + 2 * (w >> 2);        // 0 A, 1 B, 2 C, 3 Dk
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int sig = ((tp & 1) << 1) | (tp >> 1);   // σ-permuted transposed reads (see the dK/dV kernel)
  const float c2 = (float)a.scale * kLog2e;

  const int d = a.d, vd = a.v_d;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq, 2u * d * nq);
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq, 2u * vd * nq);
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;

  // ---- K, V blocks into LDS (every thread); roles A / B read their resident B operands below
  {
    constexpr int kRPT = 2 * D * (kBK / 8) / kThr, kHalf = D * (kBK / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBK / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t krs2 = make_rsrc(K, 2u * d * nk), vrs2 = make_rsrc(V, 2u * vd * nk);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      const bool in = c < (which ? vd : d) && k0 + 8 * m < nk;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? vrs2 : krs2,
                                                       in ? (uint32_t)c * (uint32_t)nk * 2u + 16u * m : 0x80000000u, 2 * k0, 0);
      else
        rv[jj] = buf_load8h(which ? vrs2 : krs2, (uint32_t)c * (uint32_t)nk * 2u, k0 + 8 * m, nk, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBK / 8), m = j % (kBK / 8);
      // (128-B rows, unswizzled: the images are read once per block)
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBK) + m * 16) = rv[jj];
    }
  }
  __syncthreads();

  // ---- query range of this key block; per-lane / per-wave query intervals of the slice's keys
  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / 32) * 32;
  const int ntiles = (qe > qb) ? (qe - qt0 + 31) / 32 : 0;
  const int key = k0 + 32 * sl + r;
  const int wk0 = k0 + 32 * sl;
  const bool wave_active = wk0 < nk;
  int qlo = 0, qspan = nq, wlo_min = 0, wlo_max = 0, whi_min = nq - 1, whi_max = nq - 1;
  if (POL == 1 && wave_active) {
    int qhi;
    query_interval(a.rule, min(key, nk - 1), &qlo, &qhi);
    qspan = max(qhi - qlo + 1, 0);
    const int last = min(31, nk - 1 - wk0);
    wlo_min = __builtin_amdgcn_readfirstlane(qlo);
    whi_min = __builtin_amdgcn_readfirstlane(qhi);
    wlo_max = __builtin_amdgcn_readlane(qlo, last);
    whi_max = __builtin_amdgcn_readlane(qhi, last);
  }
  // class of tile t for this slice (0 outside [0, ntiles): phantom steps)
  auto tcls = [&](int t) -> int {
    if (t < 0 || t >= ntiles || !wave_active) return 0;
    const int qa = qt0 + 32 * t, qz = qa + 31;
    if (POL == 0) return 2;  // q >= nq rows carry -lse2 = -inf -> P = 0; keys >= nk are never stored
    if (POL == 2) return qa < nq ? tile_class(a.rule, qa, min(qz, nq - 1), wk0, min(wk0 + 31, nk - 1)) : 0;
    if (wlo_min > qz || whi_max < qa) return 0;
    return (wlo_max <= qa && whi_min >= qz) ? 2 : 1;
  };

  // ---- query-tile staging, every thread (Q, dO chunks: 8 queries of one channel row)
  uint32_t voff[kCPT];
  int crow_[kCPT], cm_[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int idx = (tid + kThr * j) % kQChunks;
    crow_[j] = idx >> 2;
    cm_[j] = idx & 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nq * 2u + (ALN ? 16u * cm_[j] : 0u);
  }
  u32x4 qr[2][kCPT];  // two staging sets: tile t in set t&1, loaded two steps before it is stored
  float lr[2] = {0.f, 0.f};
  auto is_o = [&](int j) -> bool { return j >= kQChunks / kThr; };
  auto load_tile = [&](int qa, int set) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      if constexpr (ALN) {
        const bool out = qa + 8 * cm_[j] >= nq || crow_[j] >= (isO ? vd : d);
        qr[set][j] = buf_load16(isO ? ors : qrs, voff[j], 2 * min(qa, nq), out);
      } else {
        qr[set][j] = buf_load8h(isO ? ors : qrs, voff[j], qa + 8 * cm_[j], nq, crow_[j] < (isO ? vd : d));
      }
    }
    if (w == 0) {  // lanes 0..31: -lse2, 32..63: -D (wave-uniform branch; clamped load, select past nq)
      const int q = qa + (lane & 31);
      const float v = (lane < 32 ? glse : gD)[min(q, nq - 1)];
      lr[set] = (q < nq) ? v : ((lane < 32) ? -__builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot, int set) __attribute__((always_inline)) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = is_o(j);
      *reinterpret_cast<lds_u32x4_t*>(base + (isO ? S::offOT : S::offQT) + q16_off(crow_[j], cm_[j])) = qr[set][j];
    }
    if (w == 0) reinterpret_cast<lds_f_t*>(base + S::offLse)[lane] = lr[set];
  };
  // hand-over of this slice: two b128 per lane (k-steps 0 / 1), lane-linear
  auto poff = [&](int xs, int j) -> uint32_t { return S::offP + (2 * xs + sl) * S::kXW + j * 1024 + lane * 16; };
  auto soff = [&](int xs, int j) -> uint32_t { return S::offS + (2 * xs + sl) * S::kXW + j * 1024 + lane * 16; };

  // Steps it = 0 .. ntiles + 1: A handles tile it, B and C tile it-1, Dk tile it-2.  Whole groups of
  // four steps (ring slot it % 4, staging set (it+1) % 2, hand-over slot it % 2 compile-time); loads
  // and stores unconditional (phantom tiles move zeros), so hipcc's vmcnt waits stay exact.
  const int nsteps = ntiles + 2;
  // (TAG: a distinct marker per role, so hipcc does not merge the roles' identical staging blocks into
  // one shared block, which joins every role's live registers: 884 spilled VGPRs)
  auto stage = [&](auto C_, auto TAG_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    asm volatile("; stage, role %0" ::"i"(decltype(TAG_)::value));
    __syncthreads();
    store_tile((c + 1) % 4, (c + 1) % 2);         // tile it+1 (loaded in step it-2)
    load_tile(qt0 + 32 * (it + 3), (c + 1) % 2);  // tile it+3 into the set just stored
  };
  load_tile(qt0, 0);
  auto stage0 = [&](auto TAG_) __attribute__((always_inline)) {
    asm volatile("; stage 0, role %0" ::"i"(decltype(TAG_)::value));
    __syncthreads();  // the K / V images are retired: the ring may overwrite them
    store_tile(0, 0);
    load_tile(qt0 + 32, 1);
    load_tile(qt0 + 64, 0);
  };
  // the S / dP A operand of k-step s_ from a Q16 image (transposed reads): a lane base per half e
  // (q16_off(16 s + x) = 1024 s + q16_off(x) for x < 16), made opaque once per chain so hipcc adds the
  // ring slot's offset in the step instead of keeping a base live for every (slot, half): as
  // bwd_dq_w4_kernel, where those bases were spilled and reloaded every step
  const uint32_t rb0 = q16_off(8 * (g >> 1) + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
  const uint32_t rb1 = q16_off(8 * (g >> 1) + 4 + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
  auto read_op = [&](const lds_char_t* img, const uint32_t (&rb)[2], int s_) __attribute__((always_inline)) -> half8 {
    half8 x;
    x.lo = tr_read(img + rb[0] + 1024 * s_);
    x.hi = tr_read(img + rb[1] + 1024 * s_);
    return x;
  };
  // the resident B operand of a role A / B wave: X[c = 16s + 8h + j][key] from the K or V image
  auto resident = [&](int which, half8 (&xb)[D / 16]) __attribute__((always_inline)) {
#pragma unroll
    for (int s_ = 0; s_ < D / 16; ++s_)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s_ + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * sl + 16 * (g & 1) + 4 * tp;
        const half4 x = tr_read(smem + which * S::kRow + crow * (2 * kBK) + col * 2);
        if (e == 0) xb[s_].lo = x; else xb[s_].hi = x;
      }
  };
  // a row constant (-lse2 or -D) of the tile in `base` as the initial accumulator
  auto read_rowc = [&](const lds_char_t* base, int off, floatx16& acc) __attribute__((always_inline)) {
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {  // registers 4gq..4gq+3 = queries 16(gq>>1) + 8h + 4(gq&1) + 0..3
      const int q4 = 16 * (gq >> 1) + 8 * h + 4 * (gq & 1);
      const floatx4 v4 = *reinterpret_cast<const lds_f4_t*>(base + off + 4 * q4);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 * gq + j] = v4[j];
    }
  };
  // S / dP chain: 16 MFMAs, A operands two k-steps ahead
  auto chain = [&](const lds_char_t* img, const half8 (&xb)[D / 16], floatx16& acc) __attribute__((always_inline)) {
    constexpr int kS = D / 16, kAh = 2;
    uint32_t rb[2] = {rb0, rb1};
    asm volatile("" : "+v"(rb[0]), "+v"(rb[1]));
    half8 a8[kAh + 1];
#pragma unroll
    for (int s_ = 0; s_ < kAh; ++s_) a8[s_] = read_op(img, rb, s_);
#pragma unroll
    for (int s_ = 0; s_ < kS; ++s_) {
      if (s_ + kAh < kS) a8[(s_ + kAh) % (kAh + 1)] = read_op(img, rb, s_ + kAh);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[s_ % (kAh + 1)], xb[s_], acc, 0, 0, 0);
    }
  };
  // X += Y·Z: A = Y[row 32u + r][queries 16s + 8h + 0..7] (b128 reads of a Q16 image, two ahead), B = Z k-step s
  auto accum = [&](const lds_char_t* img, const half8 (&z)[2], floatx16 (&acc)[D / 32]) __attribute__((always_inline)) {
    constexpr int kU = D / 32, kN = 2 * kU, kAh = 2;
    half8 y[kAh + 1];
    // (row 32m + r: q16_off = 2048 m + q16_off(r); two opaque lane bases, one per unit, as read_op)
    uint32_t gb[2] = {q16_off(r, h), q16_off(r, 2 + h)};
    asm volatile("" : "+v"(gb[0]), "+v"(gb[1]));
    auto rd = [&](int n) __attribute__((always_inline)) {
      y[n % (kAh + 1)] = read_b128(img + gb[n / kU] + 2048 * (n % kU));
    };
#pragma unroll
    for (int n = 0; n < kAh; ++n) rd(n);
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      if (n + kAh < kN) rd(n + kAh);
      acc[n % kU] = __builtin_amdgcn_mfma_f32_32x32x16_f16(y[n % (kAh + 1)], z[n / kU], acc[n % kU], 0, 0, 0);
    }
  };

  if (role == 0) {
    // ================= A: S, P
    half8 kb[D / 16];
    resident(0, kb);
#pragma unroll
    for (int s_ = 0; s_ < D / 16; ++s_) kb[s_] = scale8(kb[s_], c2);  // S in log2 units straight out of the MFMA
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every image read done before the ring reuses it
    stage0(IC<0>{});
    const int ko = (POL == 2) ? seq_order(a.rule.k, a.rule, min(key, nk - 1)) : 0;
    auto astep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<0>{}, it);
      const int cls = tcls(it);
      if (cls == 0) return;
      const lds_char_t* base = smem + c * S::kSlot;
      const int qa = qt0 + 32 * it;
      floatx16 sacc;
      read_rowc(base, S::offLse, sacc);
      chain(base + S::offQT, kb, sacc);
      half8 pf[2];
      auto softmax = [&](bool masked) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float pv = __builtin_amdgcn_exp2f(sacc[i]);
          if (POL == 1 && masked) {
            const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
            pv = ((unsigned)(q - qlo) < (unsigned)qspan) ? pv : 0.f;
          }
          if (POL == 2 && masked) {
            const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
            pv = (q < nq && check_orders_bf(a.rule, seq_order(a.rule.q, a.rule, min(q, nq - 1)), ko)) ? pv : 0.f;
          }
          pf[i >> 3][i & 7] = (_Float16)pv;
        }
      };
      if (POL != 0 && cls == 1) {
        asm volatile("; edge tile" ::: );
        softmax(true);
      } else {
        asm volatile("; interior tile" ::: );
        softmax(false);
      }
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) *reinterpret_cast<lds_half8_t*>(smem + poff(c % 2, s_)) = pf[s_];
    };
    for (int it = 0; it < nsteps; it += 4) {
      astep(IC<0>{}, it);
      astep(IC<1>{}, it + 1);
      astep(IC<2>{}, it + 2);
      astep(IC<3>{}, it + 3);
    }
    return;
  }
  if (role == 1) {
    // ================= B: dP, dS of the tile before
    half8 vb[D / 16];
    resident(1, vb);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stage0(IC<1>{});
    auto bstep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<1>{}, it);
      if (tcls(it - 1) == 0) return;
      const lds_char_t* base = smem + ((c + 3) % 4) * S::kSlot;
      floatx16 pacc;
      read_rowc(base, S::offD, pacc);
      chain(base + S::offOT, vb, pacc);
      half8 pf[2], sf[2];
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) pf[s_] = read_b128(smem + poff((c + 1) % 2, s_));
#pragma unroll
      for (int i = 0; i < 16; ++i) sf[i >> 3][i & 7] = (_Float16)((float)pf[i >> 3][i & 7] * pacc[i]);
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) *reinterpret_cast<lds_half8_t*>(smem + soff((c + 1) % 2, s_)) = sf[s_];
    };
    for (int it = 0; it < nsteps; it += 4) {
      bstep(IC<0>{}, it);
      bstep(IC<1>{}, it + 1);
      bstep(IC<2>{}, it + 2);
      bstep(IC<3>{}, it + 3);
    }
    return;
  }

  // ================= C (dV += dO·P, the tile before) or Dk (dK += Q·dS, two before): one code path
  // each (a runtime role test inside the step spilled ~600 VGPRs)
  auto accumulate = [&](auto ISC_) __attribute__((always_inline)) {
    constexpr bool isC = decltype(ISC_)::value;
    stage0(IC<isC ? 2 : 3>{});
    floatx16 acc[D / 32];
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[u][i] = 0.f;
    auto cstep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<isC ? 2 : 3>{}, it);
      if constexpr (isC) {
        if (tcls(it - 1) == 0) return;
        half8 pf[2];
#pragma unroll
        for (int s_ = 0; s_ < 2; ++s_) pf[s_] = read_b128(smem + poff((c + 1) % 2, s_));
        accum(smem + ((c + 3) % 4) * S::kSlot + S::offOT, pf, acc);
      } else {
        if (tcls(it - 2) == 0) return;
        half8 sf[2];
#pragma unroll
        for (int s_ = 0; s_ < 2; ++s_) sf[s_] = read_b128(smem + soff(c % 2, s_));
        accum(smem + ((c + 2) % 4) * S::kSlot + S::offQT, sf, acc);
      }
    };
    for (int it = 0; it < nsteps; it += 4) {
      cstep(IC<0>{}, it);
      cstep(IC<1>{}, it + 1);
      cstep(IC<2>{}, it + 2);
      cstep(IC<3>{}, it + 3);
    }
    // ---- dV, or dK = scale·Σ dS·Q: rows c = 32u + (i&3) + 8(i>>2) + 4h, column = this lane's key
    if (!wave_active || key >= nk) return;
    __half* X = static_cast<__half*>(isC ? a.dV : a.dK) + bi * (int64_t)(isC ? vd : d) * nk;
    const int dx = isC ? vd : d;
    const float sc = isC ? 1.f : (float)a.scale;
    if (dx == D) {
      const __amdgpu_buffer_rsrc_t xrs = make_rsrc(X, 2u * D * nk);
      const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nk + (uint32_t)key);
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t so = 2u * (32u * u + (i & 3) + 8u * (i >> 2)) * (uint32_t)nk;
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(acc[u][i] * sc)), xrs, vlane, so,
                                                0);
        }
      return;
    }
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cc = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (cc < dx) X[(int64_t)cc * nk + key] = __float2half(acc[u][i] * sc);
      }
  };
  if (role == 2) accumulate(IC<1>{});
  else accumulate(IC<0>{});
}


// ---------------------------------------------------------------------------
// dQ at D = 256 without the recomputed products: the four-role split of bwd_dkdv_w4_kernel applied to
// the query-outer pass, a 32-query slice per role set
//   E  (Sᵀ):  Sᵀ = Kᵀ·Q' (C = -lse2), P = exp2(Sᵀ) (masked)          -> P   hand-over
//   F  (dPᵀ): dPᵀ = Vᵀ·dO (C = -D) of the tile before, dSᵀ = P∘dPᵀ    -> dSᵀ hand-over
//   G0, G1:   dQ += K·dSᵀ of the tile two before, channels 0-127 / 128-255
// (the one-wave pass with OC = 2 formed Sᵀ and dPᵀ in both channel chunks: 80 MFMAs a 32 x 32 pair,
// this pass 48).  Waves 0-3 = E0, F0, E1, F1 and 4-7 = G0/0, G1/0, G0/1, G1/1: every SIMD pairs a
// 16-MFMA role with an 8-MFMA one.  Key tiles of 32 ([D][32] images like the dK/dV pass's query tiles).
struct W4DqSmem {
  static constexpr int D = 256;
  static constexpr int kBM = 64;              // queries per workgroup: two slices of 32
  static constexpr int kRow = D * kBM * 2;    // Q (or dO) row image (prologue only): 32 KB
  static constexpr int kKT = D * 64;          // one [D][32] K16 image: 16 KB
  static constexpr int offKT = 0, offVT = kKT;
  static constexpr int kSlot = 2 * kKT;
  static constexpr int kNS = 4;               // key-tile ring
  static constexpr int kXW = 2048;            // one slice's P (or dSᵀ) of a tile, lane-linear
  static constexpr int offP = kNS * kSlot;
  static constexpr int offS = offP + 4 * kXW;
  static constexpr int kUsed = offS + 4 * kXW;
  static constexpr int kTotal = kUsed > 2 * kRow ? kUsed : 2 * kRow;
};

template <int POL, bool ALN>
__global__ __launch_bounds__(512, 1) void bwd_dq_w4_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = W4DqSmem;
  constexpr int D = S::D;
  constexpr int kThr = 512;
  constexpr int kBM = S::kBM;
  constexpr int kKChunks = D * 4;                 // 16-B chunks of one [D][32] tile
  constexpr int kCPT = 2 * kKChunks / kThr;       // K and V chunks per thread
  constexpr float kNegInf = -__builtin_huge_valf();
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sl = (w >> 1) & 1;                    // query slice
  const int role = (w & 1) + 2 * (w >> 2);        // 0 E, 1 F, 2 G0, 3 G1
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  const float c2 = (float)a.scale * kLog2e;
  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const int wq0 = q0 + 32 * sl;
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;

  // ---- Q, dO blocks into LDS (every thread, 128-B rows); roles E / F read their resident operands
  {
    constexpr int kRPT = 2 * D * (kBM / 8) / kThr, kHalf = D * (kBM / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBM / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t qrs2 = make_rsrc(Q, 2u * d * nq), ors2 = make_rsrc(dO, 2u * vd * nq);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      const bool in = c < (which ? vd : d) && q0 + 8 * m < nq;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? ors2 : qrs2,
                                                       in ? (uint32_t)c * (uint32_t)nq * 2u + 16u * m : 0x80000000u, 2 * q0, 0);
      else
        rv[jj] = buf_load8h(which ? ors2 : qrs2, (uint32_t)c * (uint32_t)nq * 2u, q0 + 8 * m, nq, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBM) + m * 16) = rv[jj];
    }
  }
  __syncthreads();

  // ---- key range of this query block, per-lane / per-wave key intervals of the slice's queries
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / 32) * 32;
  const int ntiles = (ke > kb) ? (ke - kt0 + 31) / 32 : 0;
  int klo = 0, kspan = nk, wlo_min = 0, wlo_max = 0, whi_min = nk - 1, whi_max = nk - 1;
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
  // class of tile t for this slice (0 outside [0, ntiles))
  auto tcls = [&](int t) -> int {
    if (t < 0 || t >= ntiles || !wave_active) return 0;
    const int ka = kt0 + 32 * t, kz = ka + 31;
    if (POL == 0) return kz < nk ? 2 : 1;
    if (POL == 2) {  // class 2 only for tiles wholly inside nk (the staged tail past nk is masked)
      if (ka >= nk) return 0;
      const int c = tile_class(a.rule, wq0, min(wq0 + 31, nq - 1), ka, min(kz, nk - 1));
      return (c == 2 && kz >= nk) ? 1 : c;
    }
    if (wlo_min > kz || whi_max < ka) return 0;
    return (wlo_max <= ka && whi_min >= kz && kz < nk) ? 2 : 1;
  };

  // ---- key-tile staging, every thread (K, V chunks: 8 keys of one channel row)
  uint32_t voff[kCPT];
  int crow_[kCPT], cm_[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int idx = (tid + kThr * j) % kKChunks;
    crow_[j] = idx >> 2;
    cm_[j] = idx & 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nk * 2u + (ALN ? 16u * cm_[j] : 0u);
  }
  u32x4 kr[2][kCPT];
  auto is_v = [&](int j) -> bool { return j >= kKChunks / kThr; };
  auto load_tile = [&](int ka, int set) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      if constexpr (ALN) {
        const bool out = ka + 8 * cm_[j] >= nk || crow_[j] >= (isV ? vd : d);
        kr[set][j] = buf_load16(isV ? vrs : krs, voff[j], 2 * min(ka, nk), out);
      } else {
        kr[set][j] = buf_load8h(isV ? vrs : krs, voff[j], ka + 8 * cm_[j], nk, crow_[j] < (isV ? vd : d));
      }
    }
  };
  auto store_tile = [&](int slot, int set) __attribute__((always_inline)) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      *reinterpret_cast<lds_u32x4_t*>(base + (isV ? S::offVT : S::offKT) + q16_off(crow_[j], cm_[j])) = kr[set][j];
    }
  };
  auto poff = [&](int xs, int j) -> uint32_t { return S::offP + (2 * xs + sl) * S::kXW + j * 1024 + lane * 16; };
  auto soff = [&](int xs, int j) -> uint32_t { return S::offS + (2 * xs + sl) * S::kXW + j * 1024 + lane * 16; };

  // Steps it = 0 .. ntiles + 1: E handles tile it, F tile it-1, G0 / G1 tile it-2 (as the dK/dV pass)
  const int nsteps = ntiles + 2;
  // (TAG: one marker per role, see bwd_dkdv_w4_kernel)
  auto stage = [&](auto C_, auto TAG_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    asm volatile("; stage, role %0" ::"i"(decltype(TAG_)::value));
    __syncthreads();
    store_tile((c + 1) % 4, (c + 1) % 2);
    load_tile(kt0 + 32 * (it + 3), (c + 1) % 2);
  };
  load_tile(kt0, 0);
  auto stage0 = [&](auto TAG_) __attribute__((always_inline)) {
    asm volatile("; stage 0, role %0" ::"i"(decltype(TAG_)::value));
    __syncthreads();  // the Q / dO images are retired
    store_tile(0, 0);
    load_tile(kt0 + 32, 1);
    load_tile(kt0 + 64, 0);
  };
  // transposed A-operand reads of k-step s_: a lane base per half e (q16_off(16 s + x) = 1024 s +
  // q16_off(x) for x < 16), made opaque once per chain so hipcc adds the slot's offset in the step
  // instead of keeping a (slot, half) base live for every ring slot (it spilled them and reloaded them
  // from scratch every step, with a vmcnt(0) that drained the staging loads)
  const uint32_t rb0 = q16_off(8 * (g >> 1) + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
  const uint32_t rb1 = q16_off(8 * (g >> 1) + 4 + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
  auto read_op = [&](const lds_char_t* img, const uint32_t (&rb)[2], int s_) __attribute__((always_inline)) -> half8 {
    half8 x;
    x.lo = tr_read(img + rb[0] + 1024 * s_);
    x.hi = tr_read(img + rb[1] + 1024 * s_);
    return x;
  };
  auto resident = [&](int which, half8 (&xb)[D / 16]) __attribute__((always_inline)) {
#pragma unroll
    for (int s_ = 0; s_ < D / 16; ++s_)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s_ + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * sl + 16 * (g & 1) + 4 * tp;
        const half4 x = tr_read(smem + which * S::kRow + crow * (2 * kBM) + col * 2);
        if (e == 0) xb[s_].lo = x; else xb[s_].hi = x;
      }
  };
  auto rowconst = [&](const void* ws, float dflt) -> floatx16 {
    const float* p = static_cast<const float*>(ws) + bi * (int64_t)nq;
    const float v = (qi < nq) ? p[qi] : dflt;
    floatx16 x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = v;
    return x;
  };
  auto chain = [&](const lds_char_t* img, const half8 (&xb)[D / 16], floatx16 acc) __attribute__((always_inline)) -> floatx16 {
    constexpr int kS = D / 16, kAh = 2;
    uint32_t rb[2] = {rb0, rb1};
    asm volatile("" : "+v"(rb[0]), "+v"(rb[1]));
    half8 a8[kAh + 1];
#pragma unroll
    for (int s_ = 0; s_ < kAh; ++s_) a8[s_] = read_op(img, rb, s_);
#pragma unroll
    for (int s_ = 0; s_ < kS; ++s_) {
      if (s_ + kAh < kS) a8[(s_ + kAh) % (kAh + 1)] = read_op(img, rb, s_ + kAh);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8[s_ % (kAh + 1)], xb[s_], acc, 0, 0, 0);
    }
    return acc;
  };

  if (role == 0) {
    // ================= E: Sᵀ, P
    half8 qf[D / 16];
    resident(0, qf);
#pragma unroll
    for (int s_ = 0; s_ < D / 16; ++s_) qf[s_] = scale8(qf[s_], c2);
    const floatx16 negl = rowconst(a.ws_lse, kNegInf);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stage0(IC<0>{});
    const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;
    auto estep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<0>{}, it);
      const int cls = tcls(it);
      if (cls == 0) return;
      const lds_char_t* base = smem + c * S::kSlot;
      const int ka = kt0 + 32 * it;
      const floatx16 sacc = chain(base + S::offKT, qf, negl);
      half8 pf[2];
      auto softmax = [&](bool masked) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float pv = __builtin_amdgcn_exp2f(sacc[i]);
          if (masked) {
            const int kk = ka + 16 * (i >> 3) + 8 * h + (i & 7);
            const bool ok = (POL == 1)   ? ((unsigned)(kk - klo) < (unsigned)kspan)
                            : (POL == 2) ? (kk < nk && check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1))))
                                         : (kk < nk);
            pv = ok ? pv : 0.f;
          }
          pf[i >> 3][i & 7] = (_Float16)pv;
        }
      };
      if (cls == 1) {
        asm volatile("; edge tile" ::: );
        softmax(true);
      } else {
        asm volatile("; interior tile" ::: );
        softmax(false);
      }
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) *reinterpret_cast<lds_half8_t*>(smem + poff(c % 2, s_)) = pf[s_];
    };
    for (int it = 0; it < nsteps; it += 4) {
      estep(IC<0>{}, it);
      estep(IC<1>{}, it + 1);
      estep(IC<2>{}, it + 2);
      estep(IC<3>{}, it + 3);
    }
    return;
  }
  if (role == 1) {
    // ================= F: dPᵀ, dSᵀ of the tile before
    half8 of[D / 16];
    resident(1, of);
    const floatx16 negd = rowconst(a.ws_D, 0.f);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stage0(IC<1>{});
    auto fstep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<1>{}, it);
      if (tcls(it - 1) == 0) return;
      const lds_char_t* base = smem + ((c + 3) % 4) * S::kSlot;
      const floatx16 pacc = chain(base + S::offVT, of, negd);
      half8 pf[2], sf[2];
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) pf[s_] = read_b128(smem + poff((c + 1) % 2, s_));
#pragma unroll
      for (int i = 0; i < 16; ++i) sf[i >> 3][i & 7] = (_Float16)((float)pf[i >> 3][i & 7] * pacc[i]);
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) *reinterpret_cast<lds_half8_t*>(smem + soff((c + 1) % 2, s_)) = sf[s_];
    };
    for (int it = 0; it < nsteps; it += 4) {
      fstep(IC<0>{}, it);
      fstep(IC<1>{}, it + 1);
      fstep(IC<2>{}, it + 2);
      fstep(IC<3>{}, it + 3);
    }
    return;
  }

  // ================= G0 / G1: dQ += K·dSᵀ (tile two before), one channel half each
  auto accumulate = [&](auto HH_) __attribute__((always_inline)) {
    constexpr int hh = decltype(HH_)::value;
    constexpr int kU = D / 64;  // 32-channel blocks of the half
    stage0(IC<2 + hh>{});
    floatx16 dq[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[u][i] = 0.f;
    auto gstep = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      stage(C_, IC<2 + hh>{}, it);
      if (tcls(it - 2) == 0) return;
      half8 sf[2];
#pragma unroll
      for (int s_ = 0; s_ < 2; ++s_) sf[s_] = read_b128(smem + soff(c % 2, s_));
      const lds_char_t* img = smem + ((c + 2) % 4) * S::kSlot + S::offKT;
      constexpr int kN = 2 * kU, kAh = 2;
      half8 y[kAh + 1];
      // (row 32m + r: q16_off = 2048 m + q16_off(r); two opaque lane bases, one per unit, as read_op)
      uint32_t gb[2] = {q16_off(r, h), q16_off(r, 2 + h)};
      asm volatile("" : "+v"(gb[0]), "+v"(gb[1]));
      auto rd = [&](int n) __attribute__((always_inline)) {
        y[n % (kAh + 1)] = read_b128(img + gb[n / kU] + 2048 * (kU * hh + n % kU));
      };
#pragma unroll
      for (int n = 0; n < kAh; ++n) rd(n);
#pragma unroll
      for (int n = 0; n < kN; ++n) {
        if (n + kAh < kN) rd(n + kAh);
        dq[n % kU] = __builtin_amdgcn_mfma_f32_32x32x16_f16(y[n % (kAh + 1)], sf[n / kU], dq[n % kU], 0, 0, 0);
      }
    };
    for (int it = 0; it < nsteps; it += 4) {
      gstep(IC<0>{}, it);
      gstep(IC<1>{}, it + 1);
      gstep(IC<2>{}, it + 2);
      gstep(IC<3>{}, it + 3);
    }
    if (!wave_active || qi >= nq) return;
    __half* dQ = static_cast<__half*>(a.dQ) + bi * (int64_t)d * nq;
    const float sc = (float)a.scale;
    if (d == D) {
      const __amdgpu_buffer_rsrc_t qrs_ = make_rsrc(dQ, 2u * d * nq);
      const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
      for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(dq[u][i] * sc)), qrs_, vlane,
                                                2u * (32u * (kU * hh + u) + (i & 3) + 8u * (i >> 2)) * (uint32_t)nq, 0);
      return;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cc = 32 * (kU * hh + u) + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (cc < d) dQ[(int64_t)cc * nq + qi] = __float2half(dq[u][i] * sc);
      }
  };
  if (role == 2) accumulate(IC<0>{});
  else accumulate(IC<1>{});
}

// ---------------------------------------------------------------------------
template <int D, int NW>
struct DqSmem {
  static constexpr int kBM = 32 * NW;                 // queries per workgroup
  static constexpr int kRow = D * kBM * 2;            // Q (or dO) row image
  static constexpr int kKT = D * 128;                 // one [D][64] KT image
  static constexpr int offKT = 0, offVT = kKT;
  static constexpr int kSlot = 2 * kKT;
  static constexpr int kRing = 2 * kSlot;
  static constexpr int kTotal = (kRing > 2 * kRow) ? kRing : 2 * kRow;  // the Q/dO images alias the ring
};

// dQ: query-outer.  One workgroup = NW waves x 32 queries of one (batch, head) slice.
// OC > 1 (128 < d <= 256): the workgroup accumulates dQ for one of OC chunks of D / OC channels (chunk =
// block index mod OC), recomputing Sᵀ and dPᵀ over all D channels.  ONESET: one staging register set
// (tile it+1 loaded at the head of step it and stored after its MFMAs, into the slot tile it-1 left)
// instead of two sets loaded two steps ahead: at D = 256 a set is 64 registers.
template <int D, int NW, int WPE, int POL, bool ALN, bool PRE = false, bool MSPEC = false, int OC = 1, bool ONESET = false>
__global__ __launch_bounds__(NW * 64, WPE) void bwd_dq_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = DqSmem<D, NW>;
  constexpr int kThr = NW * 64;
  constexpr int kBM = S::kBM;
  constexpr int kBN = 64;
  constexpr int kKChunks = D * 8;                     // 16-B chunks of one [D][64] tile
  static_assert((2 * kKChunks) % kThr == 0, "tile chunks must divide over the workgroup");
  constexpr int kCPT = 2 * kKChunks / kThr;           // K and V chunks per thread
  constexpr float kNegInf = -__builtin_huge_valf();

  constexpr int kDO = D / OC;  // dQ channels of this workgroup
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bidc = xcd_remap(blockIdx.x, gridDim.x);
  const int oc = (int)(bidc % OC), ou0 = oc * (kDO / 32);
  const uint32_t bid = bidc / OC;
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const float c2 = (float)a.scale * kLog2e;

  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);

  const int wq0 = q0 + 32 * w;
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;

  // ---- resident B operands: lane (r,h) holds X[c = 16s + 8h + j][q = wq0 + r]
  half8 qf[D / 16], of[D / 16];
  {
    // all loads before the stores, branch-free (see the dK/dV pass)
    constexpr int kRPT = 2 * D * (kBM / 8) / kThr, kHalf = D * (kBM / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBM / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t qrs2 = make_rsrc(Q, 2u * d * nq), ors2 = make_rsrc(dO, 2u * vd * nq);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      const bool in = c < (which ? vd : d) && q0 + 8 * m < nq;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? ors2 : qrs2,
                                                       in ? (uint32_t)c * (uint32_t)nq * 2u + 16u * m : 0x80000000u, 2 * q0, 0);
      else
        rv[jj] = buf_load8h(which ? ors2 : qrs2, (uint32_t)c * (uint32_t)nq * 2u, q0 + 8 * m, nq, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBM) + ((m * 16) ^ ((c & 3) << 6))) = rv[jj];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * w + 16 * (g & 1) + 4 * tp;
        const uint32_t off = crow * (2 * kBM) + ((col * 2) ^ ((crow & 3) << 6));
        const half4 x = tr_read(smem + off), y = tr_read(smem + S::kRow + off);
        if (e == 0) { qf[s].lo = x; of[s].lo = y; } else { qf[s].hi = x; of[s].hi = y; }
      }
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = scale8(qf[s], c2);
    __syncthreads();  // the Q/dO images are reused by the ring
  }
  // row constants (this lane's query) as the C operands of the Sᵀ / dPᵀ chains
  floatx16 negl, negd;
  {
    const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
    const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;
    const float lv = (qi < nq) ? glse[qi] : kNegInf, dv = (qi < nq) ? gD[qi] : 0.f;  // (stored negated)
#pragma unroll
    for (int i = 0; i < 16; ++i) { negl[i] = lv; negd[i] = dv; }
  }

  // ---- key range of this query block (rule-bounded), per-lane key intervals
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;
  int klo = 0, kspan = nk, wlo_min = 0, wlo_max = 0, whi_min = nk - 1, whi_max = nk - 1;
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
  auto tcls = [&](int ka) -> int {
    const int kz = ka + kBN - 1;
    if (!wave_active) return 0;
    if (POL == 0) return kz < nk ? 2 : 1;
    if (POL == 2) {  // class 2 only for tiles wholly inside nk (the staged tail past nk is masked)
      if (ka >= nk) return 0;
      const int c = tile_class(a.rule, wq0, min(wq0 + 31, nq - 1), ka, min(kz, nk - 1));
      return (c == 2 && kz >= nk) ? 1 : c;
    }
    if (wlo_min > kz || whi_max < ka) return 0;
    return (wlo_max <= ka && whi_min >= kz && kz < nk) ? 2 : 1;
  };

  const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;  // this lane's query order

  // ---- key-tile staging (K, V chunks: 8 keys of one channel row)
  uint32_t voff[kCPT];
  int crow_[kCPT];
  const int cm = tid & 7;
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    crow_[j] = ((tid + kThr * j) % kKChunks) >> 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nk * 2u + (ALN ? 16u * cm : 0u);  // (ALN: the chunk's; else the row's)
  }
  // two staging sets (tile t in set t&1): a tile is loaded two steps before it is stored
  u32x4 kr[ONESET ? 1 : 2][kCPT];
  auto is_v = [&](int j) -> bool {
    return (kKChunks % kThr == 0) ? (j >= kKChunks / kThr) : ((tid + kThr * j) >= kKChunks);
  };
  auto load_tile = [&](int ka, int set) {
    const bool out = ka + 8 * cm >= nk;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      if constexpr (ALN)
        kr[set][j] = buf_load16(isV ? vrs : krs, voff[j], 2 * min(ka, nk), out || crow_[j] >= (isV ? vd : d));
      else
        kr[set][j] = buf_load8h(isV ? vrs : krs, voff[j], ka + 8 * cm, nk, crow_[j] < (isV ? vd : d));
    }
  };
  auto store_tile = [&](int slot, int set) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      *reinterpret_cast<lds_u32x4_t*>(base + (isV ? S::offVT : S::offKT) + k2_off(crow_[j], cm)) = kr[set][j];
    }
  };
  floatx16 dq[kDO / 32];
#pragma unroll
  for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[u][i] = 0.f;

  // A-operand (Kᵀ / Vᵀ) read bases: lane 4q+p of a 16-lane group supplies channel row q, keys
  // 4σ(p)..4σ(p)+3 (σ swaps 1 and 2), so register i of Sᵀ / dPᵀ half t holds key 32t + 16(i>>3) +
  // 8h + (i&7): k-step s of dSᵀ is keys 16s + 8h + 0..7 and K's dQ A operand is one b128 row read
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t tb[2][2];  // [e][t], row 8(g>>1) + 4e + tq (+16s: immediate)
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int t = 0; t < 2; ++t) tb[e][t] = k2_off(8 * (g >> 1) + 4 * e + tq, 4 * t + 2 * (g & 1) + (sig >> 1), sig & 1);
  uint32_t kb2[4];  // dQ A operand: row 32u + r (+32u·128: immediate), chunk 2s + h
#pragma unroll
  for (int s = 0; s < 4; ++s) kb2[s] = k2_off(r, 2 * s + h);

  // unconditional (with no tiles it moves zeros): a conditional load here left hipcc's vmcnt
  // state merged, and the loop's first step then drained every load in flight
  load_tile(kt0, 0);
  store_tile(0, 0);
  if constexpr (!ONESET) {
    load_tile(kt0 + kBN, 1);
    load_tile(kt0 + 2 * kBN, 0);
  }

  auto step = [&](auto P_, int it) {
    constexpr int p = decltype(P_)::value;
    __syncthreads();
    const int ka = kt0 + it * kBN;
    const int cls = it < ntiles ? tcls(ka) : 0;  // (the loop's last pair may end on a phantom step)
    // unconditional (past the end they move zeros into a slot nobody reads): exact vmcnt waits
    if constexpr (ONESET) {
      load_tile(ka + kBN, 0);
    } else {
      store_tile(p ^ 1, p ^ 1);
      load_tile(ka + 3 * kBN, p ^ 1);
    }
    struct StoreAtExit {  // ONESET: tile it+1 into slot p^1 after this step's MFMAs (on every return)
      decltype(store_tile)& f;
      __device__ ~StoreAtExit() { if constexpr (ONESET) f(p ^ 1, 0); }
    } store_at_exit{store_tile};
    if (cls == 0) return;
    const lds_char_t* base = smem + p * S::kSlot;
    floatx16 st[2], dp[2];
    // PRE: every operand read two MFMA pairs ahead of its MFMAs (one wave per SIMD: nothing else
    // hides an LDS round trip between a read and the MFMA that consumes it)
    half8 ka8p[3];
    auto rka = [&](int n) __attribute__((always_inline)) {  // dQ operand n = (kDO/32)·s + u
      ka8p[n % 3] = read_b128(base + S::offKT + kb2[n / (kDO / 32)] + 32 * (ou0 + n % (kDO / 32)) * 128);
    };
    if constexpr (PRE) {
      constexpr int kN = 2 * (D / 16);
      half8 kf[3], vf[3];
      auto rd = [&](int n) __attribute__((always_inline)) {  // n = 2s + t
        const int s_ = n >> 1, t = n & 1;
        const uint32_t b0 = tb[0][t] + (16 * s_) * 128, b1 = tb[1][t] + (16 * s_) * 128;
        kf[n % 3].lo = tr_read(base + S::offKT + b0);
        kf[n % 3].hi = tr_read(base + S::offKT + b1);
        vf[n % 3].lo = tr_read(base + S::offVT + b0);
        vf[n % 3].hi = tr_read(base + S::offVT + b1);
      };
      rd(0);
      rd(1);
#pragma unroll
      for (int n = 0; n < kN; ++n) {
        if (n + 2 < kN) rd(n + 2);
        if (n == kN - 2) rka(0);
        if (n == kN - 1) rka(1);
        const int s_ = n >> 1, t = n & 1;
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[n % 3], qf[s_], s_ == 0 ? negl : st[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[n % 3], of[s_], s_ == 0 ? negd : dp[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int s = 0; s < (PRE ? 0 : D / 16); ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        half8 kf, vf;
        const uint32_t b0 = tb[0][t] + (16 * s) * 128, b1 = tb[1][t] + (16 * s) * 128;
        kf.lo = tr_read(base + S::offKT + b0);
        kf.hi = tr_read(base + S::offKT + b1);
        vf.lo = tr_read(base + S::offVT + b0);
        vf.hi = tr_read(base + S::offVT + b1);
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], s == 0 ? negl : st[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, of[s], s == 0 ? negd : dp[t], 0, 0, 0);
      }
    // dSᵀ = exp2(Sᵀ)∘dPᵀ; keys of register i of half t: 32t + 16(i>>3) + 8h + (i&7)
    auto dsq = [&](int cl) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 dsf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = s >> 1, i = 8 * (s & 1) + j;
        float pv = __builtin_amdgcn_exp2f(st[t][i]);
        if (cl == 1) {
          const int kk = ka + 32 * t + 16 * (i >> 3) + 8 * h + (i & 7);
          const bool ok = (POL == 1)   ? ((unsigned)(kk - klo) < (unsigned)kspan)
                          : (POL == 2) ? (kk < nk && check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1))))
                                       : (kk < nk);
          pv = ok ? pv : 0.f;
        }
        dsf[j] = (_Float16)(pv * dp[t][i]);
      }
#pragma unroll
      for (int u = 0; u < kDO / 32; ++u) {
        if constexpr (PRE) {
          const int n = (kDO / 32) * s + u;
          if (n + 2 < 4 * (kDO / 32)) rka(n + 2);
          dq[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka8p[n % 3], dsf, dq[u], 0, 0, 0);
        } else {
          const half8 ka8 = read_b128(base + S::offKT + kb2[s] + 32 * (ou0 + u) * 128);
          dq[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka8, dsf, dq[u], 0, 0, 0);
        }
      }
    }
    };
    // the edge-tile mask as a real branch (see the producer / consumer pass; MSPEC: the if-converted form)
    if constexpr (MSPEC) {
      dsq(cls);
    } else if (cls == 1) {
      asm volatile("; edge tile" ::: );
      dsq(1);
    } else {
      asm volatile("; interior tile" ::: );
      dsq(2);
    }
  };
  for (int it = 0; it < ntiles; it += 2) {  // whole pairs (see the dK/dV pass)
    step(IC<0>{}, it);
    step(IC<1>{}, it + 1);
  }

  if (!wave_active || qi >= nq) return;
  __half* dQ = static_cast<__half*>(a.dQ) + bi * (int64_t)d * nq;
  const float sc = (float)a.scale;
  if (d == D) {  // one buffer store per value (see the dK/dV pass)
    const __amdgpu_buffer_rsrc_t qrs_ = make_rsrc(dQ, 2u * d * nq);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
    for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(dq[u][i] * sc)), qrs_, vlane,
                                              2u * (32u * (ou0 + u) + (i & 3) + 8u * (i >> 2)) * (uint32_t)nq, 0);
    return;
  }
#pragma unroll
  for (int u = 0; u < kDO / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * (ou0 + u) + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dQ[(int64_t)c * nq + qi] = __float2half(dq[u][i] * sc);
    }
}

// ---------------------------------------------------------------------------
// dQ, producer / consumer (two waves per SIMD): the dK/dV pass's split applied to the query-outer
// pass.  Waves w and w+4 share a SIMD and the same 32 queries.  Wave w (producer) keeps Q' and dO
// resident, forms Sᵀ = Kᵀ·Q' and dPᵀ = Vᵀ·dO for key tile i one 32-key half at a time and
// dSᵀ = exp2(Sᵀ)∘dPᵀ, and hands dSᵀ to wave w+4 through LDS (four lane-linear b128 per lane);
// wave w+4 (consumer) stages the key tiles and accumulates dQ += K·dSᵀ for tile i-1.  The
// one-wave-per-SIMD pass above (332-345 registers) serialises its softmax and every LDS round trip
// behind its own MFMAs; here the producer's softmax runs beside the consumer's MFMAs and staging.
// Ring: four K/V slots (tile t in slot t % 4), two hand-over slots, one barrier per step;
// 4 x 32 KB + 32 KB = 160 KB at D = 128.
template <int D>
struct DqPcSmem {
  static constexpr int kBM = 128;           // queries per workgroup: four producer waves x 32
  static constexpr int kRow = D * kBM * 2;  // Q (or dO) row image (prologue only)
  static constexpr int kKT = D * 128;       // one [D][64] K2 image
  static constexpr int offKT = 0, offVT = kKT;
  static constexpr int kSlot = 2 * kKT;
  static constexpr int kNS = 4;
  static constexpr int offX = kNS * kSlot;  // dSᵀ hand-over: 2 slots x 4 waves x 4 KB
  static constexpr int kXWave = 4096, kXSlot = 4 * kXWave;
  static constexpr int kUsed = offX + 2 * kXSlot;
  static constexpr int kTotal = kUsed > 2 * kRow ? kUsed : 2 * kRow;  // the Q/dO images alias the ring
};

template <int D, int POL, bool ALN>
__global__ __launch_bounds__(512, 1) void bwd_dq_pc_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  using S = DqPcSmem<D>;
  constexpr int kThr = 512, kHalfThr = 256;  // one half of the workgroup stages
  constexpr int kBM = S::kBM, kBN = 64;
  constexpr int kKChunks = D * 8;  // 16-B chunks of one [D][64] tile
  static_assert((2 * kKChunks) % kHalfThr == 0, "tile chunks must divide over the staging waves");
  constexpr int kCPT = 2 * kKChunks / kHalfThr;  // K and V chunks per staging thread
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wl = w & 3;  // group 0 produces, group 1 consumes; wl: the query slice
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const float c2 = (float)a.scale * kLog2e;
  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __half* dO = static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq;

  const int wq0 = q0 + 32 * wl;
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;

  // ---- Q, dO blocks into LDS (every thread); the producers read their resident B operands below
  {
    constexpr int kRPT = 2 * D * (kBM / 8) / kThr, kHalf = D * (kBM / 8) / kThr;
    static_assert(kHalf * kThr == D * (kBM / 8), "resident chunks must divide over the workgroup");
    const __amdgpu_buffer_rsrc_t qrs2 = make_rsrc(Q, 2u * d * nq), ors2 = make_rsrc(dO, 2u * vd * nq);
    u32x4 rv[kRPT];
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      const bool in = c < (which ? vd : d) && q0 + 8 * m < nq;
      if constexpr (ALN)
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? ors2 : qrs2,
                                                       in ? (uint32_t)c * (uint32_t)nq * 2u + 16u * m : 0x80000000u, 2 * q0, 0);
      else
        rv[jj] = buf_load8h(which ? ors2 : qrs2, (uint32_t)c * (uint32_t)nq * 2u, q0 + 8 * m, nq, c < (which ? vd : d));
    }
#pragma unroll
    for (int jj = 0; jj < kRPT; ++jj) {
      const int which = jj >= kHalf, j = tid + kThr * (jj - which * kHalf);
      const int c = j / (kBM / 8), m = j % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + which * S::kRow + c * (2 * kBM) + ((m * 16) ^ ((c & 3) << 6))) = rv[jj];
    }
  }
  __syncthreads();

  // ---- key range of this query block (rule-bounded), per-lane / per-wave key intervals (both roles)
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;
  int klo = 0, kspan = nk, wlo_min = 0, wlo_max = 0, whi_min = nk - 1, whi_max = nk - 1;
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
  auto tcls = [&](int ka) -> int {
    const int kz = ka + kBN - 1;
    if (!wave_active) return 0;
    if (POL == 0) return kz < nk ? 2 : 1;
    if (POL == 2) {  // class 2 only for tiles wholly inside nk (the staged tail past nk is masked)
      if (ka >= nk) return 0;
      const int c = tile_class(a.rule, wq0, min(wq0 + 31, nq - 1), ka, min(kz, nk - 1));
      return (c == 2 && kz >= nk) ? 1 : c;
    }
    if (wlo_min > kz || whi_max < ka) return 0;
    return (wlo_max <= ka && whi_min >= kz && kz < nk) ? 2 : 1;
  };
  // hand-over slot of this wave pair: k-steps 0..3 of dSᵀ, one b128 each, lane-linear
  auto xoff = [&](int xs, int j) -> uint32_t { return S::offX + xs * S::kXSlot + wl * S::kXWave + j * 1024 + lane * 16; };
  // Steps it = 0 .. ntiles: the producer handles tile it (it < ntiles), the consumer tile it-1 (it >= 1),
  // in whole groups of four (ring slot it % 4, staging set (it+1) % 2, hand-over slot it % 2 compile-time)
  const int nsteps = ntiles + 1;

  // ---- key-tile staging (K, V chunks: 8 keys of one channel row) by the consumer half of the workgroup
  const int ct = tid & (kHalfThr - 1);
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  uint32_t voff[kCPT];
  int crow_[kCPT];
  const int cm = ct & 7;
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    crow_[j] = ((ct + kHalfThr * j) % kKChunks) >> 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nk * 2u + (ALN ? 16u * cm : 0u);
  }
  u32x4 kr[2][kCPT];  // two staging sets: tile t in set t&1, loaded two steps before it is stored
  auto is_v = [&](int j) -> bool {
    return (kKChunks % kHalfThr == 0) ? (j >= kKChunks / kHalfThr) : ((ct + kHalfThr * j) >= kKChunks);
  };
  auto load_tile = [&](int ka, int set) __attribute__((always_inline)) {
    const bool out = ka + 8 * cm >= nk;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      if constexpr (ALN)
        kr[set][j] = buf_load16(isV ? vrs : krs, voff[j], 2 * min(ka, nk), out || crow_[j] >= (isV ? vd : d));
      else
        kr[set][j] = buf_load8h(isV ? vrs : krs, voff[j], ka + 8 * cm, nk, crow_[j] < (isV ? vd : d));
    }
  };
  auto store_tile = [&](int slot, int set) __attribute__((always_inline)) {
    lds_char_t* base = smem + slot * S::kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isV = is_v(j);
      *reinterpret_cast<lds_u32x4_t*>(base + (isV ? S::offVT : S::offKT) + k2_off(crow_[j], cm)) = kr[set][j];
    }
  };
  // first tiles (after tile 0's loads): the barrier that retires the Q / dO images, tile 0 stored
  auto stage0 = [&]() __attribute__((always_inline)) {
    __syncthreads();
    store_tile(0, 0);
    load_tile(kt0 + kBN, 1);
    load_tile(kt0 + 2 * kBN, 0);
  };
  // resident B operands of the producer, lane (r,h) holds X[c = 16s + 8h + j][q = wq0 + r]: Q' and dO;
  // the row constants likewise
  auto resident = [&](int img, half8* x) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * wl + 16 * (g & 1) + 4 * tp;
        const uint32_t off = crow * (2 * kBM) + ((col * 2) ^ ((crow & 3) << 6));
        const half4 v = tr_read(smem + img * S::kRow + off);
        if (e == 0) x[s].lo = v; else x[s].hi = v;
      }
  };
  auto rowconst = [&](const void* ws, float dflt) -> floatx16 {
    const float* p = static_cast<const float*>(ws) + bi * (int64_t)nq;
    const float v = (qi < nq) ? p[qi] : dflt;
    floatx16 x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = v;
    return x;
  };
  // A-operand (Kᵀ / Vᵀ) read bases, σ-permuted as in the one-wave pass: register i of half t holds
  // key 32t + 16(i>>3) + 8h + (i&7), so k-step s of dSᵀ is keys 16s + 8h + 0..7
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t tb[2][2];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int t = 0; t < 2; ++t) tb[e][t] = k2_off(8 * (g >> 1) + 4 * e + tq, 4 * t + 2 * (g & 1) + (sig >> 1), sig & 1);
  // Sᵀ (or dPᵀ) of key half t: 8 MFMAs over the channels, transposed A reads two k-steps ahead
  auto half_chain = [&](const lds_char_t* img, const half8* bres, floatx16 init, int t) __attribute__((always_inline)) -> floatx16 {
    constexpr int kS = D / 16;
    half8 af[3];
    auto rd = [&](int s_) __attribute__((always_inline)) {
      af[s_ % 3].lo = tr_read(img + tb[0][t] + (16 * s_) * 128);
      af[s_ % 3].hi = tr_read(img + tb[1][t] + (16 * s_) * 128);
    };
    rd(0);
    rd(1);
    floatx16 acc = init;
#pragma unroll
    for (int s_ = 0; s_ < kS; ++s_) {
      if (s_ + 2 < kS) rd(s_ + 2);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s_ % 3], bres[s_], acc, 0, 0, 0);
    }
    return acc;
  };
  const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;  // this lane's query order
  // P of register i of key half t (exp2 of the score, zero outside the rule)
  auto pval = [&](float sv, int cls, int ka, int t, int i) __attribute__((always_inline)) -> float {
    float pv = __builtin_amdgcn_exp2f(sv);
    if (cls == 1) {
      const int kk = ka + 32 * t + 16 * (i >> 3) + 8 * h + (i & 7);
      const bool ok = (POL == 1)   ? ((unsigned)(kk - klo) < (unsigned)kspan)
                      : (POL == 2) ? (kk < nk && check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1))))
                                   : (kk < nk);
      pv = ok ? pv : 0.f;
    }
    return pv;
  };

  if (grp == 0) {
    // ================= producer
    half8 qf[D / 16];
    resident(0, qf);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = scale8(qf[s], c2);
    const floatx16 negl = rowconst(a.ws_lse, kNegInf);
    {
      half8 of[D / 16];
      resident(1, of);
      const floatx16 negd = rowconst(a.ws_D, 0.f);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __syncthreads();  // (stage0 of the consumers)
      auto pstep = [&](auto C_, int it) __attribute__((always_inline)) {
        constexpr int c = decltype(C_)::value;
        __syncthreads();
        const int ka = kt0 + it * kBN;
        const int cls = it < ntiles ? tcls(ka) : 0;
        if (cls == 0) return;
        const lds_char_t* base = smem + c * S::kSlot;
#pragma unroll
        for (int t = 0; t < 2; ++t) {  // one 32-key half at a time: 16 MFMAs, then its two dSᵀ k-steps
          const floatx16 st = half_chain(base + S::offKT, qf, negl, t);
          const floatx16 dp = half_chain(base + S::offVT, of, negd, t);
          auto softmax = [&](int cl) __attribute__((always_inline)) {
#pragma unroll
            for (int sh = 0; sh < 2; ++sh) {
              half8 dsf;
#pragma unroll
              for (int j = 0; j < 8; ++j) dsf[j] = (_Float16)(pval(st[8 * sh + j], cl, ka, t, 8 * sh + j) * dp[8 * sh + j]);
              *reinterpret_cast<lds_half8_t*>(smem + xoff(c % 2, 2 * t + sh)) = dsf;
            }
          };
          // the edge-tile mask as a real branch (see the dK/dV pass)
          if (cls == 1) {
            asm volatile("; edge tile" ::: );
            softmax(1);
          } else {
            asm volatile("; interior tile" ::: );
            softmax(2);
          }
        }
      };
      for (int it = 0; it < nsteps; it += 4) {
        pstep(IC<0>{}, it);
        pstep(IC<1>{}, it + 1);
        pstep(IC<2>{}, it + 2);
        pstep(IC<3>{}, it + 3);
      }
      return;
    }
  }

  // ================= consumer: dQ += K·dSᵀ for tile it-1; it stages the key tiles
  load_tile(kt0, 0);
  stage0();
  floatx16 dq[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[u][i] = 0.f;
  uint32_t kb2[4];  // dQ A operand: row 32u + r (+32u·128: immediate), chunk 2s + h
#pragma unroll
  for (int s = 0; s < 4; ++s) kb2[s] = k2_off(r, 2 * s + h);

  auto cwork = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    const int ka = kt0 + (it - 1) * kBN;
    const int cls = (it >= 1 && it - 1 < ntiles) ? tcls(ka) : 0;
    if (cls == 0) return;
    const lds_char_t* base = smem + ((c + 3) % 4) * S::kSlot;
    half8 dsf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) dsf[s] = read_b128(smem + xoff((c + 1) % 2, s));
    constexpr int kN = 4 * (D / 32);
    half8 ka8p[3];
    auto rka = [&](int n) __attribute__((always_inline)) {  // operand n = (D/32)·s + u, two ahead
      ka8p[n % 3] = read_b128(base + S::offKT + kb2[n / (D / 32)] + 32 * (n % (D / 32)) * 128);
    };
    rka(0);
    rka(1);
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      if (n + 2 < kN) rka(n + 2);
      const int s = n / (D / 32), u = n % (D / 32);
      dq[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka8p[n % 3], dsf[s], dq[u], 0, 0, 0);
    }
  };
  // one step: the barrier, tile it+1 stored (loaded in step it-2), tile it+3 loaded into the set just
  // stored (unconditional: past the end they move zeros into a slot nobody reads, so the vmcnt waits
  // stay exact), then dQ += K·dSᵀ of tile it-1
  auto cstep = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    __syncthreads();
    store_tile((c + 1) % 4, (c + 1) % 2);
    load_tile(kt0 + kBN * (it + 3), (c + 1) % 2);
    cwork(C_, it);
  };
  for (int it = 0; it < nsteps; it += 4) {
    cstep(IC<0>{}, it);
    cstep(IC<1>{}, it + 1);
    cstep(IC<2>{}, it + 2);
    cstep(IC<3>{}, it + 3);
  }

  if (!wave_active || qi >= nq) return;
  __half* dQ = static_cast<__half*>(a.dQ) + bi * (int64_t)d * nq;
  const float sc = (float)a.scale;
  if (d == D) {  // one buffer store per value (see the dK/dV pass)
    const __amdgpu_buffer_rsrc_t qrs_ = make_rsrc(dQ, 2u * d * nq);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
    for (int u = 0; u < D / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(dq[u][i] * sc)), qrs_, vlane,
                                              2u * (32u * u + (i & 3) + 8u * (i >> 2)) * (uint32_t)nq, 0);
    return;
  }
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (c < d) dQ[(int64_t)c * nq + qi] = __float2half(dq[u][i] * sc);
    }
}

// kernel POL from the rule: 0 full, 1 interval rules (causal, 1d unit-stride local), 2 any other local rule
inline int bwd_pol(const Rule& r) { return r.policy == 0 ? 0 : rule_is_interval(r) ? 1 : 2; }
// 16-B chunk staging: every tensor 16-B aligned and both lengths multiples of 8 (each channel row starts
// on a 16-B boundary)
inline bool bwd_aligned(const BwdArgs& a) {
  const uintptr_t al = reinterpret_cast<uintptr_t>(a.Q) | reinterpret_cast<uintptr_t>(a.K) |
                       reinterpret_cast<uintptr_t>(a.V) | reinterpret_cast<uintptr_t>(a.dO);
  return (al % 16) == 0 && a.rule.q.n % 8 == 0 && a.rule.k.n % 8 == 0;
}
using BwdKernel = void (*)(BwdArgs);

template <int D, int NW, int WPE>
hipError_t launch_dkdv(const BwdArgs& a, hipStream_t s) {
  using S = DkdvSmem<D, NW>;
  const int64_t nkb = (a.rule.k.n + S::kBK - 1) / S::kBK;
  const int pol = bwd_pol(a.rule);
  const BwdKernel kern =
      bwd_aligned(a) ? (pol == 0   ? bwd_dkdv_kernel<D, NW, WPE, 0, true>
                        : pol == 1 ? bwd_dkdv_kernel<D, NW, WPE, 1, true>
                                   : bwd_dkdv_kernel<D, NW, WPE, 2, true>)
                     : (pol == 0   ? bwd_dkdv_kernel<D, NW, WPE, 0, false>
                        : pol == 1 ? bwd_dkdv_kernel<D, NW, WPE, 1, false>
                                   : bwd_dkdv_kernel<D, NW, WPE, 2, false>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(NW * 64), S::kTotal, s, a);
  return hipGetLastError();
}

template <int D>
hipError_t launch_dkdv_pc(const BwdArgs& a, hipStream_t s) {
  using S = PcSmem<D>;
  const int64_t nkb = (a.rule.k.n + S::kBK - 1) / S::kBK;
  const int pol = bwd_pol(a.rule);
  const BwdKernel kern = bwd_aligned(a) ? (pol == 0   ? bwd_dkdv_pc_kernel<D, 0, true>
                                           : pol == 1 ? bwd_dkdv_pc_kernel<D, 1, true>
                                                      : bwd_dkdv_pc_kernel<D, 2, true>)
                                        : (pol == 0   ? bwd_dkdv_pc_kernel<D, 0, false>
                                           : pol == 1 ? bwd_dkdv_pc_kernel<D, 1, false>
                                                      : bwd_dkdv_pc_kernel<D, 2, false>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(512), S::kTotal, s, a);
  return hipGetLastError();
}

template <int D, int NW, int WPE, bool PRE = false, bool MSPEC = false>
hipError_t launch_dq(const BwdArgs& a, hipStream_t s) {
  using S = DqSmem<D, NW>;
  const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
  const int pol = bwd_pol(a.rule);
  const BwdKernel kern = bwd_aligned(a) ? (pol == 0   ? bwd_dq_kernel<D, NW, WPE, 0, true, PRE, MSPEC>
                                           : pol == 1 ? bwd_dq_kernel<D, NW, WPE, 1, true, PRE, MSPEC>
                                                      : bwd_dq_kernel<D, NW, WPE, 2, true, PRE, MSPEC>)
                                        : (pol == 0   ? bwd_dq_kernel<D, NW, WPE, 0, false, PRE, MSPEC>
                                           : pol == 1 ? bwd_dq_kernel<D, NW, WPE, 1, false, PRE, MSPEC>
                                                      : bwd_dq_kernel<D, NW, WPE, 2, false, PRE, MSPEC>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(NW * 64), S::kTotal, s, a);
  return hipGetLastError();
}

// 128 < max(d, v_d) <= 256, any alignment and length (the ALN = false instances stage element-wise):
// the passes at D = 256
// OC / OCQ = 0: the four-role dK / dV / dQ passes; > 0: the one-wave passes on that many output-channel
// chunks (round 4's structure, FA_BWD_VARIANT=1421)
template <int OC = 0, int OCQ = 0>
hipError_t launch_bwd_wide(const BwdArgs& a, hipStream_t s) {
  constexpr int D = 256, NW = 4;
  const int pol = bwd_pol(a.rule);
  if constexpr (OC == 0) {  // the four-role pass: S / dP formed once per pair
    using S = W4Smem;
    const int64_t nkb = (a.rule.k.n + S::kBK - 1) / S::kBK;
    const bool aln = bwd_aligned(a);
    const BwdKernel kern = aln ? (pol == 0   ? bwd_dkdv_w4_kernel<0, true>
                                  : pol == 1 ? bwd_dkdv_w4_kernel<1, true>
                                             : bwd_dkdv_w4_kernel<2, true>)
                               : (pol == 0   ? bwd_dkdv_w4_kernel<0, false>
                                  : pol == 1 ? bwd_dkdv_w4_kernel<1, false>
                                             : bwd_dkdv_w4_kernel<2, false>);
    hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(512), S::kTotal, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  } else {
    using S = DkdvSmem<D, NW>;
    const int64_t nkb = (a.rule.k.n + S::kBK - 1) / S::kBK;
    const BwdKernel kern = pol == 0   ? bwd_dkdv_kernel<D, NW, 1, 0, true, OC>
                           : pol == 1 ? bwd_dkdv_kernel<D, NW, 1, 1, true, OC>
                                      : bwd_dkdv_kernel<D, NW, 1, 2, true, OC>;
    hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb * OC)), dim3(NW * 64), S::kTotal, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if constexpr (OCQ == 0) {  // the four-role pass: Sᵀ / dPᵀ formed once per pair
    using S = W4DqSmem;
    const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
    const bool aln = bwd_aligned(a);
    const BwdKernel kern = aln ? (pol == 0   ? bwd_dq_w4_kernel<0, true>
                                  : pol == 1 ? bwd_dq_w4_kernel<1, true>
                                             : bwd_dq_w4_kernel<2, true>)
                               : (pol == 0   ? bwd_dq_w4_kernel<0, false>
                                  : pol == 1 ? bwd_dq_w4_kernel<1, false>
                                             : bwd_dq_w4_kernel<2, false>);
    hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(512), S::kTotal, s, a);
    return hipGetLastError();
  } else {
    using S = DqSmem<D, NW>;
    const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
    const BwdKernel kern = pol == 0   ? bwd_dq_kernel<D, NW, 1, 0, true, false, false, OCQ, true>
                           : pol == 1 ? bwd_dq_kernel<D, NW, 1, 1, true, false, false, OCQ, true>
                                      : bwd_dq_kernel<D, NW, 1, 2, true, false, false, OCQ, true>;
    hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb * OCQ)), dim3(NW * 64), S::kTotal, s, a);
    return hipGetLastError();
  }
}

template <int D>
hipError_t launch_dq_pc(const BwdArgs& a, hipStream_t s) {
  using S = DqPcSmem<D>;
  const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
  const int pol = bwd_pol(a.rule);
  const BwdKernel kern = bwd_aligned(a) ? (pol == 0   ? bwd_dq_pc_kernel<D, 0, true>
                                           : pol == 1 ? bwd_dq_pc_kernel<D, 1, true>
                                                      : bwd_dq_pc_kernel<D, 2, true>)
                                        : (pol == 0   ? bwd_dq_pc_kernel<D, 0, false>
                                           : pol == 1 ? bwd_dq_pc_kernel<D, 1, false>
                                                      : bwd_dq_pc_kernel<D, 2, false>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), S::kTotal);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(512), S::kTotal, s, a);
  return hipGetLastError();
}

}  // namespace

bool bwd_f16_fast_supported(const BwdArgs& a) {
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  // (buffer offsets are 32-bit: a channel row set of one slice stays below 2^31 bytes; the element-wise
  // staging of the unaligned form addresses up to 2·n + 14 bytes past a row start)
  return dm >= 1 && dm <= 256 && nq > 0 && nk > 0 &&
         (int64_t)dm * (nq + 8) * 2 < (1ll << 31) &&
         (int64_t)dm * (nk + 8) * 2 < (1ll << 31) && a.b * ((nk + 127) / 128) * 2 < (1ll << 31) &&
         a.b * ((nq + 127) / 128) * 2 < (1ll << 31);
}

hipError_t launch_bwd_f16_fast(const BwdArgs& a, hipStream_t s) {
  const int64_t nrows = a.b * (int64_t)a.rule.q.n;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool prep8 = (a.rule.q.n % 8) == 0 && al16(a.O) && al16(a.dO) && al16(a.ws_D) && al16(a.ws_lse);
#ifdef FA_DIAG
  if (diag_variant("FA_BWD_VARIANT") == 1430) prep8 = false;  // the one-query-a-thread prep, for A/B
#endif
  if (prep8)
    hipLaunchKernelGGL(bwd_prep8_kernel, dim3((unsigned)((nrows / 8 + kThrPrep - 1) / kThrPrep)), dim3(kThrPrep), 0, s, a);
  else
    hipLaunchKernelGGL(bwd_prep_kernel, dim3((unsigned)((nrows + kThrPrep - 1) / kThrPrep)), dim3(kThrPrep), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
#ifdef FA_DIAG
  // FA_BWD_VARIANT=1421: round 4's D = 256 dK/dV pass (two 128-channel chunks, S / dP formed in each)
  if (max(a.d, a.v_d) > 128 && bwd_aligned(a) && diag_variant("FA_BWD_VARIANT") == 1421) return launch_bwd_wide<2, 2>(a, s);
#endif
  if (max(a.d, a.v_d) > 128) return launch_bwd_wide(a, s);
#ifdef FA_DIAG
  // FA_BWD_VARIANT (diagnostic library): d <= 64 — 82 eight-wave blocks, 1068 / 1069 the dQ pass's
  // operand reads run ahead, 1071 its edge mask as a branch; d = 128 — 1599 the one-wave dQ pass (the
  // unaligned shapes' structure) on aligned shapes.  The other A/B variants of rounds 2-4 (stamp
  // builds, LDS-DMA staging, the four-role dK/dV pass) were measured and removed.
  const int v = diag_variant("FA_BWD_VARIANT");
  if (max(a.d, a.v_d) <= 64 && v >= 0) {
    e = v == 82 ? launch_dkdv<64, 8, 2>(a, s) : launch_dkdv<64, 4, 2>(a, s);
    if (e != hipSuccess) return e;
    switch (v) {
      case 82: return launch_dq<64, 8, 2, false, true>(a, s);
      case 1068: case 1069: return launch_dq<64, 4, 2, true>(a, s);
      case 1071: return launch_dq<64, 4, 2>(a, s);
      default: return launch_dq<64, 4, 2, false, true>(a, s);
    }
  }
  if (max(a.d, a.v_d) > 64 && v >= 1700 && v < 1800 && bwd_dkdv_k64_supported(a)) {  // the 64-keys-a-wave dK/dV pass
    e = launch_dkdv_k64(a, s);
    if (e != hipSuccess) return e;
    return launch_dq_pc<128>(a, s);
  }
  if (max(a.d, a.v_d) > 64 && v >= 0) {
    e = launch_dkdv_pc<128>(a, s);
    if (e != hipSuccess) return e;
    if (v == 1599 || !bwd_aligned(a)) return launch_dq<128, 4, 1, true>(a, s);
    return launch_dq_pc<128>(a, s);
  }
#endif
  if (max(a.d, a.v_d) <= 64) {
    e = launch_dkdv<64, 4, 2>(a, s);
    if (e != hipSuccess) return e;
    // (the d <= 64 dQ pass keeps the if-converted edge mask: the branch form spills 8-42 VGPRs there)
    return launch_dq<64, 4, 2, false, true>(a, s);
  }
  // tuned (c3): the producer / consumer dK/dV pass (one-process A/B: 9.20 -> 8.59 ms backward; two
  // barriers per step, 1402, and a prioritised producer, 1401, measured 8.70 / 8.77) and, for 16-B
  // chunk staging, the producer / consumer dQ pass (8.58 -> 8.36 ms backward, gradients bit-identical;
  // its element-wise staging form spills, so other shapes keep the one-wave pass with operand reads
  // two MFMA pairs ahead: 10.97 -> 9.93 ms backward before)
  e = launch_dkdv_pc<128>(a, s);
  if (e != hipSuccess) return e;
  if (bwd_aligned(a)) return launch_dq_pc<128>(a, s);
  return launch_dq<128, 4, 1, true>(a, s);
}

}  // namespace fa
