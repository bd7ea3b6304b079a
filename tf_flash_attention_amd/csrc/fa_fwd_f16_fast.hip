// fa_fwd_f16_fast.hip — fp16 fused attention forward, streamlined main loop for
// the common shapes (32 < max(d, v_d) <= 128, channels zero-padded to D ∈ {64, 128};
// K/V rows 16-byte aligned, nk % 8 == 0) under the full policy and the interval
// rules (causal, 1d unit-stride local).
//
// Same algorithm and operand layouts as fa_fwd_f16.hip (which remains the path
// for every other shape and for strided / 2d local rules); what differs is how
// the key loop is laid out for the gfx950 issue port:
//   * K and V have separate LDS rings of 2·TPB tiles, filled TPB tiles per barrier
//     (TPB = tiles per barrier).  Tile `it` reads K(it+1) (for the Sᵀ MFMAs of the
//     next tile) and V(it) (for its own PV MFMAs); each barrier phase writes the
//     K and V tiles the previous phase finished with.  The loop is unrolled over
//     the ring so every LDS address is a lane constant plus an immediate;
//   * K/V tiles are fetched with buffer loads (one SGPR descriptor per slice,
//     the tile offset in soffset): no per-tile address VALU;
//   * K fragments are read right after the barrier, V fragments after the
//     rebase decision (LDS latency overlaps the Sᵀ MFMAs / the row max);
//   * the Sᵀ MFMAs of tile it+1 share a basic block with the row max of tile it;
//     the exponentials of tile it interleave with its PV MFMAs;
//   * full tiles take a branch-free path; only mixed tiles (rule edge / nk tail)
//     evaluate a per-element mask.
// Replaces the reference's ForwardImpl (flash_attention.cu:425-1077) for these
// shapes; numerics (fp32 accumulation, lazy log2-domain rescale, l relative to
// the stored fp16 m) are identical to fa_fwd_f16.hip.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

#include <stdlib.h>

namespace fa {
namespace {

using namespace mf;

constexpr int kBN = 64;             // keys per tile
constexpr int kVPad = 1;            // V group row padding, in 16-byte rows
constexpr float kRescaleThr = 8.f;  // log2 units (cdna_hip_programming.md T13)

// structure flags of the shipped instances (the launcher picks them per shape class)
constexpr int kFPrio = 2;    // s_setprio 1 for the second half of the waves (guide T5, static form)
constexpr int kFLateV = 4;   // read the V fragments after the rebase decision (shorter live range)
constexpr int kFTpb2 = 8;    // two key tiles per barrier (ring of 4 tiles for K and for V)

template <int D, int NW, int TPB>
struct FastSmem {
  static constexpr int kBM = 32 * NW;               // query rows per workgroup
  static constexpr int kQRow = 2 * kBM;             // bytes per Q row
  static constexpr int kQ = D * kQRow;              // Q [D][BM] halfs
  static constexpr int kK = D * kBN * 2;            // K tile [D][64] halfs, 128-B rows
  static constexpr int kV = 8 * (D + kVPad) * 16;   // V tile [8 groups][D+pad][8] halfs
  static constexpr int kNS = 2 * TPB;               // ring slots (K and V each)
  static constexpr int offK = kQ;
  static constexpr int offV = kQ + kNS * kK;
  static constexpr int kTotal = kQ + kNS * (kK + kV);
};

constexpr int fast_waves_per_eu(int D) { return D >= 128 ? 1 : 2; }

// One workgroup = NW waves; each wave owns 32 queries of one (batch, head) slice
// and sweeps the key tiles its rule allows.
//   POL 0: full policy (only the nk tail tile is masked)
//       1: interval rules (causal, 1d unit-stride local): per-lane key interval,
//          tile class from the wave's bounds, skipped tiles cost nothing.
template <int D, int NW, int POL, int F>
__global__ __launch_bounds__(NW * 64, fast_waves_per_eu(D)) void fwd_f16_fast_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr int TPB = (F & kFTpb2) ? 2 : 1;
  using S = FastSmem<D, NW, TPB>;
  constexpr int NS = S::kNS;
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

  // channels d (Q/K) and v_d (V/O) may be smaller than D: rows past them are staged as zeros
  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;

  // ---- key range of this query block (rule-bounded)
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;

  // ---- staging: chunk j of this thread = 8 keys of channel row c
  uint32_t voff[kCPT], kwo[kCPT], vwo[kCPT];
  int crow[kCPT];
  const int cm = tid & 7;  // chunk index within the 64-key row (same for every j)
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int c = (tid + kThr * j) >> 3;
    crow[j] = c;
    voff[j] = (uint32_t)c * (uint32_t)nk * 2u + 16u * cm;
    kwo[j] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));  // K: 64-B halves swapped on rows with c&2
    // V: group (s, h) = keys {16s + 4h + 0..3, 16s + 8 + 4h + 0..3}, [v][8 keys] rows, so one
    // ds_read_b128 is a PV A operand; chunk cm = keys 8cm..8cm+7 -> groups (cm/2, 0) and (cm/2, 1)
    vwo[j] = ((2 * (cm >> 1)) * (D + kVPad) + c) * 16 + (cm & 1) * 8;
  }
  // register staging: TPB K tiles and TPB V tiles loaded one barrier phase ahead of their store
  u32x4 kr[TPB][kCPT], vr[TPB][kCPT];
  // chunks past nk (tail tile) or past the tensor's channel count read as zeros (offset beyond
  // the descriptor's range)
  auto load_into = [&](u32x4 (&dst)[kCPT], __amdgpu_buffer_rsrc_t rs, int k0, int rows) {
    if (k0 + kBN <= nk && rows == D) {
#pragma unroll
      for (int j = 0; j < kCPT; ++j) dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[j], 2 * k0, 0);
    } else {
      const bool out = k0 + 8 * cm >= nk;
#pragma unroll
      for (int j = 0; j < kCPT; ++j) dst[j] = buf_load16(rs, voff[j], 2 * k0, out || crow[j] >= rows);
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

  // ---- prologue: K(0..TPB), V(0..TPB-1) into the ring, K(TPB+1..2TPB) / V(TPB..2TPB-1) into
  //      the staging registers; all in flight together with the Q tile
  {
    u32x4 pk[TPB + 1][kCPT], pv[TPB][kCPT];
#pragma unroll
    for (int x = 0; x <= TPB; ++x)
      if (x < ntiles) load_into(pk[x], krs, kt0 + x * kBN, d);
#pragma unroll
    for (int x = 0; x < TPB; ++x)
      if (x < ntiles) load_into(pv[x], vrs, kt0 + x * kBN, vd);
    // Q [D][BM], 64-B blocks XOR-swizzled by c&3: all of a thread's chunks loaded before any is
    // stored (a rolled loop serialised D/16 memory latencies in every block's prologue)
    constexpr int kQPT = D * (kBM / 8) / kThr;
    static_assert(kQPT * kThr == D * (kBM / 8), "Q chunks must divide over the workgroup");
    u32x4 qv[kQPT];
    if (qvec) {  // branch-free buffer loads (chunks past d or nq read as zeros)
      const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Q, 2u * d * nq);
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int idx = tid + j * kThr, c = idx / (kBM / 8), m = idx % (kBM / 8);
        const bool in = c < d && q0 + 8 * m < nq;
        qv[j] = __builtin_amdgcn_raw_buffer_load_b128(qrs, in ? (uint32_t)c * (uint32_t)nq * 2u + 16u * m : 0x80000000u,
                                                      2 * q0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int idx = tid + j * kThr, c = idx / (kBM / 8), m = idx % (kBM / 8);
        qv[j] = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, false) : u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
      const int idx = tid + j * kThr, c = idx / (kBM / 8), m = idx % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + c * S::kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[j];
    }
#pragma unroll
    for (int x = 0; x <= TPB; ++x)
      if (x < ntiles) store_k(x, pk[x]);
#pragma unroll
    for (int x = 0; x < TPB; ++x)
      if (x < ntiles) store_v(x, pv[x]);
#pragma unroll
    for (int x = 0; x < TPB; ++x) {
      if (TPB + 1 + x < ntiles) load_into(kr[x], krs, kt0 + (TPB + 1 + x) * kBN, d);
      if (TPB + x < ntiles) load_into(vr[x], vrs, kt0 + (TPB + x) * kBN, vd);
    }
  }
  __syncthreads();

  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r]
  half8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
      const int col = 32 * w + 16 * (g & 1) + 4 * tp;
      const half4 t = tr_read(smem + crow * S::kQRow + ((col * 2) ^ ((crow & 3) << 6)));
      if (e == 0) qf[s].lo = t; else qf[s].hi = t;
    }
    qf[s] = scale8(qf[s], c2);
  }

  const int wq0 = q0 + 32 * w;
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;
  // POL 1: this lane's allowed keys [klo, klo + kspan) and the wave's bounds on them
  // (both interval ends are non-decreasing in the query, so the first / last valid lane bound them)
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
    if (POL == 0) return (k1 < nk && wq0 + 32 <= nq) ? 2 : 1;
    if (wlo_min > k1 || whi_max < k0) return 0;
    return (wlo_max <= k0 && whi_min >= k1 && k1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants; every read is base + immediate)
  //   K: element (crow, col) of [D][64] at crow*128 + ((2*col) ^ ((crow & 2) << 5)); crow&2 == tq&2
  const uint32_t kbase0 = (8 * (g >> 1) + tq) * 128 + (((16 * (g & 1) + 4 * tp) * 2) ^ ((tq & 2) << 5));
  const uint32_t kbase1 = (8 * (g >> 1) + tq) * 128 + (((32 + 16 * (g & 1) + 4 * tp) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r,h) reads group (s, h), channel row 32u + r
  const uint32_t vbase = (h * (D + kVPad) + r) * 16;

  floatx16 acc_o[D / 32];
#pragma unroll
  for (int u = 0; u < D / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_o[u][i] = 0.f;
  // m_run: lazily moved softmax reference (log2 units) that l_run / acc_o are relative to;
  // negm = -m_run broadcast (the C operand of every Sᵀ chain); m_max: exact row max.
  // thr: rescale trigger — -FLT_MAX until the lane's first allowed key seeds m_run, then
  // kRescaleThr, so the per-tile test is one compare.
  // pend: a rebase of tile it moved m_run after the Sᵀ MFMAs of tile it+1 were issued against
  // the old value; tile it+1 subtracts it when it becomes current (rare; keeps the in-flight
  // accumulators out of the rebase branch)
  float m_run = 0.f, l_run = 0.f, l_run2 = 0.f, m_max = kNegInf, thr = -__FLT_MAX__, pend = 0.f;
  floatx16 negm;
#pragma unroll
  for (int i = 0; i < 16; ++i) negm[i] = 0.f;

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
      for (int u = 0; u < D / 32; ++u) vf[s][u] = read_b128(vb_ + ((2 * s) * (D + kVPad) + 32 * u) * 16);
  };
  auto qk = [&](const half8 (&kf)[2][D / 16], floatx16 (&st)[2]) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qf[s], s == 0 ? negm : st[t], 0, 0, 0);
  };
  // per-element rule / tail mask of a mixed tile
  auto mask = [&](int k0, floatx16 (&st)[2]) {
    const int base = k0 + 4 * h - klo;
    const bool qok = qi < nq;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = 32 * t + (i & 3) + 8 * (i >> 2);
        const bool ok = (POL == 1) ? ((unsigned)(base + off) < (unsigned)kspan) : (qok && (k0 + off + 4 * h < nk));
        st[t][i] = ok ? st[t][i] : kNegInf;
      }
  };
  // row max of tile `st` (lanes l and l^32 together)
  auto rowmax = [&](floatx16 (&st)[2]) -> float {
    float mx0 = fmaxf(st[0][0], st[0][1]), mx1 = fmaxf(st[1][0], st[1][1]);
#pragma unroll
    for (int i = 2; i < 16; i += 2) {
      mx0 = fmaxf(fmaxf(mx0, st[0][i]), st[0][i + 1]);
      mx1 = fmaxf(fmaxf(mx1, st[1][i]), st[1][i + 1]);
    }
    const float mt = max_pair32(fmaxf(mx0, mx1));
    m_max = fmaxf(m_max, m_run + mt);
    return mt;
  };
  // lazy rebase (rare): after it exp2(st) are the tile's probabilities relative to m_run
  auto rebase = [&](float mt, floatx16 (&st)[2], bool has_next) {
    if (__any(mt > thr)) {  // rare: seed, or the tile max moved past the threshold
      const bool unset = thr < 0.f;
      const bool seed = unset && (mt > thr);
      const float delta = unset ? (seed ? mt : 0.f) : fmaxf(mt, 0.f);
      const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
      m_run += delta;
      thr = (unset && !seed) ? thr : kRescaleThr;
      l_run *= alpha;
      l_run2 *= alpha;
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
      pend = has_next ? delta : 0.f;  // the next tile's in-flight scores used the old m_run
    }
  };
  // P = exp2(st) (fp16) as the B operand of Oᵀ = V·Pᵀ; row sums; PV MFMAs
  auto exp_pv = [&](floatx16 (&st)[2], const half8 (&vf)[4][D / 32]) {
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 pf;
#pragma unroll
      for (int x = 0; x < 8; ++x) pf[x] = (_Float16)__builtin_amdgcn_exp2f(st[s >> 1][8 * (s & 1) + x]);
#pragma unroll
      for (int x = 0; x < 8; x += 4) {
        l_run = __builtin_amdgcn_fdot2(half2v{pf[x], pf[x + 1]}, one2, l_run, false);
        l_run2 = __builtin_amdgcn_fdot2(half2v{pf[x + 2], pf[x + 3]}, one2, l_run2, false);
      }
#pragma unroll
      for (int u = 0; u < D / 32; ++u) acc_o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], pf, acc_o[u], 0, 0, 0);
    }
  };

  // ---- S(0)
  floatx16 stA[2], stB[2];
  if (ntiles > 0 && tcls(kt0) != 0) {
    half8 kf[2][D / 16];
    read_k(0, kf);
    qk(kf, stA);
  }

  // tile it (c = it mod NS, static after the unroll): K(it+1) in slot (c+1)%NS, V(it) in slot c.
  // A barrier phase starts at every tile with c % TPB == 0 (phase tiles it..it+TPB-1) and
  //   stores K(it+TPB+1 .. it+2TPB) into slots (c+TPB+1 .. c+2TPB)%NS  (read in the previous phase),
  //   stores V(it+TPB .. it+2TPB-1) into slots (c+TPB .. c+2TPB-1)%NS   (read in the previous phase),
  //   loads K(it+2TPB+1 ..) and V(it+2TPB ..) into the staging registers (stored next phase).
  // Order within a tile: [mask(it) if mixed] [Sᵀ MFMAs of it+1 beside the row max of it]
  //                      [rare rebase] [V reads] [exp2 / convert / row sums of it beside its PV MFMAs]
  auto step = [&](auto C_, int it, floatx16 (&cur)[2], floatx16 (&nxt)[2]) {
    constexpr int c = decltype(C_)::value;
    if (c % TPB == 0) {
      __syncthreads();
#pragma unroll
      for (int x = 0; x < TPB; ++x) {
        if (it + TPB + 1 + x < ntiles) store_k((c + TPB + 1 + x) % NS, kr[x]);
        if (it + TPB + x < ntiles) store_v((c + TPB + x) % NS, vr[x]);
      }
#pragma unroll
      for (int x = 0; x < TPB; ++x) {
        if (it + 2 * TPB + 1 + x < ntiles) load_into(kr[x], krs, kt0 + (it + 2 * TPB + 1 + x) * kBN, d);
        if (it + 2 * TPB + x < ntiles) load_into(vr[x], vrs, kt0 + (it + 2 * TPB + x) * kBN, vd);
      }
    }
    const int k0 = kt0 + it * kBN;
    const int ccur = tcls(k0);
    const bool has_next = it + 1 < ntiles;
    const int cnxt = has_next ? tcls(k0 + kBN) : 0;
    half8 kf[2][D / 16];
    half8 vf[4][D / 32];
    if (cnxt != 0) read_k((c + 1) % NS, kf);
    if (ccur != 0 && !(F & kFLateV)) read_v(c, vf);
    if (__any(pend != 0.f)) {  // rare: this tile's scores predate the last rebase
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        cur[0][i] -= pend;
        cur[1][i] -= pend;
      }
      pend = 0.f;
    }
    if (ccur == 1) mask(k0, cur);
    float mt = 0.f;
    if (cnxt != 0 && ccur != 0) {  // one basic block: next tile's MFMAs beside this tile's max
      qk(kf, nxt);
      mt = rowmax(cur);
    } else {
      if (cnxt != 0) qk(kf, nxt);
      if (ccur != 0) mt = rowmax(cur);
    }
    if (ccur != 0) {
      rebase(mt, cur, cnxt != 0);
      if (F & kFLateV) read_v(c, vf);
      exp_pv(cur, vf);
    }
  };
  for (int it = 0; it < ntiles; it += NS) {
    step(IC<0>{}, it, stA, stB);
    if (it + 1 < ntiles) step(IC<1>{}, it + 1, stB, stA);
    if (NS > 2) {
      if (it + 2 < ntiles) step(IC<2 % NS>{}, it + 2, stA, stB);
      if (it + 3 < ntiles) step(IC<3 % NS>{}, it + 3, stB, stA);
    }
  }

  if (!wave_active) return;
  const float l_tot = sum_pair32(l_run + l_run2);
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi < nq) {
    __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
    if (vd == D) {  // one buffer store per value, no per-store address / predicate (see the ping-pong kernel)
      const __amdgpu_buffer_rsrc_t ors = make_rsrc(O, 2u * vd * nq);
      const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t cst = 32u * u + (i & 3) + 8u * (i >> 2);
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(acc_o[u][i] * inv)), ors,
                                                vlane, 2u * cst * (uint32_t)nq, 0);
        }
    } else {
#pragma unroll
      for (int u = 0; u < D / 32; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (v < vd) O[(int64_t)v * nq + qi] = __float2half(acc_o[u][i] * inv);
        }
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
hipError_t launch_fast_t(const FwdArgs& a, hipStream_t s) {
  using S = FastSmem<D, NW, (F & kFTpb2) ? 2 : 1>;
  const int64_t nqb = (a.rule.q.n + S::kBM - 1) / S::kBM;
  const int smem = S::kTotal;
  auto kern = a.rule.policy == 0 ? fwd_f16_fast_kernel<D, NW, 0, F> : fwd_f16_fast_kernel<D, NW, 1, F>;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(NW * 64), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool fwd_f16_fast_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return dm > 32 && dm <= 128 && (nk % 8 == 0) && nk > 0 &&
         (int64_t)dm * nk * 2 < (1ll << 31) && (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) &&
         (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) &&
         rule_is_interval(a.rule) && a.b * ((a.rule.q.n + 127) / 128) < (1ll << 31);
}

hipError_t launch_fwd_f16_fast(const FwdArgs& a, hipStream_t s) {
  const bool d64 = max(a.d, a.v_d) <= 64;
#ifdef FA_DIAG
  // FA_FWD_VARIANT forces one of the shipped structures onto a shape the dispatcher would send
  // elsewhere (parity coverage of every rule each accepts): 1814 / 146 the 8-wave / 4-wave
  // instances below, 2200 / 2301 the ping-pong kernels, 2000 the paired-block study (csrc/diag/)
  const int v = diag_variant("FA_FWD_VARIANT");
  if (fwd_f16_pp_supported(a) && v >= 2000 && v < 2200) return launch_fwd_f16_pp(a, s);  // 21xx: its ablations
  if (fwd_f16_pingpong_supported(a) && v == 2200) return launch_fwd_f16_pingpong(a, s);
  if (fwd_f16_gap_supported(a) && v >= 2600 && v < 2700) return launch_fwd_f16_gap(a, s);  // 26xx: its ablations
  if (fwd_f16_gap128_supported(a) && v >= 2700 && v < 2800) return launch_fwd_f16_gap128(a, s);
  if (fwd_f16_pingpong128_supported(a) && v == 2301) return launch_fwd_f16_pingpong128(a, s);
  if (d64 && v == 1814) return launch_fast_t<64, 8, kFPrio | kFLateV | kFTpb2>(a, s);
  if (v == 146) return d64 ? launch_fast_t<64, 4, kFPrio | kFLateV>(a, s) : launch_fast_t<128, 4, kFPrio | kFLateV>(a, s);
  const bool tuned = v < 0;
  if (v >= 2400 && v < 2500 && fwd_f16_band_supported(a)) return launch_fwd_f16_band(a, s);
#else
  constexpr bool tuned = true;
#endif
  // 1d local windows at d <= 64: the persistent band kernel (no per-block start / end cost)
  if (tuned && fwd_f16_band_supported(a)) return launch_fwd_f16_band(a, s);
  // ping-pong kernel (two wave groups alternating MFMA / softmax phases): the default for
  // d <= 64 under the full policy (c2: 948 vs 904 TF/s for the 8-wave kernel below)
  if (tuned && a.rule.policy == 0 && fwd_f16_pingpong_supported(a)) return launch_fwd_f16_pingpong(a, s);
  // d in (64, 128], full and causal policies: the one-wave gap-stream kernel (c3 forward 2.29 against
  // 2.40 ms for the ping-pong below, full policy at c3's shape 3.95 against 4.34: DESIGN.md §3.0b), then the
  // ping-pong (c3 forward: 2.52 vs 3.16 ms for the 4-wave kernel below) where it does not fit; local windows
  // keep the 4-wave blocks
  if (tuned && a.rule.policy != 2 && fwd_f16_gap128_supported(a)) return launch_fwd_f16_gap128(a, s);
  if (tuned && a.rule.policy != 2 && fwd_f16_pingpong128_supported(a)) return launch_fwd_f16_pingpong128(a, s);
  if (d64) {
    // tuned on MI355X: full-length key loops 8 waves x 32 queries, two key tiles per barrier;
    // rule-bounded short loops (local windows, c4) 4-wave blocks with one tile per barrier
    // (48 KB of LDS) so two blocks per CU cover each other's prologue / epilogue
    if (a.rule.policy == 2) return launch_fast_t<64, 4, kFPrio | kFLateV>(a, s);
    return launch_fast_t<64, 8, kFPrio | kFLateV | kFTpb2>(a, s);
  }
  // tuned (c3 forward, MI355X): 4 waves (one per SIMD), static priority, late V reads
  return launch_fast_t<128, 4, kFPrio | kFLateV>(a, s);
}

}  // namespace fa
