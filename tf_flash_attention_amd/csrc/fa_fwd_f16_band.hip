// fa_fwd_f16_band.hip — persistent fp16 forward for 1d local windows (a band of 2·ws-1 keys
// around each query, unit stride), 32 < max(d, v_d) <= 64.  BASELINE config 4's shape.
//
// A band block touches few key tiles (ws = 256, 256 queries: 12 tiles), so a kernel that
// launches one workgroup per query block spends a large share of its time starting and
// ending blocks: loading Q, filling the K/V pipeline, storing O (round 1: c4 at 20 % MFMA
// busy, 10 scalar instructions per MFMA).  Here one workgroup per CU walks a contiguous
// list of blocks ("items": the query blocks of consecutive (batch, head) slices in order)
// as ONE stream of key tiles:
//
//   * every item is exactly T positions (T + 3 a multiple of 4, 9 <= T <= 21); wave pair o (the
//     item's queries 64o .. 64o+63) works o key tiles ahead of pair 0, so an item streams T + 3
//     tiles (a ws = 256 band: 9 positions for 12 tiles, each pair inside its own band at every
//     position).  Positions past an item's band load zeros and are skipped by every wave.  The
//     item loop is unrolled over its T positions, so ring slots, staging registers and every
//     per-position decision are compile-time;
//   * the K/V staging (registers, loaded one position ahead of their LDS store, 1.33 tiles a
//     position; LDS rings of four slots) runs straight across item boundaries;
//   * the next item's Q image is loaded one 16-B chunk per thread at positions 2-5 and stored
//     into the second of two LDS Q buffers one position later (3-6); each wave reads its new Q
//     fragments in the VALU phase of the item's last position;
//   * at positions 0-1 of the next item the waves write the finished item's O (fp16, [c][256 q])
//     over its dead Q buffer and its l / m beside it (MFMA phases, beside the other group's
//     softmax); at positions 2-3 whole 16-B rows leave
//     for HBM (coalesced; the per-value stores of a per-block kernel touch 32-64 lines each);
//   * every MFMA phase issues a fixed set of vector-memory operations, so hipcc's vmcnt waits
//     stay exact (a conditional store anywhere in the stream made every staging store wait
//     for the loads issued one phase earlier);
//   * K / V fragments are read inside the MFMA phase that uses them, two k-steps ahead: the
//     registers that would carry them across the VALU phase hold the stream's staging;
//   * the running reference m_run carries over items: an item's first tile seeds it once
//     (one exp pass), and its first PV / row sums start the accumulators (no reset).
//
// Inside an item the structure is the ping-pong of fa_fwd_f16_pingpong.hip (eight waves, two
// groups alternating MFMA and softmax phases, unconditional MFMAs with P zeroed for a wave's
// skipped tiles, fp32 accumulation, log2-domain lazy rebase at 8, row sums in running
// accumulators, the rebase check on the packed P, l relative to the stored fp16 m).  Replaces the reference's ForwardImpl
// (flash_attention.cu:425-1077) under LocalAttentionPolicy (flash_attention.h:117-140) for
// these shapes.
//
// Structures measured against this one (the unstaggered item, the whole epilogue in VALU(0), staging
// two positions ahead, LDS-DMA staging, packed edge-mask bounds, a hand-ordered softmax stream) and
// the stamp / ablation builds were taken out in round 5; their numbers are in DESIGN.md §3.0c, §6.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

#include <string.h>

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 64;
constexpr int kBN = 64;              // keys per tile
constexpr int kNW = 8;               // waves per workgroup, two per SIMD
constexpr int kBM = 32 * kNW;        // queries per item
constexpr int kQRow = 2 * kBM;       // bytes per Q row in LDS
constexpr int kQImg = kD * kQRow;    // 32 KB
constexpr int kTile = kD * kBN * 2;  // 8 KB
constexpr int kNS = 4;               // ring slots (K and V each)
constexpr int kOffK = 2 * kQImg;     // two Q buffers first
constexpr int kOffV = kOffK + kNS * kTile;
constexpr int kOffLM = kOffV + kNS * kTile;   // l (fp32) and m (fp16) of a finished item: 1.5 KB
constexpr int kOffTab = kOffLM + 6 * kBM;     // kt0 of every query block of a slice (int32)
constexpr int kMaxTab = 4096;                 // query blocks per slice: nq <= 1M
constexpr int kOffDummy = kOffTab + 4 * kMaxTab;  // scratch chunk per thread for the padding stores
constexpr int kSmem = kOffDummy + 16 * kNW * 64;  // 153.5 KB
// Item timeline (positions it = 0 .. T-1 of item n+1): MFMA(0) writes item n's l / m (and group
// 1's O) into LDS, MFMA(1) group 0's O (O over Q buffer n&1, dead by then); MFMA(2), MFMA(3) store
// it to HBM; MFMA(2..5) load item n+2's Q chunks, MFMA(3..6) store them into buffer n&1 (after the
// O reads); VALU(T-1) reads them as fragments: with T >= 9 a barrier separates every store from
// every read.
constexpr int kMinT = 9;
constexpr int kMaxT = 21;
// Staggered wave pairs (T positions, NT = T + 3 tiles an item, rings of four slots: tile j of the
// stream in slot j & 3).  Wave pair o (waves 2o and 2o + 1, the item's queries 64o .. 64o + 63; o =
// 2·grp + ((w >> 1) & 1)) works on tile p + o at position p, so each pair spans only the tiles of its
// own 64 queries (a ws = 256 band: 9 positions for 12 tiles, where one offset per group of four waves
// needed 10 and every wave spent one of them outside its band).  K of tile j is read by pair o at
// position j - o (interval 2p + (o >> 1)), V of tile j at position j - o + 1 (the PV of the position
// before).  A chunk stored in a group's MFMA phase (interval I) is published by the lgkmcnt(0) before
// that phase's barrier, so it is readable from interval I + 1, and it may be stored only after the last
// read of the slot's previous tile (j - 4).  Each interior tile then has two intervals, one per group,
// and each group stores its own threads' chunks: K(p+3) and V(p+2) by group 0, K(p+4) and V(p+3) by
// group 1 at position p.  The item boundary has one: group 1 stores the next item's K(0), K(1) whole at
// position T-1 and V(0), V(1) whole at position 0, group 0 K(2), K(3) whole at 0 and V(2), V(3) whole at
// 1 ("whole": its own chunk and the other group's, channel rows 32 apart).
// Entry i of the chunks group g stores at position p: the tile j relative to the item (T + 3 + j: the
// next item's j; -1: the previous item's T + 2) and the part (0 the thread's own chunk, 1 the other
// group's).  kStDummy: no tile (the entry loads zeros and stores them to a scratch chunk, so every
// position issues a fixed set of vector-memory operations and hipcc's vmcnt waits stay exact).
constexpr int kStDummy = -1000;
__host__ __device__ constexpr int stk_n(int T, int p) { return (p == 0 || p == T - 1) ? 4 : 1; }
__host__ __device__ constexpr int stk_j(int T, int p, int g, int i) {
  if (g == 0) return p == 0 ? (i < 2 ? 2 : 3) : (i == 0 ? p + 3 : kStDummy);
  return p == T - 1 ? (i < 2 ? T + 3 : T + 4) : (i == 0 ? p + 4 : kStDummy);
}
__host__ __device__ constexpr int stk_part(int T, int p, int g, int i) {
  return ((g == 0 && p == 0) || (g == 1 && p == T - 1)) ? (i & 1) : 0;
}
__host__ __device__ constexpr int stv_n(int, int p) { return p <= 1 ? 4 : 1; }
__host__ __device__ constexpr int stv_j(int, int p, int g, int i) {
  if (g == 0) return p == 0 ? (i == 0 ? -1 : kStDummy) : p == 1 ? (i < 2 ? 2 : 3) : (i == 0 ? p + 2 : kStDummy);
  return p == 0 ? (i < 2 ? 0 : 1) : (i == 0 ? p + 3 : kStDummy);
}
__host__ __device__ constexpr int stv_part(int, int p, int g, int i) {
  return ((g == 0 && p == 1) || (g == 1 && p == 0)) ? (i & 1) : 0;
}
constexpr float kRescaleThr = 8.f;
// after a 16-B buffer store: a wait state before any VALU may overwrite its data VGPRs (hipcc,
// ROCm 7.2, emitted such a write as the very next instruction and the stored dword arrived corrupted:
// DESIGN.md §6 toolchain finding (b); tools/check_store_hazard.py checks the shipped library)
__device__ __forceinline__ void store_data_guard() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// masked scores sit at or below -2^99 (the arithmetic edge mask); a row maximum at or below this
// floor means "nothing allowed yet" (never a reference).  Every finite score formed from fp16 inputs
// lies far inside (-2^98, 2^99), so no allowed score is clipped and no disallowed one stays above an
// allowed one (the 2^20 scale had a +-2^18 range).
constexpr float kMaskFloor = -0x1p98f;

struct BandArgs {
  FwdArgs a;
  int64_t n_items;  // b * ceil(nq / kBM)
  int32_t T;        // tile positions per item
  int32_t n_wg;     // workgroups (persistent)
  int32_t inter;    // 1: XCD-interleaved item order (below)
  int32_t n_xcd;    // XCDs the workgroups are dealt over (device_xcds(); n_wg % n_xcd == 0 when inter)
};

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    static_for<B + 1, E>(f);
  }
}

// wave-uniform description of one item
struct Item {
  int32_t sl;   // slice, relative to the workgroup's first slice
  int32_t q0;   // first query (nq past the list: no wave active)
  int32_t kt0;  // first key of its first tile (nk past the list: every load reads zeros)
};

// T (positions per item) is a template parameter, T + 3 a multiple of 4: the item loop is unrolled
// over its positions, so ring slots, staging registers and every "which position of the item"
// decision are compile-time (no per-phase selects)
template <int T>
__global__ __launch_bounds__(kNW * 64, 2) void fwd_f16_band_kernel(BandArgs ba) {
  constexpr int NT = T + 3;  // tiles an item streams
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  const FwdArgs& a = ba.a;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  static_assert((T + 3) % 4 == 0 && T >= kMinT && T <= kMaxT, "T: T + 3 a multiple of 4, in [kMinT, kMaxT]");
  const int nqb = (nq + kBM - 1) / kBM;
  // this workgroup's items: first + stride * local, inside [it_begin, it_end).
  //   contiguous: a run of consecutive items per workgroup (stride 1);
  //   XCD-interleaved (inter): the X XCDs (workgroup g runs on XCD g mod X; X = 8 on a whole MI355X)
  //   each take one X-th of the items, and the J workgroups of an XCD take every J-th item of it, so at any time an
  //   XCD's CUs walk J consecutive items whose key bands overlap: each K/V tile is re-read from that
  //   XCD's L2 instead of re-fetched (a contiguous run re-reads a tile one and two items later, a
  //   window of ~24 tiles per CU that the 4 MB L2 shared by 32 CUs does not hold)
  const int64_t g = blockIdx.x;
  int64_t it_begin, it_end, first, stride;
  if (ba.inter) {
    const int64_t X = ba.n_xcd, x = g % X, J = (ba.n_wg - x + X - 1) / X;
    it_begin = x * ba.n_items / X;
    it_end = (x + 1) * ba.n_items / X;
    first = it_begin + g / X;
    stride = J;
  } else {
    it_begin = g * ba.n_items / ba.n_wg;
    it_end = (g + 1) * ba.n_items / ba.n_wg;
    first = it_begin;
    stride = 1;
  }
  const int n_local = first < it_end ? (int)((it_end - first + stride - 1) / stride) : 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2;  // waves w and w+4 share a SIMD
  const int toff = 2 * grp + ((w >> 1) & 1);  // this wave pair's tile at position p is p + toff
  const int h = lane >> 5, r = lane & 31;
  const int gq = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int d = a.d, vd = a.v_d;
  const float c2 = (float)a.scale * kLog2e;

  // one buffer descriptor per tensor over the workgroup's slices [sl0, sl0 + nsl): per-item
  // offsets ride in soffset (host check: the span stays below 2^31 bytes, so offset 0x80000000
  // still reads zeros)
  const int64_t sl0 = it_begin / nqb;
  const int nsl = (int)((it_end - 1) / nqb - sl0 + 1);
  const uint32_t qsl = 2u * d * nq, ksl = 2u * d * nk, vsl = 2u * vd * nk;  // bytes per slice
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(static_cast<const __half*>(a.Q) + sl0 * (int64_t)d * nq, qsl * nsl);
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + sl0 * (int64_t)d * nk, ksl * nsl);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + sl0 * (int64_t)vd * nk, vsl * nsl);
  // first key tile of each query block (the same for every slice): computed once per workgroup
  // into LDS, so the stream's item switch is a table read, not two binary searches
  const lds_char_t* tab = smem + kOffTab;
  for (int qb = threadIdx.x; qb < nqb; qb += kNW * 64) {
    // the item's first tile: o tiles below wave pair o's first, the lowest over the pairs (may be < 0)
    int kt = nk;
    for (int o = 0; o < 4 && qb * kBM + 64 * o < nq; ++o) {
      int kb, ke;
      k_range_for_q_block(a.rule, qb * kBM + 64 * o, min(qb * kBM + 64 * o + 64, nq) - 1, &kb, &ke);
      if (ke > kb) kt = min(kt, (kb / kBN) * kBN - o * kBN);
    }
    *reinterpret_cast<__attribute__((address_space(3))) int*>(smem + kOffTab + 4 * qb) = kt;
  }
  __syncthreads();
  // the walk's item index n = first + local * stride as (slice, query block), advanced by
  // scalar adds (the host keeps n_items below 2^31; a 64-bit division per item lowered to ~100
  // scalar and vector instructions and spilled SGPRs across the stream)
  int walk_sl = 0, walk_qb = 0;
  {
    const int n0 = (int)((first < it_end ? first : it_begin) - sl0 * nqb);  // (relative to sl0)
    walk_sl = __builtin_amdgcn_readfirstlane(n0 / nqb);
    walk_qb = __builtin_amdgcn_readfirstlane(n0 - walk_sl * nqb);
  }
  const int stride_qb = __builtin_amdgcn_readfirstlane((int)(stride % nqb)),
            stride_sl = __builtin_amdgcn_readfirstlane((int)(stride / nqb));
  // the item at the walk position, then the walk advanced by one stride
  auto make_item = [&](int local) -> Item {
    Item x;
    const bool live = local < n_local;
    x.sl = live ? walk_sl : 0;  // (a dead item reads zeros from slice 0: offsets stay in range)
    x.q0 = live ? walk_qb * kBM : nq;
    const int kt0 = *reinterpret_cast<const __attribute__((address_space(3))) int*>(tab + 4 * walk_qb);
    x.kt0 = live ? __builtin_amdgcn_readfirstlane(kt0) : nk;
    if (live) {
      walk_qb += stride_qb;
      walk_sl += stride_sl;
      if (walk_qb >= nqb) {
        walk_qb -= nqb;
        ++walk_sl;
      }
    }
    return x;
  };
  Item cur = make_item(0), nxt = make_item(1);
  int prv_sl = 0, prv_q0 = nq;  // the finished item (none before the first)

  // ---- staging lanes: this thread owns chunk `tid` of every K/V tile = 8 keys of channel row crow
  const int cm = tid & 7, crow = tid >> 3;
  const uint32_t goff = (uint32_t)crow * (uint32_t)nk * 2u + 16u * cm;
  const uint32_t koff = crow < d ? goff : 0x80000000u, voff = crow < vd ? goff : 0x80000000u;
  // the other group's chunk of the same 8 keys (channel row crow ^ 32): the whole-tile stores at the
  // item boundary
  const int crowp = crow ^ 32;
  const uint32_t goffp = (uint32_t)crowp * (uint32_t)nk * 2u + 16u * cm;
  const uint32_t koffp = crowp < d ? goffp : 0x80000000u, voffp = crowp < vd ? goffp : 0x80000000u;
  const uint32_t kwo = crow * 128 + ((cm * 16) ^ ((crow & 2) << 5));
  const uint32_t vwo = crow * 128 + 16 * (cm ^ ((crow >> 1) & 7));
  auto load = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t slb, int k0) -> u32x4 __attribute__((always_inline)) {
    // (an item may start before key 0: those tiles read zeros)
    const bool in = k0 >= 0 && k0 + 8 * cm < nk;
    return __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off : 0x80000000u, slb + 2 * min(max(k0, 0), nk), 0);
  };
  auto store = [&](int off, u32x4 v) __attribute__((always_inline)) { *reinterpret_cast<lds_u32x4_t*>(smem + off) = v; };
  //      Q image [64][256] (64-B blocks XOR-swizzled by c&3): chunk j of a thread = channel row
  //      (tid>>5) + 16j, 8 queries at 8*(tid&31)
  const int qc0 = tid >> 5, qm = tid & 31;
  const uint32_t ql_lane = qc0 * kQRow + ((qm * 16) ^ ((qc0 & 3) << 6));
  // (inside the item loop the lane offsets are recomputed where used from an opaque copy of the
  // thread id: hoisted, they would stay live across the whole stream, a VGPR each)
  auto opaque_tid = [&]() -> int __attribute__((always_inline)) {
    int t = tid;
    asm volatile("" : "+v"(t));
    return t;
  };
  auto qload = [&](const Item& x, int j) -> u32x4 __attribute__((always_inline)) {
    const int t = opaque_tid(), qc = t >> 5, qq = 8 * (t & 31);
    const uint32_t qg = (uint32_t)qc * (uint32_t)nq * 2u + 2u * (uint32_t)qq;
    const bool in = qc + 16 * j < d && x.q0 + qq < nq;
    // (nt: Q is read once; its lines should not push the band's K / V tiles, which the XCD's other
    // workgroups re-read, out of the L2)
    return __builtin_amdgcn_raw_buffer_load_b128(qrs, in ? qg + (uint32_t)j * 32u * (uint32_t)nq : 0x80000000u,
                                                 x.sl * qsl + 2 * min(x.q0, nq), 2);
  };

  // ---- staging entries (see stk_j / stv_j): the LDS place of entry (j, part) and its load
  auto st_off = [&](int base, int j, int pt, uint32_t wo) -> int __attribute__((always_inline)) {
    return j == kStDummy ? kOffDummy + 16 * tid : base + (j & 3) * kTile + (int)(pt ? wo ^ 4096u : wo);
  };
  // entry (j0, pt0) of group 0 / (j1, pt1) of group 1 for a store one position on: j relative to the
  // current item (>= NT: the next item's j - NT); a dummy entry reads zeros (k0 = nk).  One load with
  // the group's operands selected (scalar selects: a load per group behind a branch costs ~12 SALU)
  auto st_load = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t offp, uint32_t slsz, int j0, int pt0, int j1,
                     int pt1) -> u32x4 __attribute__((always_inline)) {
    const bool d0 = j0 == kStDummy, d1 = j1 == kStDummy, n0 = !d0 && j0 >= NT, n1 = !d1 && j1 >= NT;
    const int k00 = d0 ? nk : (n0 ? nxt.kt0 + (j0 - NT) * kBN : cur.kt0 + j0 * kBN);
    const int k01 = d1 ? nk : (n1 ? nxt.kt0 + (j1 - NT) * kBN : cur.kt0 + j1 * kBN);
    const int sl0 = n0 ? nxt.sl : cur.sl, sl1 = n1 ? nxt.sl : cur.sl;
    const int k0 = (k00 == k01) ? k00 : (grp ? k01 : k00);
    const int slb = ((sl0 == sl1) ? sl0 : (grp ? sl1 : sl0)) * (int)slsz;
    const int pt = (pt0 == pt1) ? pt0 : (grp ? pt1 : pt0);
    return load(rs, pt ? offp : off, (uint32_t)slb, k0);
  };

  // ---- prologue: Q(item 0) into Q buffer 0, K(0) and K(1) whole into their ring slots, every V slot
  //      zeroed (position 0's PVs read them against P = 0); the chunks this thread's group stores at
  //      position 0 into the staging registers
  u32x4 kst[4], vst[4];
  {
    u32x4 kp[4], qv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) kp[j] = load(krs, (j & 1) ? koffp : koff, cur.sl * ksl, cur.kt0 + (j >> 1) * kBN);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kst[i] = st_load(krs, koff, koffp, ksl, stk_j(T, 0, 0, i), stk_part(T, 0, 0, i), stk_j(T, 0, 1, i),
                       stk_part(T, 0, 1, i));
      vst[i] = st_load(vrs, voff, voffp, vsl, stv_j(T, 0, 0, i), stv_part(T, 0, 0, i), stv_j(T, 0, 1, i),
                       stv_part(T, 0, 1, i));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) qv[j] = qload(cur, j);
#pragma unroll
    for (int j = 0; j < 4; ++j) store(ql_lane + j * 16 * kQRow, qv[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) store(kOffK + (j >> 1) * kTile + ((j & 1) ? kwo ^ 4096u : kwo), kp[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) store(kOffV + j * kTile + 16 * tid, u32x4{0, 0, 0, 0});
  }
  __syncthreads();

  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r]
  half8 qf[4];
  auto read_q = [&](int buf) __attribute__((always_inline)) {
    const lds_char_t* qb = smem + buf * kQImg;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int cr = 16 * s + 8 * (gq >> 1) + 4 * e + tq;
        const int col = 32 * w + 16 * (gq & 1) + 4 * tp;
        const half4 t = tr_read(qb + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
        if (e == 0) qf[s].lo = t; else qf[s].hi = t;
      }
      qf[s] = scale8(qf[s], c2);
    }
  };
  read_q(0);

  // ---- per-item lane state (the current item's rule bounds)
  int wq0 = 0, qi = 0, klo = 0, kspan = 0, wlo_min = 0, wlo_max = 0, whi_min = 0, whi_max = 0;
  bool wave_active = false;
  auto item_state = [&](const Item& x) __attribute__((always_inline)) {
    wq0 = x.q0 + 32 * w;
    qi = wq0 + r;
    wave_active = wq0 < nq;
    klo = 0; kspan = 0; wlo_min = wlo_max = whi_min = whi_max = 0;
    if (wave_active) {
      int khi;
      const Rule& R = a.rule;
      if (R.k.s0 == 1) {  // unit key stride (none_front, or Nk >= Nq): the interval in closed form
        const int qo = R.q.o0 + R.q.s0 * min(qi, nq - 1);
        const int ohi = R.look_ahead == 1 ? qo : sat_add32(qo, R.ws - 1);
        klo = min(max(qo - (R.ws - 1) - R.k.o0, 0), nk);
        khi = min(ohi - R.k.o0, nk - 1);
      } else {
        // (strides made opaque here: else hipcc hoists the divisions' reciprocals to the kernel
        // top, and they stay live, spilled, across the whole stream)
        Rule R2 = R;
        R2.seq_dims = 1;  // (the host admits 1d rules only: no 2d coordinate division compiled in)
        asm volatile("" : "+s"(R2.k.s0), "+s"(R2.q.s0));
        key_interval(R2, min(qi, nq - 1), &klo, &khi);
      }
      kspan = max(khi - klo + 1, 0);
      const int last = min(31, nq - 1 - wq0);
      wlo_min = __builtin_amdgcn_readfirstlane(klo);
      whi_min = __builtin_amdgcn_readfirstlane(khi);
      wlo_max = __builtin_amdgcn_readlane(klo, last);
      whi_max = __builtin_amdgcn_readlane(khi, last);
    }
  };
  item_state(cur);
  // tile class of position `it` of the current item: 0 no allowed pair, 2 all allowed; mixed: 3 only
  // some lanes' first allowed key lies inside the tile (the band's leading edge), 4 only some lanes'
  // last one (the trailing edge), 1 both (windows narrower than a tile).  (khi <= nk - 1 for every
  // lane, so the tail past nk is a trailing edge.)
  auto tcls = [&](int it) -> int __attribute__((always_inline)) {
    const int k0 = cur.kt0 + it * kBN, k1 = k0 + kBN - 1;
    if (!wave_active || wlo_min > k1 || whi_max < k0) return 0;
    const bool lo = wlo_max > k0, hi = whi_min < k1;
    return lo ? (hi ? 1 : 3) : (hi ? 4 : 2);
  };

  // fragment read bases (lane constants), as fa_fwd_f16_pingpong.hip
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (gq >> 1) + tq) * 128 + (((32 * t + 16 * (gq & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  auto read_kstep = [&](const lds_char_t* p, int s, half8 (&f)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f[t].lo = tr_read(p + kbase[t] + (16 * s) * 128);
      f[t].hi = tr_read(p + kbase[t] + (16 * s + 4) * 128);
    }
  };
  auto read_vstep = [&](const lds_char_t* p, int s, half8 (&f)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) f[u] = read_b128(p + vbase[s] + 32 * u * 128);
  };

  floatx16 st[2];      // Sᵀ of the tile being softmaxed
  uint32_t pw[4][4];   // P (fp16 pairs), dword x of PV k-step s
  floatx16 o[2];       // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
  floatx16 negm;       // -m_run broadcast: the C operand of every Sᵀ chain
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
    negm[i] = 0.f;
  }
  float m_run = 0.f, m_max = kNegInf;
  float lacc[4] = {0.f, 0.f, 0.f, 0.f};

  // edge-tile mask, arithmetic: key k0 + 8h + off is allowed iff 0 <= base + off < kspan (base = k0 +
  // 8h - klo), so min(s, (base + off + 0.5)·2^100) (leading edge) and min(s, (kspan - base - off -
  // 0.5)·2^100) (trailing edge) keep an allowed score (the bound is >= 2^99) and take a disallowed
  // one to <= -2^99, whose exp2 is 0 against any reference (base + off + 0.5 is a half-integer of at
  // most a few thousand, exact in fp32, and the power-of-two scale keeps it exact; past the fp32
  // range the bound is +-inf with the same sign).  One fma and one min per score and edge, no
  // compare, no VCC select and so no hazard wait (the select form cost an add, a compare, a 2-state
  // s_nop and a v_cndmask per score); one copy of the code serves both edges (the edge picks the
  // per-lane constant and the sign), and a tile holding both edges (windows narrower than a tile)
  // runs it twice.  Rows with nothing allowed stay below kMaskFloor (never seeded).
  auto mask = [&](int k0, int cls) __attribute__((always_inline)) {
    constexpr float kBig = 0x1p100f;
    const float fb = (float)(k0 + 8 * h - klo);
    const float ca = __builtin_fmaf(fb, kBig, 0.5f * kBig), cb = __builtin_fmaf((float)kspan - fb, kBig, -0.5f * kBig);
    const int npass = cls == 1 ? 2 : 1;
#pragma nounroll
    for (int pass = 0; pass < npass; ++pass) {
      const bool lo = (cls == 3) || (cls == 1 && pass == 0);
      const float cc = lo ? ca : cb, sg = lo ? kBig : -kBig;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          st[t][i] = fminf(st[t][i], __builtin_fmaf(sg, (float)(32 * t + 16 * (i >> 3) + (i & 7)), cc));
    }
  };
  // the exponentials of a P k-step (8) issued as one batch into their own registers before its four
  // conversions (at ~235 VGPRs hipcc otherwise reuses two temporaries, so every v_cvt_pk_f16_f32
  // waits on the v_exp_f32 just before it: an s_nop plus the transcendental latency, 16 times a tile)
  auto exp_cvt = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = __builtin_amdgcn_exp2f(st[s >> 1][8 * (s & 1) + j]);
      asm volatile("" : "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]), "+v"(e[4]), "+v"(e[5]), "+v"(e[6]), "+v"(e[7]));
#pragma unroll
      for (int x = 0; x < 4; ++x)
        pw[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)e[2 * x], (_Float16)e[2 * x + 1]});
    }
  };
  // the exact fp32 row max of the tile (both key halves)
  auto row_max = [&]() -> float __attribute__((always_inline)) {
    float mx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(st[j >> 1][8 * (j & 1)], st[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
    for (int i = 2; i < 8; i += 2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        mx[j] = fmaxf(fmaxf(mx[j], st[j >> 1][8 * (j & 1) + i]), st[j >> 1][8 * (j & 1) + i + 1]);
    return max_pair32(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
  };
  // the running max of P over the current epoch (per lane) and 2^thr (-1: no reference yet)
  half2v pmr = {(_Float16)0.f, (_Float16)0.f};
  _Float16 thr_h = (_Float16)-1.f;
  auto pmax_tile = [&]() -> half2v __attribute__((always_inline)) {
    auto M3 = [](half2v x, half2v y, half2v z) __attribute__((always_inline)) {
      return __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z);
    };
    auto H = [&](int s_, int x) __attribute__((always_inline)) { return __builtin_bit_cast(half2v, pw[s_][x]); };
    half2v a0 = M3(H(0, 0), H(0, 1), H(0, 2)), b0 = M3(H(2, 0), H(2, 1), H(2, 2));
    a0 = M3(a0, H(0, 3), H(1, 0));
    b0 = M3(b0, H(2, 3), H(3, 0));
    a0 = M3(a0, H(1, 1), H(1, 2));
    b0 = M3(b0, H(3, 1), H(3, 2));
    return M3(M3(a0, H(1, 3), H(3, 3)), b0, b0);
  };
  auto softmax = [&](int it, int cls, bool first) __attribute__((always_inline)) {
    if (cls != 2) mask(cur.kt0 + it * kBN, cls);
    if (first) {  // an item's first tile: nothing to rescale (O and l start fresh): seed, then exp once
      const float mt = row_max();
      m_max = fmaxf(m_max, m_run + mt);
      const bool seed = mt > kMaskFloor;  // else (an empty row so far) a later tile seeds
      const float delta = seed ? mt : 0.f;
      m_run += delta;
      thr_h = seed ? (_Float16)(1 << (int)kRescaleThr) : (_Float16)-1.f;
      pmr = half2v{(_Float16)0.f, (_Float16)0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[0][i] -= delta;
        st[1][i] -= delta;
        negm[i] = -m_run;
      }
      exp_cvt();
    } else {
      // the rebase check on the packed P (as fa_fwd_f16_pingpong.hip): the exponentials run against
      // m_run anyway; the exact fp32 max is formed only in the (rare) rebase branch
      exp_cvt();
#pragma unroll
      for (int x = 0; x < 4; ++x)  // pinned here: else they sink past the (rare) rebase branch
        asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
      const half2v tm = pmax_tile();
      const _Float16 tmx = __builtin_elementwise_maximum(tm[0], tm[1]);
      const half2v pmr_old = pmr;
      pmr = __builtin_elementwise_maximum(pmr, tm);
      if (__any(tmx > thr_h)) {
        const float mt = row_max();
        // close the epoch: its P maximum (approximate) and this tile (exact) into m_max
        const float pold = (float)__builtin_elementwise_maximum(pmr_old[0], pmr_old[1]);
        m_max = fmaxf(m_max, fmaxf(m_run + mt, m_run + __log2f(pold)));
        // (thr_h alone carries the state: -1 until the row has a reference)
        const bool unset = thr_h < (_Float16)0.f;
        const bool seed = unset && (mt > kMaskFloor);
        const float delta = unset ? (seed ? mt : 0.f) : fmaxf(mt, 0.f);
        const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
        m_run += delta;
        thr_h = (unset && !seed) ? (_Float16)-1.f : (_Float16)(1 << (int)kRescaleThr);
#pragma unroll
        for (int x = 0; x < 4; ++x) lacc[x] *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o[0][i] *= alpha;
          o[1][i] *= alpha;
          st[0][i] -= delta;
          st[1][i] -= delta;
          negm[i] = -m_run;
        }
        exp_cvt();
        pmr = half2v{(_Float16)0.f, (_Float16)0.f};
      }
    }
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x)  // an item's first tile starts the sums (no reset at the boundary)
        lacc[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, pw[s][x]), one2, (first && s == 0) ? 0.f : lacc[x],
                                         false);
  };

  int n = 0;  // local item index (positions of the item are static in the unrolled body)

  // O, l, m of the item that just finished (its last PV ran in the MFMA phase before) into LDS:
  // O [c][256 q] fp16 over the finished item's Q buffer, l / m at the l/m area; in two parts: l / m
  // (returns 1/l), O
  auto epi_lm = [&]() -> float __attribute__((always_inline)) {
    const float l_tot = sum_pair32((lacc[0] + lacc[1]) + (lacc[2] + lacc[3]));
    const float inv = (l_tot > 0.f) ? __builtin_amdgcn_rcpf(l_tot) : 0.f;
    const float m_fin = max_pair32(fmaxf(m_max, m_run + __log2f((float)__builtin_elementwise_maximum(pmr[0], pmr[1]))));
    if (h == 0) {
      float lv = 0.f;
      __half mv = neg_inf_approx<__half>();
      if (l_tot > 0.f) {
        mv = __float2half(m_fin * kLn2);
        lv = l_tot * __builtin_amdgcn_exp2f(m_run - __half2float(mv) * kLog2e);
      }
      *reinterpret_cast<__attribute__((address_space(3))) float*>(smem + kOffLM + 4 * (32 * w + r)) = lv;
      *reinterpret_cast<__attribute__((address_space(3))) unsigned short*>(smem + kOffLM + 4 * kBM + 2 * (32 * w + r)) =
          __half_as_ushort(mv);
    }
    return inv;
  };
  auto epi_o = [&](float inv) __attribute__((always_inline)) {
    lds_char_t* ob = smem + ((n + 1) & 1) * kQImg + 2 * (32 * w + r);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cch = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        *reinterpret_cast<__attribute__((address_space(3))) _Float16*>(ob + cch * kQRow) = (_Float16)(o[u][i] * inv);
        if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
  };
  float oinv = 0.f;  // (group 0) the finished item's 1/l from MFMA(0) to MFMA(1)
  auto item_switch = [&]() __attribute__((always_inline)) {
    const float inv = epi_lm();
    if (grp == 1) epi_o(inv);
    else oinv = inv;
    m_max = kNegInf;
    m_run = 0.f;  // (this item's first Sᵀ ran against -m = 0: see the end of VALU(T-1))
    pmr = half2v{(_Float16)0.f, (_Float16)0.f};
    thr_h = (_Float16)-1.f;
    item_state(cur);
  };
  // the next item's Q chunk in flight (loaded at positions 2-5, stored one position later: one
  // set of registers; the load has a whole position to land)
  u32x4 qst;
  // the finished item's O / l / m leave from LDS at positions 2-3: lane constants
  const uint32_t osl = 2u * vd * nq;  // bytes per O slice
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(static_cast<__half*>(a.O) + sl0 * (int64_t)vd * nq, osl * nsl);
  const __amdgpu_buffer_rsrc_t lrs = make_rsrc(static_cast<float*>(a.l) + sl0 * (int64_t)nq, 4u * nq * nsl);
  const __amdgpu_buffer_rsrc_t mrs = make_rsrc(static_cast<__half*>(a.m) + sl0 * (int64_t)nq, 2u * nq * nsl);

  // MFMA(it): Sᵀ of the wave pair's tile it + toff (K k-steps 0-1 read at the phase head, 2-3 after
  // the first MFMAs), PV of its previous tile (V read two k-steps ahead of its MFMAs); the group's
  // staging entries of this position (stk_j / stv_j) stored after Sᵀ k-step 0 and the next
  // position's loaded; the item's fixed-position traffic (O / l / m out at 2-3, the next item's Q
  // loaded at 2-5 and stored into LDS at 3-6); an lgkmcnt(0) at the end publishes the stores
  auto mfma_phase = [&](auto IT_) __attribute__((always_inline)) {
    constexpr int it = decltype(IT_)::value;
    constexpr int c = it & 3;
    __builtin_amdgcn_s_setprio(1);
    // (this pair's tiles are p + toff, tile j in slot j & 3 = ((j & 3) + toff) & 3; the PV at position 0
    // is of the previous item's tile T-1+toff)
    constexpr int cv = (it == 0) ? ((T - 1) & 3) : ((c + 3) & 3);
    const lds_char_t* pk = smem + kOffK + ((c + toff) & 3) * kTile;
    const lds_char_t* pv = smem + kOffV + ((cv + toff) & 3) * kTile;
    // every fragment is read in the phase that uses it, two k-steps ahead (nothing lives across
    // the VALU phase: the register budget holds the stream's staging); the first two K k-steps
    // are read at the phase start, their latency the only one exposed
    if constexpr (it == 1) {  // group 0: the finished item's O, before o restarts
      if (grp == 0 && n > 0) {
        epi_o(oinv);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // this phase's LDS stores: the group's staging entries (stk_j / stv_j) and the next item's Q chunk.
    // Issued after Sᵀ k-step 0 (hipcc keeps them in source order against the fragment reads: it cannot
    // tell the slots apart), so the lgkmcnt(0) that publishes them at the phase end finds them done
    auto lds_stores = [&]() __attribute__((always_inline)) {
      static_for<0, stk_n(T, it)>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = decltype(I_)::value;
        store(grp ? st_off(kOffK, stk_j(T, it, 1, i), stk_part(T, it, 1, i), kwo)
                  : st_off(kOffK, stk_j(T, it, 0, i), stk_part(T, it, 0, i), kwo),
              kst[i]);
      });
      static_for<0, stv_n(T, it)>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = decltype(I_)::value;
        store(grp ? st_off(kOffV, stv_j(T, it, 1, i), stv_part(T, it, 1, i), vwo)
                  : st_off(kOffV, stv_j(T, it, 0, i), stv_part(T, it, 0, i), vwo),
              vst[i]);
      });
      if constexpr (it >= 3 && it <= 6) {
        // the next item's Q chunk j = it-3 (channel rows 16j..16j+15) over the finished item's O,
        // whose rows 16j.. both groups read out at MFMA(2 + j/2), an interval or more before
        const int t = opaque_tid(), qc = t >> 5, qm2 = t & 31;
        const uint32_t ql = qc * kQRow + ((qm2 * 16) ^ ((qc & 3) << 6));
        store(((n + 1) & 1) * kQImg + ql + (it - 3) * 16 * kQRow, qst);
      }
    };
    half8 kf[4][2], vf[4][2];
    read_kstep(pk, 0, kf[0]);
    read_kstep(pk, 1, kf[1]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[s][t], qf[s], s == 0 ? negm : st[t], 0, 0, 0);
      if (s < 2) read_kstep(pk, s + 2, kf[s + 2]);
      else read_vstep(pv, s - 2, vf[s - 2]);
      if (s == 0) lds_stores();
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half8 pp = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
      // position 1 holds an item's first PV (tile 0): it starts the accumulator (the finished
      // item's O left for LDS in the VALU phase before; no reset keeps both alive)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], pp, (it == 1 && s == 0) ? floatx16{} : o[u], 0, 0, 0);
      if (s < 2) read_vstep(pv, s + 2, vf[s + 2]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // K k-steps 0-1
    // this phase's LDS stores (staging, the next item's Q chunk) after Sᵀ k-step 0: done well before
    // the lgkmcnt(0) that publishes them at the phase end
    constexpr int nst = stk_n(T, it) + stv_n(T, it) + ((it >= 3 && it <= 6) ? 1 : 0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // Sᵀ k-steps 0-1, each followed by a K k-step's reads
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      if (s == 0) __builtin_amdgcn_sched_group_barrier(0x200, nst, 0);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // Sᵀ k-steps 2-3 and PV k-steps 0-1, each followed by a V k-step
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // PV k-steps 2-3
    if constexpr (it == 2 || it == 3) {  // the finished item's O rows (at 2 also l / m); none before item 1
      const bool on = prv_q0 < nq;
      const lds_char_t* ob = smem + ((n + 1) & 1) * kQImg;
      const int tt = opaque_tid(), orw = tt >> 5, ocl = tt & 31;  // 16-B chunk (c = orw + 16j, queries 8*ocl..)
      // the item's offsets are wave-uniform; readfirstlane proves it to hipcc (else every store below
      // is wrapped in a waterfall loop with an lgkmcnt(0) inside: cdna_hip_programming.md T20)
      const int osoff = __builtin_amdgcn_readfirstlane(prv_sl * osl + 2 * min(prv_q0, nq));
      // (sc1: the written lines leave the L2 instead of displacing K / V tiles; O, l, m are not re-read)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cc = orw + 16 * (2 * (it & 1) + j);
        const u32x4 v = *reinterpret_cast<const lds_u32x4_t*>(ob + cc * kQRow + 16 * ocl);
        const bool in = on && prv_q0 + 8 * ocl < nq;
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, in ? (uint32_t)cc * (uint32_t)nq * 2u + 16u * ocl : 0x80000000u,
                                               osoff, 16);
        store_data_guard();
      }
      if constexpr (it == 2) {
        // l (64 chunks of 4 queries) from threads 0-63, m (32 chunks of 8) from threads 64-95
        const int lmc = tt < 64 ? tt : (tt < 96 ? tt : 0);
        const u32x4 v = *reinterpret_cast<const lds_u32x4_t*>(smem + kOffLM + 16 * lmc);
        const uint32_t loff = (on && tt < 64 && prv_q0 + 4 * tt < nq) ? 16u * tt : 0x80000000u;
        const uint32_t moff = (on && tt >= 64 && tt < 96 && prv_q0 + 8 * (tt - 64) < nq) ? 16u * (tt - 64) : 0x80000000u;
        const int lsoff = __builtin_amdgcn_readfirstlane(prv_sl * 4 * nq + 4 * min(prv_q0, nq));
        const int msoff = __builtin_amdgcn_readfirstlane(prv_sl * 2 * nq + 2 * min(prv_q0, nq));
        __builtin_amdgcn_raw_buffer_store_b128(v, lrs, loff, lsoff, 16);
        store_data_guard();
        __builtin_amdgcn_raw_buffer_store_b128(v, mrs, moff, msoff, 16);
        store_data_guard();
      }
    }
    if constexpr (it >= 2 && it <= 5) qst = qload(nxt, it - 2);
    {
      // the entries the group stores at the next position (the next item's position 0 at T-1), one
      // position ahead (relative to the current item: + NT for the next item's)
      constexpr int pn = it + 1 < T ? it + 1 : 0, add = it + 1 < T ? 0 : NT;
      auto rel = [](int j) constexpr { return j == kStDummy ? kStDummy : j + add; };
      static_for<0, stk_n(T, pn)>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = decltype(I_)::value;
        kst[i] = st_load(krs, koff, koffp, ksl, rel(stk_j(T, pn, 0, i)), stk_part(T, pn, 0, i),
                         rel(stk_j(T, pn, 1, i)), stk_part(T, pn, 1, i));
      });
      static_for<0, stv_n(T, pn)>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = decltype(I_)::value;
        vst[i] = st_load(vrs, voff, voffp, vsl, rel(stv_j(T, pn, 0, i)), stv_part(T, pn, 0, i),
                         rel(stv_j(T, pn, 1, i)), stv_part(T, pn, 1, i));
      });
    }
    if constexpr (it == 0) {
      // the finished item's l / m (and group 1's O: its last PV ran above); the new item's state
      if (n > 0) {
        __builtin_amdgcn_sched_barrier(0);
        item_switch();
      }
    }
    // publish this phase's staging stores before its barrier: the other group may read them in the
    // next interval
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_setprio(0);
  };

  // VALU(it): [position 0 past the first item: O / l / m of the finished item into LDS, the new
  // item's lane state] softmax of the tile; [last position: the next item's Q fragments]
  auto valu_phase = [&](auto IT_) __attribute__((always_inline)) {
    constexpr int it = decltype(IT_)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staging stores / reads landed
    const int cls = tcls(it + toff);
    if (cls != 0) {
      softmax(it + toff, cls, it == 0);
    } else {  // the next (unconditional) PV must add nothing
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int z = 0; z < 4; ++z) pw[y][z] = 0u;
      if constexpr (it == 0) {
#pragma unroll
        for (int y = 0; y < 4; ++y) lacc[y] = 0.f;
      }
    }
    if constexpr (it == T - 1) {
      read_q((n + 1) & 1);  // before this wave's first Sᵀ of the next item
      // the next item's scores start relative to 0, not to this item's m_run: an item's result
      // must not depend on the item the workgroup walked before it (bitwise: a slice's O / l / m
      // are the same wherever it sits in the batch)
#pragma unroll
      for (int i = 0; i < 16; ++i) negm[i] = 0.f;
    }
  };

  if (grp == 1) __builtin_amdgcn_s_barrier();
  auto step = [&](auto IT_) __attribute__((always_inline)) {
    constexpr int it = decltype(IT_)::value;
    if constexpr (it == 0) {
      if (n > 0) {  // shift the item window (wave-uniform scalars)
        prv_sl = cur.sl;
        prv_q0 = cur.q0;
        cur = nxt;
        nxt = make_item(n + 1);
      }
    }
    __builtin_amdgcn_s_barrier();
    mfma_phase(IT_);
    __builtin_amdgcn_s_barrier();
    valu_phase(IT_);
  };
  // one extra (phantom) item at the end: its positions 0-3 carry the last item's PV, its O / l /
  // m into LDS and out to HBM; the rest only move zeros
  for (n = 0; n <= n_local; ++n) static_for<0, T>(step);
  if (grp == 0) __builtin_amdgcn_s_barrier();
}

int64_t band_workgroups(int64_t n_items) {
  const int cus = device_cus();  // per device (fa_api.hip)
  return n_items < cus ? n_items : cus;
}

// the XCD-interleaved item order needs whole XCD groups and several items per workgroup
bool band_interleaved(int64_t n_items, int64_t n_wg, int n_xcd) { return n_wg % n_xcd == 0 && n_items >= 2 * n_wg; }

struct TCache {
  Rule r;
  int T;
  bool valid;
};
thread_local TCache g_scache = {{}, 0, false};

}  // namespace

// positions T an item takes when wave pair o runs o tiles ahead of pair 0 (the item's first tile o
// below pair o's first, the lowest over the pairs); T + 3 a multiple of 4, >= kMinT
int band_positions_stag(const FwdArgs& a) {
  if (g_scache.valid && !memcmp(&g_scache.r, &a.rule, sizeof(Rule))) return g_scache.T;
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const int nqb = (nq + kBM - 1) / kBM;
  int T = 0;
  for (int qb = 0; qb < nqb; ++qb) {
    const int q0 = qb * kBM;
    int kb[4], ke[4], kt = nk;
    for (int o = 0; o < 4; ++o) {
      kb[o] = ke[o] = 0;
      if (q0 + 64 * o >= nq) continue;
      k_range_for_q_block(a.rule, q0 + 64 * o, min(q0 + 64 * o + 64, nq) - 1, &kb[o], &ke[o]);
      if (ke[o] > kb[o]) kt = min(kt, (kb[o] / kBN) * kBN - o * kBN);
    }
    for (int o = 0; o < 4; ++o)
      if (q0 + 64 * o < nq && ke[o] > kb[o]) T = max(T, (ke[o] - kt + kBN - 1) / kBN - o);
  }
  T = (max(T, kMinT) + 3 + 3) / 4 * 4 - 3;
  g_scache.r = a.rule;
  g_scache.T = T;
  g_scache.valid = true;
  return T;
}

bool fwd_f16_band_supported(const FwdArgs& a) {
  const Rule& r = a.rule;
  const int nq = r.q.n, nk = r.k.n;
  const int dm = max(a.d, a.v_d);
  if (!(r.policy == 2 && r.seq_dims == 1 && r.ls == 0)) return false;
  // v_d == 64: the epilogue's per-value buffer stores need no channel predicate (a predicated
  // form keeps 32 lane-dependent 64-bit offsets live across the stream: 116 spilled VGPRs)
  if (!(a.v_d == kD && a.d > 32 && a.d <= kD && nk % 8 == 0 && nk > 0 && nq > 0)) return false;
  if ((int64_t)dm * nk * 2 >= (1ll << 31) || (int64_t)dm * nq * 2 >= (1ll << 31)) return false;
  if ((reinterpret_cast<uintptr_t>(a.K) % 16) || (reinterpret_cast<uintptr_t>(a.V) % 16) ||
      (reinterpret_cast<uintptr_t>(a.Q) % 16) || nq % 8)
    return false;
  // a band: every block spans few tiles (else the per-launch kernels cover it at no loss)
  if (band_positions_stag(a) > kMaxT) return false;
  // the per-slice table of first key tiles lives in LDS: kMaxTab query blocks (nq <= 1M)
  if ((nq + kBM - 1) / kBM > kMaxTab) return false;
  // one descriptor per tensor spans a workgroup's slices: below 2^31 bytes
  const int64_t nqb = (nq + kBM - 1) / kBM, n_items = a.b * nqb, n_wg = band_workgroups(n_items);
  if (n_items >= (1ll << 31)) return false;  // the walk's item arithmetic is 32-bit
  const int xcds = device_xcds();
  const int64_t span =
      (band_interleaved(n_items, n_wg, xcds) ? (n_items + xcds - 1) / xcds : (n_items + n_wg - 1) / n_wg) / nqb + 2;
  return span * 2 * (int64_t)dm * (nq > nk ? nq : nk) < (1ll << 31);
}

template <int T>
hipError_t launch_band_t(const BandArgs& ba, hipStream_t s) {
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(fwd_f16_band_kernel<T>), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((fwd_f16_band_kernel<T>), dim3((unsigned)ba.n_wg), dim3(kNW * 64), kSmem, s, ba);
  return hipGetLastError();
}

hipError_t launch_fwd_f16_band(const FwdArgs& a, hipStream_t s) {
  BandArgs ba;
  ba.a = a;
  ba.T = band_positions_stag(a);
  ba.n_items = a.b * (int64_t)((a.rule.q.n + kBM - 1) / kBM);
  ba.n_wg = (int)band_workgroups(ba.n_items);
  ba.n_xcd = device_xcds();
  ba.inter = band_interleaved(ba.n_items, ba.n_wg, ba.n_xcd) ? 1 : 0;
#ifdef FA_DIAG
  // FA_FWD_VARIANT=2402: the round-2 item order (contiguous runs of items per workgroup), for the
  // L2-traffic comparison of DESIGN.md §3.0c
  if (diag_variant("FA_FWD_VARIANT") == 2402) ba.inter = 0;
#endif
  switch (ba.T) {
    case 9: return launch_band_t<9>(ba, s);
    case 13: return launch_band_t<13>(ba, s);
    case 17: return launch_band_t<17>(ba, s);
    default: return launch_band_t<21>(ba, s);
  }
}

}  // namespace fa
