// fa_fwd_f16_pp.hip — fp16 fused attention forward for 32 < max(d, v_d) <= 64:
// one wave per SIMD, 64 queries per wave as two 32-query blocks whose softmax
// runs half a key tile apart ("paired blocks").
//
// Why: at d = 64 a 32-query × 64-key tile costs 16 MFMAs (512 matrix cycles) but
// ≈ 470 cycles of VALU / transcendental issue (row max, 32 v_exp, cvt, row sums).
// With two waves per SIMD the waves phase-lock behind the workgroup barrier and
// their softmax and MFMA phases collide.  Here a single wave owns the SIMD and
// its own instruction stream carries the overlap: every MFMA segment of one
// block is issued beside the softmax of the other block,
//
//   segment 2i   : Sᵀ MFMAs of block A, tile i+1 | softmax of block B, tile i | PV MFMAs of A, tile i
//   segment 2i+1 : Sᵀ MFMAs of block B, tile i+1 | softmax of block A, tile i+1 | PV MFMAs of B, tile i
//
// so each segment holds 16 MFMAs and the VALU work they hide, and a block's next
// Sᵀ is always issued after its own rebase decision (no pending corrections).
// K and V fragments are read from LDS once per wave and feed both blocks.
//
// LDS images ([channel][64 keys], 128-B rows, one 8 KB tile each, 3-slot rings):
//   * K: 64-B halves swapped on rows with c&2; the Sᵀ A operand is a transposed
//     read (ds_read_b64_tr_b16) whose key columns are permuted (bits 2 and 3 of
//     the key within 16 swapped) so that register x of P's k-step s holds key
//     16s + 8h + x — lane half h's eight keys are contiguous;
//   * V: plain rows with 16-B chunks XOR-swizzled by (c>>1)&7, so the PV A operand of
//     k-step s is one conflict-free ds_read_b128 of chunk 2s+h (16 lanes = 16 rows cover
//     the 64 banks).
// One barrier per key tile.  Staging is register-based (global → registers two
// steps ahead → LDS); tiles i+2 (K) / i+1 (V) are already resident when tile i runs.
// Round 5: the K / V fragments are double-buffered (by step parity, 4-slot rings): step i reads
// K(i+2) in its first segment and V(i+1) in its second into the buffers the next step uses, so no
// segment starts behind an LDS round trip.
//
// Numerics are those of fa_fwd_f16.hip / fa_fwd_f16_fast.hip (fp32 accumulation,
// log2-domain lazy rebase with threshold 8, l relative to the stored fp16 m).
// Replaces the reference's ForwardImpl (flash_attention.cu:425-1077) for these shapes.
#include "../fa_device.h"
#include "../fa_kernels.h"
#include "../fa_mfma.h"


namespace fa {
namespace {

using namespace mf;

constexpr int kD = 64;
constexpr int kBN = 64;                 // keys per tile
constexpr int kNW = 4;                  // waves per workgroup (one per SIMD)
constexpr int kBM = 64 * kNW;           // queries per workgroup
constexpr int kNS = 4;                  // ring slots for K and for V
constexpr int kQRow = 2 * kBM;          // bytes per Q row in LDS
constexpr int kTile = kD * kBN * 2;     // 8 KB
constexpr int kOffK = kD * kQRow;       // Q image [64][256] first (prologue only)
constexpr int kOffV = kOffK + kNS * kTile;
constexpr int kSmem = kOffV + kNS * kTile;
constexpr int kCPT = kD * 8 / (kNW * 64);  // 16-B chunks per thread per tile
constexpr float kRescaleThr = 8.f;

// one 32-query block of a wave
struct Blk {
  floatx16 st[2];  // Sᵀ of the current tile: keys 32t + 16(i>>3) + 8h + (i&7) in register i of half t
  uint32_t pw[4][4];  // P (fp16 pairs) of the current tile: dword x of PV k-step s
                      // (kept as dwords: extracting dwords from a bit-cast half8 miscompiles)
  floatx16 o[2];   // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
  floatx16 negm;   // -m_run broadcast: the C operand of every Sᵀ chain
  half8 qf[4];     // Q * scale * log2(e), k-step s = channels 16s .. 16s+15
  float m_run, l0, l1, m_max, thr;
  int qi, klo, kspan;
  int wlo_min, wlo_max, whi_min, whi_max;
  bool active;
};

// ablation bits (timing-only diagnostic builds, outputs are WRONG; FA_FWD_VARIANT=2100+bits)
constexpr int kANoBar = 1, kANoLoad = 2, kANoExp = 4, kANoFrag = 8, kANoRebase = 16;
// stamps (diagnostic build, FA_FWD_VARIANT=2132): per-wave s_memtime sums of the step's phases,
// written over l (the output l of that build is garbage)
constexpr int kAStamp = 32;
constexpr int kANoSoftmax = 64;  // P = cvt(Sᵀ) only: no max / exp / rebase / row sums

template <int POL, int ABL = 0>
__global__ __launch_bounds__(kNW * 64, 1) void fwd_f16_pp_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
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

  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;

  // ---- key range of the workgroup (rule-bounded)
  const int qlast = min(q0 + kBM, nq) - 1;
  int kb = 0, ke = nk;
  if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
  const int kt0 = (kb / kBN) * kBN;
  const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;

  // ---- staging: chunk j of this thread = 8 keys (16 B) of channel row c
  const int cm = tid & 7;
  uint32_t goff[kCPT], kwo[kCPT], vwo[kCPT];
  int crow[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int c = (tid + kNW * 64 * j) >> 3;
    crow[j] = c;
    goff[j] = (uint32_t)c * (uint32_t)nk * 2u + 16u * cm;
    kwo[j] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));
    vwo[j] = c * 128 + 16 * (cm ^ ((c >> 1) & 7));
  }
  // per-lane source offsets with the channel bound folded in (rows past d / v_d read as zeros)
  uint32_t koff[kCPT], voffs[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    koff[j] = crow[j] < d ? goff[j] : 0x80000000u;
    voffs[j] = crow[j] < vd ? goff[j] : 0x80000000u;
  }
  // Branch-free tile load (chunks past nk — the tail tile, tiles past the end — read as zeros):
  // loads and stores in the key loop carry no control flow, so the compiler's vmcnt waits stay
  // exact and a load issued two steps ahead is not drained early.
  auto load_tile = [&](u32x4 (&dst)[kCPT], __amdgpu_buffer_rsrc_t rs, const uint32_t (&off)[kCPT], int k0) {
    const bool in = k0 + 8 * cm < nk;
#pragma unroll
    for (int j = 0; j < kCPT; ++j)
      dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off[j] : 0x80000000u, 2 * min(k0, nk), 0);
  };
  auto load_chunk = [&](u32x4 (&dst)[kCPT], int j, __amdgpu_buffer_rsrc_t rs, const uint32_t (&off)[kCPT], int k0) {
    const bool in = k0 + 8 * cm < nk;
    dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off[j] : 0x80000000u, 2 * min(k0, nk), 0);
  };
  auto store_tile = [&](int off, const uint32_t (&wo)[kCPT], const u32x4 (&src)[kCPT]) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) *reinterpret_cast<lds_u32x4_t*>(smem + off + wo[j]) = src[j];
  };
  // staging buffers: buffer j holds K(i+3) / V(i+2) for the step i with i mod kNS == j; loads
  // are issued two steps before their store
  u32x4 kr[kNS][kCPT], vr[kNS][kCPT];

  // ---- prologue: Q, K(0..2), V(0..1) into LDS; K(3), V(2) into the staging registers
  {
    u32x4 pk[3][kCPT], pv[2][kCPT];
#pragma unroll
    for (int x = 0; x < 3; ++x)
      if (x < ntiles) load_tile(pk[x], krs, koff, kt0 + x * kBN);
#pragma unroll
    for (int x = 0; x < 2; ++x)
      if (x < ntiles) load_tile(pv[x], vrs, voffs, kt0 + x * kBN);
    for (int idx = tid; idx < kD * (kBM / 8); idx += kNW * 64) {  // Q [64][256], 64-B blocks XOR-swizzled by c&3
      const int c = idx / (kBM / 8), m = idx % (kBM / 8);
      const u32x4 v = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = v;
    }
#pragma unroll
    for (int x = 0; x < 3; ++x)
      if (x < ntiles) store_tile(kOffK + x * kTile, kwo, pk[x]);
#pragma unroll
    for (int x = 0; x < 2; ++x)
      if (x < ntiles) store_tile(kOffV + x * kTile, vwo, pv[x]);
    load_tile(kr[0], krs, koff, kt0 + 3 * kBN);
    load_tile(vr[0], vrs, voffs, kt0 + 2 * kBN);
    load_tile(kr[1], krs, koff, kt0 + 4 * kBN);
    load_tile(vr[1], vrs, voffs, kt0 + 3 * kBN);
  }
  __syncthreads();

  Blk A, B;
  auto init_blk = [&](Blk& X, int blk) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int cr = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 64 * w + 32 * blk + 16 * (g & 1) + 4 * tp;
        const half4 t = tr_read(smem + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
        if (e == 0) X.qf[s].lo = t; else X.qf[s].hi = t;
      }
      X.qf[s] = scale8(X.qf[s], c2);
      // (kept as plain values: the allocator places them)
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) X.o[u][i] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) X.negm[i] = 0.f;
    X.m_run = 0.f; X.l0 = 0.f; X.l1 = 0.f; X.m_max = kNegInf; X.thr = -__FLT_MAX__;
    const int wq0 = q0 + 64 * w + 32 * blk;
    X.qi = wq0 + r;
    X.active = wq0 < nq;
    X.klo = 0; X.kspan = 0; X.wlo_min = X.wlo_max = X.whi_min = X.whi_max = 0;
    if (POL == 1 && X.active) {
      int khi;
      key_interval(a.rule, min(X.qi, nq - 1), &X.klo, &khi);
      X.kspan = max(khi - X.klo + 1, 0);
      const int last = min(31, nq - 1 - wq0);
      X.wlo_min = __builtin_amdgcn_readfirstlane(X.klo);
      X.whi_min = __builtin_amdgcn_readfirstlane(khi);
      X.wlo_max = __builtin_amdgcn_readlane(X.klo, last);
      X.whi_max = __builtin_amdgcn_readlane(khi, last);
    }
  };
  init_blk(A, 0);
  init_blk(B, 1);

  // tile class of block X at key offset k0: 0 no allowed pair (skipped), 1 mixed (masked), 2 all allowed
  auto tcls = [&](const Blk& X, int k0) -> int {
    const int k1 = k0 + kBN - 1;
    if (POL == 0) return (k1 < nk) ? 2 : 1;
    if (!X.active || X.wlo_min > k1 || X.whi_max < k0) return 0;
    return (X.wlo_max <= k0 && X.whi_min >= k1 && k1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants; every read is base + immediate)
  //   K: lane 4q+p of a 16-lane group supplies channel row q, keys 4σ(p)..4σ(p)+3, σ swapping 1 and 2
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g >> 1) + tq) * 128 + (((32 * t + 16 * (g & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r, h) reads chunk 2s+h of channel row 32u + r
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  half8 kf[2][2][4];  // K fragments (two buffers, by step parity)
  half8 vf[2][4][2];  // V fragments (two buffers, by step parity)
  auto read_k = [&](int slot, int bf) {
    const lds_char_t* p = smem + kOffK + slot * kTile;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[bf][t][s].lo = tr_read(p + kbase[t] + (16 * s) * 128);
        kf[bf][t][s].hi = tr_read(p + kbase[t] + (16 * s + 4) * 128);
      }
  };
  auto read_v = [&](int slot, int bf) {
    const lds_char_t* p = smem + kOffV + slot * kTile;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) vf[bf][s][u] = read_b128(p + vbase[s] + 32 * u * 128);
  };
  // Sᵀ MFMAs of k-steps [s0, s1) for block X (K fragments of buffer bf)
  auto qk = [&](Blk& X, int s0, int s1, int bf) {
#pragma unroll
    for (int s = s0; s < s1; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        X.st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[bf][t][s], X.qf[s], s == 0 ? X.negm : X.st[t], 0, 0, 0);
  };
  // per-element rule / tail mask of a mixed tile; the key offset inside the tile is an immediate
  auto mask = [&](Blk& X, int k0) {
    const int lim = nk - k0 - 8 * h;            // POL 0: offset o is in range iff o < lim
    const int base = k0 + 8 * h - X.klo;        // POL 1: allowed iff base + o in [0, kspan)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 32 * t + 16 * (i >> 3) + (i & 7);
        const bool ok = (POL == 1) ? ((unsigned)(base + o) < (unsigned)X.kspan) : (o < lim);
        X.st[t][i] = ok ? X.st[t][i] : kNegInf;
      }
  };
  auto rowmax = [&](Blk& X) -> float {
    float mx0 = fmaxf(X.st[0][0], X.st[0][1]), mx1 = fmaxf(X.st[1][0], X.st[1][1]);
#pragma unroll
    for (int i = 2; i < 16; i += 2) {
      mx0 = fmaxf(fmaxf(mx0, X.st[0][i]), X.st[0][i + 1]);
      mx1 = fmaxf(fmaxf(mx1, X.st[1][i]), X.st[1][i + 1]);
    }
    const float mt = max_pair32(fmaxf(mx0, mx1));
    X.m_max = fmaxf(X.m_max, X.m_run + mt);
    return mt;
  };
  // P = exp2(Sᵀ) in fp16 (the PV B operand), one pinned dword at a time: pinned, the
  // exponentials stay in the segment that issues them (unpinned they sink next to their
  // users, the next segment's MFMAs).  (Element access through a pinned half8 / u32x4
  // miscompiles with this toolchain, hence the dword-by-dword form.)
  auto exp_cvt = [&](Blk& X) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const float s0 = X.st[s >> 1][8 * (s & 1) + 2 * x], s1 = X.st[s >> 1][8 * (s & 1) + 2 * x + 1];
        const half2v p2 = (ABL & kANoExp) ? half2v{(_Float16)s0, (_Float16)s1}
                                          : half2v{(_Float16)__builtin_amdgcn_exp2f(s0),
                                                   (_Float16)__builtin_amdgcn_exp2f(s1)};
        X.pw[s][x] = __builtin_bit_cast(uint32_t, p2);
        asm volatile("" : "+v"(X.pw[s][x]));
      }
    }
  };
  // row sums of the final P (fp32 dot2 over the fp16 pairs)
  auto row_sums = [&](Blk& X) {
    if constexpr ((ABL & kANoSoftmax) != 0) return;
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      X.l0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, X.pw[s][0]), one2, X.l0, false);
      X.l1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, X.pw[s][1]), one2, X.l1, false);
      X.l0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, X.pw[s][2]), one2, X.l0, false);
      X.l1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, X.pw[s][3]), one2, X.l1, false);
    }
    asm volatile("" : "+v"(X.l0), "+v"(X.l1));
  };
  // Softmax of a tile for block X up to the row sums.  The exponentials are computed
  // speculatively against the current m_run, beside the row max; only when the tile max
  // passed the threshold (or seeds m_run — rare) are O, l, Sᵀ and -m rebased and P recomputed.
  // So the branch on the max does not hold up the exponentials.
  auto softmax = [&](Blk& X) {
    if constexpr ((ABL & kANoSoftmax) != 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const half2v p2 = {(_Float16)X.st[s >> 1][8 * (s & 1) + 2 * x], (_Float16)X.st[s >> 1][8 * (s & 1) + 2 * x + 1]};
          X.pw[s][x] = __builtin_bit_cast(uint32_t, p2);
          asm volatile("" : "+v"(X.pw[s][x]));
        }
      return;
    }
    const float mt = rowmax(X);
    exp_cvt(X);
    if (!(ABL & kANoRebase) && __any(mt > X.thr)) {
      const bool unset = X.thr < 0.f;
      const bool seed = unset && (mt > X.thr);
      const float delta = unset ? (seed ? mt : 0.f) : fmaxf(mt, 0.f);
      const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
      X.m_run += delta;
      X.thr = (unset && !seed) ? X.thr : kRescaleThr;
      X.l0 *= alpha;
      X.l1 *= alpha;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) X.o[u][i] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        X.st[0][i] -= delta;
        X.st[1][i] -= delta;
        X.negm[i] = -X.m_run;
      }
      exp_cvt(X);
    }
  };
  auto pv = [&](Blk& X, int s0, int s1, int bf) {
#pragma unroll
    for (int s = s0; s < s1; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const half8 p = __builtin_bit_cast(half8, u32x4{X.pw[s][0], X.pw[s][1], X.pw[s][2], X.pw[s][3]});
        X.o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[bf][s][u], p, X.o[u], 0, 0, 0);
      }
  };

  // tiles a rule leaves partly or wholly disallowed, and phantom tiles past the end, are masked
  auto need_mask = [&](const Blk& X, int k0) -> bool {
    return k0 >= kt0 + ntiles * kBN || tcls(X, k0) != 2;
  };

  // ---- prologue compute: Sᵀ(0) of both blocks, softmax of A(0); K(1) and V(0) fragments
  if (ntiles > 0) {
    read_k(0, 0);
    qk(A, 0, 4, 0);
    qk(B, 0, 4, 0);
    read_k(1, 1);  // (stale when ntiles == 1: a phantom tile, fully masked)
    read_v(0, 0);
    if (need_mask(A, kt0)) mask(A, kt0);
    softmax(A);
    row_sums(A);
  }

  // ---- step i (ring slot c = i mod 4, fragment buffer p = i mod 2): K(i+1) fragments are in kf[p ^ 1],
  // V(i) fragments in vf[p] on entry.  Every step has the same straight-line shape: tiles a rule leaves
  // partly (or wholly) disallowed for a block are masked in a rare uniform branch, and the last step
  // issues a phantom Sᵀ for tile i+1 (stale LDS, fully masked, never multiplied into O).
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  auto stamp = [&](int k) {
    if constexpr ((ABL & kAStamp) != 0) {
      __builtin_amdgcn_sched_barrier(0);
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (k >= 0) st_acc[k] += t - st_prev;
      st_prev = t;
    }
  };
  auto step = [&](auto C_, int it) {
    constexpr int c = decltype(C_)::value, p = c & 1;
    stamp(-1);
    if (!(ABL & kANoBar)) __builtin_amdgcn_s_barrier();
    stamp(0);
    const int k0 = kt0 + it * kBN;
    // Stores are unconditional: past the end they write zeros into slots nobody reads unmasked.

    // segment 2i: Sᵀ A(i+1) | softmax B(i) | PV A(i); K(i+2) fragments into the other buffer
    if (need_mask(B, k0)) mask(B, k0);
    stamp(1);
    store_tile(kOffK + ((c + 3) % kNS) * kTile, kwo, kr[c]);  // K(i+3) over K(i-1)
    if (!(ABL & kANoLoad)) load_chunk(kr[(c + 2) % kNS], 0, krs, koff, kt0 + (it + 5) * kBN);
    qk(A, 0, 4, p ^ 1);
    pv(A, 0, 2, p);
    softmax(B);
    stamp(2);
    if (!(ABL & kANoLoad)) load_chunk(kr[(c + 2) % kNS], 1, krs, koff, kt0 + (it + 5) * kBN);
    if (!(ABL & kANoFrag)) read_k((c + 2) % kNS, p);
    row_sums(B);
    pv(A, 2, 4, p);
    stamp(3);

    // segment 2i+1: Sᵀ B(i+1) | softmax A(i+1) | PV B(i); V(i+1) fragments into the other buffer
    if (need_mask(A, k0 + kBN)) mask(A, k0 + kBN);
    store_tile(kOffV + ((c + 2) % kNS) * kTile, vwo, vr[c]);  // V(i+2) over V(i-2)
    if (!(ABL & kANoLoad)) load_chunk(vr[(c + 2) % kNS], 0, vrs, voffs, kt0 + (it + 4) * kBN);
    qk(B, 0, 4, p ^ 1);
    pv(B, 0, 2, p);
    softmax(A);
    stamp(4);
    if (!(ABL & kANoLoad)) load_chunk(vr[(c + 2) % kNS], 1, vrs, voffs, kt0 + (it + 4) * kBN);
    row_sums(A);
    pv(B, 2, 4, p);
    // this step's LDS stores are complete before any wave reaches the next barrier; the V(i+1)
    // reads (for the next step's PVs, a segment of Sᵀ MFMAs later) go after that wait
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (!(ABL & kANoFrag)) read_v((c + 1) % kNS, p ^ 1);
    stamp(5);
  };
  for (int it = 0; it < ntiles; it += kNS) {
    step(IC<0>{}, it);
    if (it + 1 < ntiles) step(IC<1>{}, it + 1);
    if (it + 2 < ntiles) step(IC<2>{}, it + 2);
    if (it + 3 < ntiles) step(IC<3>{}, it + 3);
  }

  // ---- epilogue
  __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
  float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
  __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
  auto finish = [&](Blk& X) {
    if (!X.active) return;
    const float l_tot = sum_pair32(X.l0 + X.l1);
    const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
    if (X.qi >= nq) return;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (v < vd) O[(int64_t)v * nq + X.qi] = __float2half(X.o[u][i] * inv);
      }
    if (h == 0) {
      if (l_tot > 0.f) {
        const __half mT = __float2half(X.m_max * kLn2);
        // l relative to the STORED (rounded) m, so exp(s - m)/l is exact downstream
        lo[X.qi] = l_tot * __builtin_amdgcn_exp2f(X.m_run - __half2float(mT) * kLog2e);
        mo[X.qi] = mT;
      } else {
        lo[X.qi] = 0.f;
        mo[X.qi] = neg_inf_approx<__half>();
      }
    }
  };
  finish(A);
  finish(B);
  if constexpr ((ABL & kAStamp) != 0) {
    if (lane < 6 && q0 + 64 * w + 8 <= nq) {
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 6; ++k) v = (lane == k) ? st_acc[k] : v;
      lo[q0 + 64 * w + lane] = (float)v;
    }
  }
}

}  // namespace

bool fwd_f16_pp_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return dm > 32 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) &&
         rule_is_interval(a.rule) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16_pp(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  auto kern = a.rule.policy == 0 ? fwd_f16_pp_kernel<0> : fwd_f16_pp_kernel<1>;
  switch (diag_variant("FA_FWD_VARIANT") - 2100) {  // ablations, full policy only (timing diagnostics)
    case 1: kern = fwd_f16_pp_kernel<0, 1>; break;
    case 2: kern = fwd_f16_pp_kernel<0, 2>; break;
    case 3: kern = fwd_f16_pp_kernel<0, 3>; break;
    case 4: kern = fwd_f16_pp_kernel<0, 4>; break;
    case 8: kern = fwd_f16_pp_kernel<0, 8>; break;
    case 16: kern = fwd_f16_pp_kernel<0, 16>; break;
    case 11: kern = fwd_f16_pp_kernel<0, 11>; break;
    case 15: kern = fwd_f16_pp_kernel<0, 15>; break;
    case 32: kern = fwd_f16_pp_kernel<0, 32>; break;
    case 34: kern = fwd_f16_pp_kernel<0, 34>; break;
    case 40: kern = fwd_f16_pp_kernel<0, 40>; break;
    case 64: kern = fwd_f16_pp_kernel<0, 64>; break;
    case 75: kern = fwd_f16_pp_kernel<0, 75>; break;
    case 96: kern = fwd_f16_pp_kernel<0, 96>; break;
    default: break;
  }
  hipError_t e =
      set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
