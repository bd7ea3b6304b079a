// fa_fwd_f16_pingpong.hip — fp16 fused attention forward for 32 < max(d, v_d) <= 64,
// full policy and interval rules: eight waves (two per SIMD) in two groups that
// alternate MFMA and softmax phases ("ping-pong").
//
// At d = 64 a 32-query × 64-key tile is 16 MFMAs (512 matrix cycles) against ≈ 470
// cycles of VALU / transcendental issue.  One wave cannot overlap the two (its softmax
// depends on its own Sᵀ), and two free-running waves on a SIMD phase-lock behind the
// workgroup barrier so their MFMA and softmax phases collide.  Here the workgroup
// barrier itself keeps them apart: waves 0-3 (group 0) and waves 4-7 (group 1) share
// the four SIMDs, and every barrier interval is an MFMA phase for one group and a
// VALU phase for the other:
//
//   interval  2i  : group 0 MFMA(i)      | group 1 VALU(i-1)
//   interval 2i+1 : group 0 VALU(i)      | group 1 MFMA(i)
//
// (both groups run the same loop; group 1 enters it one barrier late)
//
//   MFMA(i) = Sᵀ MFMAs of tile i + PV MFMAs of tile i-1 (16 MFMAs), beside all of the
//             wave's LDS traffic: K(i+1) / V(i) fragment reads, its share of the staging
//   VALU(i) = softmax of tile i (mask, max, speculative exp2, rare rebase, row sums)
//
// K/V tiles move global → registers (three steps ahead) → LDS; each thread owns one 16-B
// chunk of every tile and stores it in its own MFMA phase, so a tile is complete and
// published after the barrier that ends the second group's MFMA phase.  LDS images and
// operand layouts are those of fa_fwd_f16_pp.hip (K: transposed reads with the key
// permutation that makes P's k-step registers contiguous keys; V: plain rows, chunks
// XOR-swizzled by (c>>1)&7).  Rings of three slots for K and V.
//
// Numerics as fa_fwd_f16.hip (fp32 accumulation, log2-domain lazy rebase at 8, l
// relative to the stored fp16 m), except that the rebase check runs on the packed fp16
// exponentials (kFPMax): m is exact for tiles that rebased and m_run + log2(max P) for the
// others (< 4.9e-4 from the exact max).  Replaces the reference's ForwardImpl
// (flash_attention.cu:425-1077) for these shapes.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"
#include "fa_softmax_stream.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 64;
constexpr int kBN = 64;              // keys per tile
constexpr int kNW = 8;               // waves per workgroup, two per SIMD
constexpr int kBM = 32 * kNW;        // queries per workgroup
constexpr int kQRow = 2 * kBM;       // bytes per Q row in LDS
constexpr int kTile = kD * kBN * 2;  // 8 KB
constexpr int kOffK = kD * kQRow;    // Q image [64][256] first (prologue only)
// ring slots for K and for V: 3 with register staging, 5 with LDS-DMA staging (kFDma)
template <bool DMA> struct Ring {
  static constexpr int kNS = DMA ? 5 : 3;
  static constexpr int kOffV = kOffK + kNS * kTile;
  static constexpr int kSmem = kOffV + kNS * kTile;
};
constexpr float kRescaleThr = 8.f;

// structure flags (FA_FWD_VARIANT=22xx selects them for A/B timing)
constexpr int kFPrio = 1;      // s_setprio 1 over each MFMA phase (the default)
constexpr int kFStamp = 2;     // diagnostic: per-wave s_memtime sums per phase part, written over l (l garbage)
constexpr int kFSumsLate = 4;  // row sums of P(i-1) in MFMA(i) instead of VALU(i-1) (measured slower)
// ablations (timing diagnostics, outputs WRONG): no exp2 (P = cvt(S)), no row max / rebase, no row sums
constexpr int kANoExp = 8, kANoMax = 16, kANoSums = 32;
// ... and in the MFMA phase: no staging loads, no LDS stores, no fragment reads
constexpr int kANoLoad = 64, kANoStore = 128, kANoFrag = 256;
// staging by LDS-DMA (buffer_load ... lds straight into the ring, no VGPR round trip / ds_write)
constexpr int kFDma = 512;
// (with kFDma) the LDS-DMA issued by inline assembly: hipcc does not see an LDS write, so it adds no
// vmcnt(0) before the later fragment reads (it does for its own LDS-DMA builtin, which it cannot
// prove disjoint from them); the waits are the explicit vmcnt(6) before each barrier
constexpr int kFDmaAsm = 1 << 23;
// row sums on the matrix pipe: one v_mfma_f32_16x16x32_f16 per PV k-step in the MFMA phase, its A
// operand a 0/1 selector (row 0 sums the P columns of queries 0-15, row 1 those of 16-31), instead
// of 16 v_dot2c in the softmax phase; lanes 0-15 hold the running sums of queries c and 16 + c
constexpr int kFSumsMfma = 1 << 24;
// diagnostic: workgroup timeline (s_memrealtime at entry / after the prologue / after the loop /
// at exit, cycle counts, HW_ID, XCC_ID) written as raw words over the block's first l entries
constexpr int kFStampWG = 2048;
// the MFMA phase's staging stores after its MFMAs and fragment reads (their vmcnt waits and
// store-path cycles under the running PV MFMAs); lgkmcnt(0) at the start of the VALU phase
constexpr int kFStoresLate = 4096;
// full policy: the K(i+1) / V(i) fragment reads interleaved with the MFMAs that free their
// registers (sched_group_barrier), so the four waves of a group spread their LDS traffic over the
// phase instead of bursting it between the Sᵀ and PV MFMAs.  The MFMAs become unconditional: P is
// zeroed for a skipped tile and V's fragments start at zero.
constexpr int kFInterleave = 8192;
constexpr int kFIlvFine = 16384;  // ... one MFMA at a time (2 / 1 reads after each)
constexpr int kFIlvStores = 32768;  // ... and the staging stores / loads pinned after the 2nd MFMA pair of each half
constexpr int kFIlvAt0 = 65536;     // ... (after the 1st pair)
constexpr int kFIlvAt2 = 131072;    // ... (after the 3rd pair)
// row sums into four running fp32 accumulators that live across tiles (rescaled at a rebase),
// instead of four per-tile chains folded into l0 / l1: 10 fewer VALU per tile
constexpr int kFSumsAcc = 262144;
// (with kFSumsAcc) the tile's row sums as fp32 adds of the exponentials inside exp_cvt instead of
// v_dot2c on the packed P (v_dot2c is priced well above a plain add beside MFMAs)
constexpr int kFSumsF32 = 524288;
// the per-tile rebase check on this lane's half of the row (32 keys) with no cross-lane step; the
// exact row max is formed only inside the (rare) rebase branch, and the m output's running max
// stays per lane until the epilogue combines the two halves once
constexpr int kFHalfMax = 1048576;
// rebase check and m on P: the tile max is taken over the packed fp16 exponentials (8
// v_pk_maximum3_f16 instead of 16 fp32 max3 plus a cross-lane step), tested against 2^thr; the
// exact fp32 row max is formed only in the (rare) rebase branch.  m = m_run + log2(max P) for the
// tiles of the current epoch (fp16 rounding of P: |error| <= 2^-11 log2(e) in log2 units, i.e.
// < 4.9e-4 in m), exact for the tiles that rebased.
constexpr int kFPMax = 1 << 22;
// the exp2 / pack / packed-max part of the softmax as a hand-ordered stream (fa_softmax_stream.h):
// conversions one pair (kFAsmSm) or two pairs (kFAsmSm2) behind their exponentials
constexpr int kFAsmSm = 1 << 25, kFAsmSm2 = 1 << 26;

template <int POL, int F>
__global__ __launch_bounds__(kNW * 64, 2) void fwd_f16_pingpong_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr float kNegInf = -__builtin_huge_valf();
  constexpr bool DMA = (F & kFDma) != 0;
  constexpr int kNS = Ring<DMA>::kNS;
  constexpr int kOffV = Ring<DMA>::kOffV;

  uint64_t wg_t0 = 0, wg_c0 = 0;
  if constexpr ((F & kFStampWG) != 0) {
    wg_t0 = __builtin_amdgcn_s_memrealtime();
    wg_c0 = __builtin_amdgcn_s_memtime();
  }
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;  // latest (heaviest under causal) blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2;  // waves w and w+4 share a SIMD
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

  // ---- staging: this thread owns chunk `tid` of every tile = 8 keys (16 B) of channel row c
  const int cm = tid & 7, crow = tid >> 3;
  const uint32_t goff = (uint32_t)crow * (uint32_t)nk * 2u + 16u * cm;
  const uint32_t koff = crow < d ? goff : 0x80000000u, voff = crow < vd ? goff : 0x80000000u;
  const uint32_t kwo = crow * 128 + ((cm * 16) ^ ((crow & 2) << 5));
  const uint32_t vwo = crow * 128 + 16 * (cm ^ ((crow >> 1) & 7));
  // branch-free (exact vmcnt waits): chunks past nk — the tail, tiles past the end — read as zeros
  auto load = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, int k0) -> u32x4 __attribute__((always_inline)) {
    const bool in = k0 + 8 * cm < nk;
    return __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off : 0x80000000u, 2 * min(k0, nk), 0);
  };
  auto store = [&](int off, u32x4 v) __attribute__((always_inline)) { *reinterpret_cast<lds_u32x4_t*>(smem + off) = v; };
  // LDS-DMA: wave w fills bytes [1024w, 1024w + 1024) of a tile image, lane L the 16 B at 16L:
  // row c = 8w + L/8, position L%8, i.e. source chunk cm = pos ^ swizzle(c) (the images' XORs)
  const int dpos = lane & 7, drow = 8 * w + (lane >> 3);
  const int kcm = dpos ^ (4 * ((drow >> 1) & 1)), vcm = dpos ^ ((drow >> 1) & 7);
  const uint32_t kdoff = drow < d ? (uint32_t)drow * (uint32_t)nk * 2u + 16u * kcm : 0x80000000u;
  const uint32_t vdoff = drow < vd ? (uint32_t)drow * (uint32_t)nk * 2u + 16u * vcm : 0x80000000u;
  auto dma = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, int cmx, int k0, int lds_off) __attribute__((always_inline)) {
    const bool in = k0 + 8 * cmx < nk;
    if constexpr ((F & kFDmaAsm) != 0) {
      // M0 = the wave's LDS destination (lane L writes its 16 B at M0 + 16 L)
      const uint32_t m0v = (uint32_t)(uintptr_t)(smem + lds_off) + 1024u * (uint32_t)w;
      // (s_nop 0: the one wait state between the SALU write of M0 and an LDS-DMA that reads it)
      asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                   :
                   : "v"(in ? off : 0x80000000u), "s"(rs), "s"(2 * min(k0, nk)), "{m0}"(m0v)
                   : "memory");
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(smem + lds_off + 1024 * w),
                                               16, in ? off : 0x80000000u, 2 * min(k0, nk), 0, 0);
    }
  };

  u32x4 kst[3], vst[3];
  if constexpr (DMA) {
    // ---- prologue: K(0..4), V(0..3) by LDS-DMA, Q through registers
#pragma unroll
    for (int j = 0; j < kNS; ++j) dma(krs, kdoff, kcm, kt0 + j * kBN, kOffK + j * kTile);
#pragma unroll
    for (int j = 0; j < kNS - 1; ++j) dma(vrs, vdoff, vcm, kt0 + j * kBN, kOffV + j * kTile);
    for (int idx = tid; idx < kD * (kBM / 8); idx += kNW * 64) {  // Q [64][256], 64-B blocks XOR-swizzled by c&3
      const int c = idx / (kBM / 8), m = idx % (kBM / 8);
      const u32x4 v = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = v;
    }
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): the DMA'd tiles have landed
  } else {
  // ---- prologue: Q, K(0..2), V(0..1) into LDS; K(3..5), V(2..4) into the staging registers
  // (set j serves MFMA(i) with i mod 3 == j; loads run three steps ahead of their store)
  {
    // every load of the prologue in flight at once (the staging registers' too): one memory
    // latency before the loop instead of two
    u32x4 kp[3], vp[2];
#pragma unroll
    for (int j = 0; j < 3; ++j) kp[j] = load(krs, koff, kt0 + j * kBN);
#pragma unroll
    for (int j = 0; j < 2; ++j) vp[j] = load(vrs, voff, kt0 + j * kBN);
#pragma unroll
    for (int j = 0; j < kNS; ++j) {
      kst[j] = load(krs, koff, kt0 + (3 + j) * kBN);
      vst[j] = load(vrs, voff, kt0 + (2 + j) * kBN);
    }
    // Q [64][256], 64-B blocks XOR-swizzled by c&3: four chunks a thread, all loads before the stores
    // (a rolled loop here serialised four memory latencies: ~6000 cycles of prologue)
    constexpr int kQPT = kD * (kBM / 8) / (kNW * 64);
    u32x4 qv[kQPT];
    if (qvec) {  // branch-free buffer loads (chunks past d or nq read as zeros)
      const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Q, 2u * d * nq);
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int idx = tid + j * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        const bool in = c < d && q0 + 8 * m < nq;
        qv[j] = __builtin_amdgcn_raw_buffer_load_b128(qrs, in ? (uint32_t)c * (uint32_t)nq * 2u + 16u * m : 0x80000000u,
                                                      2 * q0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < kQPT; ++j) {
        const int idx = tid + j * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        qv[j] = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, false) : u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
      const int idx = tid + j * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) store(kOffK + j * kTile + kwo, kp[j]);
#pragma unroll
    for (int j = 0; j < 2; ++j) store(kOffV + j * kTile + vwo, vp[j]);
  }
  }
  __syncthreads();

  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r]
  half8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int cr = 16 * s + 8 * (g >> 1) + 4 * e + tq;
      const int col = 32 * w + 16 * (g & 1) + 4 * tp;
      const half4 t = tr_read(smem + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
      if (e == 0) qf[s].lo = t; else qf[s].hi = t;
    }
    qf[s] = scale8(qf[s], c2);
  }

  const int wq0 = q0 + 32 * w;
  const int qi = wq0 + r;
  const bool wave_active = wq0 < nq;
  // POL 1: this lane's allowed keys [klo, klo + kspan) and the wave's bounds on them
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
  // tile class for this wave: 0 no allowed pair (skipped), 1 mixed (masked), 2 all allowed
  auto tcls = [&](int it) -> int __attribute__((always_inline)) {
    if (it < 0 || it >= ntiles) return 0;
    const int k0 = kt0 + it * kBN, k1 = k0 + kBN - 1;
    if (POL == 0) return (k1 < nk) ? 2 : 1;
    if (!wave_active || wlo_min > k1 || whi_max < k0) return 0;
    return (wlo_max <= k0 && whi_min >= k1 && k1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants)
  //   K: lane 4q+p of a 16-lane group supplies channel row q, keys 4σ(p)..4σ(p)+3, σ swapping 1 and 2,
  //      so register i of Sᵀ half t holds key 32t + 16(i>>3) + 8h + (i&7)
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g >> 1) + tq) * 128 + (((32 * t + 16 * (g & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r, h) reads chunk 2s+h of channel row 32u + r
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  half8 kf[2][4];  // K fragments for the next Sᵀ
  half8 vf[4][2];  // V fragments for the next PV
  // (the builtin LDS-DMA's vmcnt(0) before every fragment read defeats the interleave; the inline-asm
  // DMA has none)
  constexpr bool ILV = (F & kFInterleave) != 0 && POL == 0 && (!DMA || (F & kFDmaAsm) != 0);
  if constexpr (ILV) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) vf[s][u][e] = (_Float16)0.f;
  }
  auto read_k = [&](int slot) __attribute__((always_inline)) {
    const lds_char_t* p = smem + kOffK + slot * kTile;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[t][s].lo = tr_read(p + kbase[t] + (16 * s) * 128);
        kf[t][s].hi = tr_read(p + kbase[t] + (16 * s + 4) * 128);
      }
  };
  auto read_v = [&](int slot) __attribute__((always_inline)) {
    const lds_char_t* p = smem + kOffV + slot * kTile;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) vf[s][u] = read_b128(p + vbase[s] + 32 * u * 128);
  };

  floatx16 st[2];      // Sᵀ of the tile being softmaxed
  uint32_t pw[4][4];   // P (fp16 pairs), dword x of PV k-step s (dwords: extracting them from a
                       // bit-cast half8 miscompiles with this toolchain)
  floatx16 o[2];       // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
  floatx16 negm;       // -m_run broadcast: the C operand of every Sᵀ chain
  if constexpr (ILV) {  // PV(-1) runs unconditionally: P starts at zero
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o[0][i] = 0.f;
    o[1][i] = 0.f;
    negm[i] = 0.f;
  }
  float m_run = 0.f, l0 = 0.f, l1 = 0.f, m_max = kNegInf, thr = -__FLT_MAX__;
  constexpr bool PMAX = (F & kFPMax) != 0;
  half2v pmr = {(_Float16)0.f, (_Float16)0.f};  // PMAX: running max of P over the current epoch (per lane)
  _Float16 thr_h = (_Float16)-1.f;              // PMAX: 2^thr once seeded; -1 (always exceeded) before

  auto mask = [&](int k0) __attribute__((always_inline)) {
    const int lim = nk - k0 - 8 * h;       // POL 0: offset o is in range iff o < lim
    const int base = k0 + 8 * h - klo;     // POL 1: allowed iff base + o in [0, kspan)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = 32 * t + 16 * (i >> 3) + (i & 7);
        const bool ok = (POL == 1) ? ((unsigned)(base + off) < (unsigned)kspan) : (off < lim);
        st[t][i] = ok ? st[t][i] : kNegInf;
      }
  };
  float lacc[4] = {0.f, 0.f, 0.f, 0.f};  // kFSumsAcc: running row sums (chains x = 0..3)
  constexpr bool MSUM = (F & kFSumsMfma) != 0;
  floatx4 lsum = {0.f, 0.f, 0.f, 0.f};     // MSUM: lane c < 16: [0] query c, [1] query 16 + c
  half8 lsel;                               // MSUM: selector row (lane & 15) over k = 8 (lane >> 4) + j
  {
    const int srow = lane & 15, sg = (lane >> 4) & 1;
    const _Float16 sv = (_Float16)(((srow == 0 && sg == 0) || (srow == 1 && sg == 1)) ? 1.f : 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) lsel[j] = sv;
  }
  float ts[4];                            // kFSumsF32: this tile's row sums (four chains)
  auto row_sums = [&]() __attribute__((always_inline)) {
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
    if constexpr ((F & kFSumsF32) != 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) lacc[x] += ts[x];
      return;
    }
    if constexpr ((F & kFSumsAcc) != 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 4; ++x)
          lacc[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, pw[s][x]), one2, lacc[x], false);
      return;
    }
    float ls[4] = {0.f, 0.f, 0.f, 0.f};  // four chains, folded into l0 / l1 once
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x) ls[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, pw[s][x]), one2, ls[x], false);
    l0 += ls[0] + ls[2];
    l1 += ls[1] + ls[3];
  };
  auto exp_cvt = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const float s0 = st[s >> 1][8 * (s & 1) + 2 * x], s1 = st[s >> 1][8 * (s & 1) + 2 * x + 1];
        if constexpr ((F & kFSumsF32) != 0) {
          const float e0 = __builtin_amdgcn_exp2f(s0), e1 = __builtin_amdgcn_exp2f(s1);
          pw[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)e0, (_Float16)e1});
          ts[x] = (s == 0) ? e0 + e1 : ts[x] + e0 + e1;
          continue;
        }
        pw[s][x] = (F & kANoExp) ? __builtin_bit_cast(uint32_t, half2v{(_Float16)s0, (_Float16)s1})
                                 : __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0),
                                                                       (_Float16)__builtin_amdgcn_exp2f(s1)});
      }
  };
  // softmax of tile `it`: the exponentials are computed speculatively against m_run beside the
  // row max; only a seed or a max past the threshold (rare) rebases O, l, Sᵀ, -m and redoes them
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
  auto softmax_p = [&](int it, int cls) __attribute__((always_inline)) {
    if (cls == 1) mask(kt0 + it * kBN);
    half2v tm;
    if constexpr ((F & (kFAsmSm | kFAsmSm2)) != 0) {
      uint32_t pm;
      softmax_stream_tile<(F & kFAsmSm2) ? 2 : 1>(st, pw, pm);
      tm = __builtin_bit_cast(half2v, pm);
    } else {
      exp_cvt();
#pragma unroll
      for (int x = 0; x < 4; ++x)
        asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
      tm = pmax_tile();
    }
    const _Float16 tmx = __builtin_elementwise_maximum(tm[0], tm[1]);
    const half2v pmr_old = pmr;
    pmr = __builtin_elementwise_maximum(pmr, tm);
    if (__any(tmx > thr_h)) {
      // the exact fp32 row max of this tile (relative to m_run), both key halves
      float mx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) mx[j] = fmaxf(st[j >> 1][8 * (j & 1)], st[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
      for (int i = 2; i < 8; i += 2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mx[j] = fmaxf(fmaxf(mx[j], st[j >> 1][8 * (j & 1) + i]), st[j >> 1][8 * (j & 1) + i + 1]);
      const float mtf = max_pair32(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
      // close the epoch: its P maximum (approximate) and this tile (exact) into m_max
      const float pold = (float)__builtin_elementwise_maximum(pmr_old[0], pmr_old[1]);
      m_max = fmaxf(m_max, fmaxf(m_run + mtf, m_run + __log2f(pold)));
      const bool unset = thr < 0.f;
      const bool seed = unset && (mtf > thr);
      const float delta = unset ? (seed ? mtf : 0.f) : fmaxf(mtf, 0.f);
      const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
      m_run += delta;
      thr = (unset && !seed) ? thr : kRescaleThr;
      thr_h = (unset && !seed) ? (_Float16)-1.f : (_Float16)(1 << (int)kRescaleThr);
      if constexpr ((F & kFSumsAcc) != 0) {
#pragma unroll
        for (int x = 0; x < 4; ++x) lacc[x] *= alpha;
      }
      if constexpr (MSUM) {  // lane c's [1] holds query 16 + c: that lane's factor
        const float ahi = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * ((lane & 15) + 16), __float_as_int(alpha)));
        lsum[0] *= alpha;
        lsum[1] *= ahi;
      }
      l0 *= alpha;
      l1 *= alpha;
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
    if (!(F & (kFSumsLate | kANoSums | kFSumsMfma))) row_sums();
  };
  auto softmax = [&](int it, int cls) __attribute__((always_inline)) {
    if constexpr (PMAX) {
      softmax_p(it, cls);
      return;
    }
    if (cls == 1) mask(kt0 + it * kBN);
    // four independent max3 chains (one wave does the VALU work on its SIMD: latency shows)
    float mx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(st[j >> 1][8 * (j & 1)], st[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
    for (int i = 2; i < 8; i += 2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        mx[j] = fmaxf(fmaxf(mx[j], st[j >> 1][8 * (j & 1) + i]), st[j >> 1][8 * (j & 1) + i + 1]);
    constexpr bool HALF = (F & kFHalfMax) != 0;
    const float mth = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
    const float mt = (F & kANoMax) ? -1.f : (HALF ? mth : max_pair32(mth));
    m_max = fmaxf(m_max, m_run + mt);
    exp_cvt();
#pragma unroll
    for (int x = 0; x < 4; ++x)  // pinned here: else they sink past the (rare) rebase branch
      asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
    if (__any(mt > thr)) {
      const float mtf = HALF ? max_pair32(mth) : mt;  // the whole row's tile max
      const bool unset = thr < 0.f;
      const bool seed = unset && (mtf > thr);
      const float delta = unset ? (seed ? mtf : 0.f) : fmaxf(mtf, 0.f);
      const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
      m_run += delta;
      thr = (unset && !seed) ? thr : kRescaleThr;
      l0 *= alpha;
      l1 *= alpha;
      if constexpr ((F & kFSumsAcc) != 0) {
#pragma unroll
        for (int x = 0; x < 4; ++x) lacc[x] *= alpha;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o[0][i] *= alpha;
        o[1][i] *= alpha;
        st[0][i] -= delta;
        st[1][i] -= delta;
        negm[i] = -m_run;
      }
      exp_cvt();
    }
    if (!(F & (kFSumsLate | kANoSums | kFSumsMfma))) row_sums();
  };

  // MFMA(i): this wave's chunks of K(i+3) / V(i+2) into LDS (over K(i) / V(i-1), whose
  // fragments were read in MFMA(i-1)), loads of K(i+6) / V(i+5); Sᵀ of tile i; K(i+1)
  // fragments; PV of tile i-1 (P from VALU(i-1)); V(i) fragments.  The LDS traffic sits in the
  // MFMA phase, beside the matrix pipe, so the VALU phase is the softmax alone.
  auto mfma_phase = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;  // it mod 3
    if (F & kFPrio) __builtin_amdgcn_s_setprio(1);
    // (unconditional: past the end these move zeros into slots nobody reads unmasked)
    if constexpr (DMA) {
      // K(i+5) over K(i) (its fragments were read in MFMA(i-1)), V(i+4) over V(i-1)
      dma(krs, kdoff, kcm, kt0 + (it + kNS) * kBN, kOffK + c * kTile);
      dma(vrs, vdoff, vcm, kt0 + (it + kNS - 1) * kBN, kOffV + ((c + kNS - 1) % kNS) * kTile);
    } else {
      if (!(F & (kANoStore | kFStoresLate))) {
        store(kOffK + c * kTile + kwo, kst[c]);
        store(kOffV + ((c + 2) % kNS) * kTile + vwo, vst[c]);
      }
      if (!(F & (kANoLoad | kFStoresLate))) {
        kst[c] = load(krs, koff, kt0 + (it + 6) * kBN);
        vst[c] = load(vrs, voff, kt0 + (it + 5) * kBN);
      }
    }
    if constexpr (ILV) {
      const lds_char_t* pk = smem + kOffK + ((c + 1) % kNS) * kTile;
      const lds_char_t* pv = smem + kOffV + c * kTile;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qf[s], s == 0 ? negm : st[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (F & kANoFrag) break;
          kf[t][s].lo = tr_read(pk + kbase[t] + (16 * s) * 128);
          kf[t][s].hi = tr_read(pk + kbase[t] + (16 * s + 4) * 128);
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const half8 p = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
#pragma unroll
        for (int u = 0; u < 2; ++u) o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, o[u], 0, 0, 0);
        if constexpr (MSUM) lsum = __builtin_amdgcn_mfma_f32_16x16x32_f16(lsel, p, lsum, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (!(F & kANoFrag)) vf[s][u] = read_b128(pv + vbase[s] + 32 * u * 128);
      }
      constexpr int kIlvAt = (F & kFIlvAt0) ? 0 : (F & kFIlvAt2) ? 2 : 1;
      if constexpr ((F & kFIlvFine) != 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
          if constexpr ((F & kFIlvStores) != 0) {
            if (s == kIlvAt) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // a staging store
            if (s == kIlvAt) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // a staging load
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          __builtin_amdgcn_sched_group_barrier(0x008, MSUM ? 3 : 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          if constexpr ((F & kFIlvStores) != 0) {
            if (s == kIlvAt) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            if (s == kIlvAt) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          }
        }
      }
    }
    if (!ILV && tcls(it) != 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qf[s], s == 0 ? negm : st[t], 0, 0, 0);
    }
    if (!ILV && !(F & kANoFrag)) read_k((c + 1) % kNS);
    if (!ILV && tcls(it - 1) != 0) {
      if (F & kFSumsLate) row_sums();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const half8 p = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
#pragma unroll
        for (int u = 0; u < 2; ++u) o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, o[u], 0, 0, 0);
        if constexpr (MSUM) lsum = __builtin_amdgcn_mfma_f32_16x16x32_f16(lsel, p, lsum, 0, 0, 0);
      }
    }
    if (!ILV && !(F & kANoFrag)) read_v(c);
    if constexpr ((F & kFStoresLate) != 0 && !DMA) {
      if (!(F & kANoStore)) {
        store(kOffK + c * kTile + kwo, kst[c]);
        store(kOffV + ((c + 2) % kNS) * kTile + vwo, vst[c]);
      }
      if (!(F & kANoLoad)) {
        kst[c] = load(krs, koff, kt0 + (it + 6) * kBN);
        vst[c] = load(vrs, voff, kt0 + (it + 5) * kBN);
      }
    }
    // DMA: the tiles issued three MFMA phases ago (K(i+2), V(i+1), read from MFMA(i+1) on) have
    // landed before this wave's next barrier: all but its six most recent DMAs are done
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0x0F76);  // vmcnt(6)
    // No lgkmcnt drain here: a wave's LDS operations complete in order, and each wave waits for
    // its fragment reads before the MFMAs that use them (MFMA(i+1)), which orders its stores of
    // this phase before any other wave reads those tiles (MFMA(i+2)) and its reads before any
    // wave overwrites their slots (MFMA(i+1) for itself, one interval later for the others).
    if (F & kFPrio) __builtin_amdgcn_s_setprio(0);
  };
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if constexpr ((F & kFStamp) != 0) {
      __builtin_amdgcn_sched_barrier(0);
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (k >= 0) st_acc[k] += t - st_prev;
      st_prev = t;
    }
  };
  // VALU(i): the softmax of tile i
  auto valu_phase = [&](int it) __attribute__((always_inline)) {
    if constexpr ((F & kFStoresLate) != 0) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): stores landed
    const int cls = tcls(it);
    stamp(3);
    if (cls != 0) softmax(it, cls);
    if constexpr (ILV) {
      if (cls == 0) {  // the next (unconditional) PV must add nothing
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
      }
    }
    stamp(4);
    stamp(5);
  };

  uint64_t wg_t1 = 0, wg_c1 = 0, wg_t2 = 0, wg_c2 = 0;
  if constexpr ((F & kFStampWG) != 0) {
    wg_t1 = __builtin_amdgcn_s_memrealtime();
    wg_c1 = __builtin_amdgcn_s_memtime();
  }
  // Both groups run the same loop (one code path keeps the register allocation sane); group 1
  // enters it one barrier late and group 0 leaves it one barrier late, so every barrier
  // interval pairs one group's MFMA(i) with the other's VALU phase.
  read_k(0);
  if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0xC07F);  // K(0)'s slot is DMA'd over in MFMA(0)
  if (grp == 1) __builtin_amdgcn_s_barrier();
  auto iter = [&](auto C_, int it) __attribute__((always_inline)) {
    stamp(-1);
    __builtin_amdgcn_s_barrier();
    stamp(0);
    mfma_phase(C_, it);
    stamp(1);
    __builtin_amdgcn_s_barrier();
    stamp(2);
    valu_phase(it);
  };
  // Whole groups of three iterations, none conditional (the last ones past the end only move
  // zeros): with no control flow around the staging loads, hipcc's vmcnt waits stay exact and
  // a store waits only for the load issued three steps earlier.
  for (int it = 0; it <= ntiles; it += kNS) {
    iter(IC<0>{}, it);
    iter(IC<1>{}, it + 1);
    iter(IC<2>{}, it + 2);
    if constexpr (kNS > 3) {
      iter(IC<3 % kNS>{}, it + 3);
      iter(IC<4 % kNS>{}, it + 4);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  if constexpr ((F & kFStampWG) != 0) {
    wg_t2 = __builtin_amdgcn_s_memrealtime();
    wg_c2 = __builtin_amdgcn_s_memtime();
  }

  // ---- epilogue
  if (!wave_active) return;
  if constexpr ((F & kFSumsAcc) != 0) l0 = (lacc[0] + lacc[1]) + (lacc[2] + lacc[3]);
  if constexpr ((F & kFHalfMax) != 0) m_max = max_pair32(m_max);
  if constexpr (PMAX)
    m_max = max_pair32(fmaxf(m_max, m_run + __log2f((float)__builtin_elementwise_maximum(pmr[0], pmr[1]))));
  float l_tot;
  if constexpr (MSUM) {  // query q = lane & 31 sits in lane q & 15, register q >> 4
    const int src = 4 * (lane & 15);
    const float s0 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(lsum[0])));
    const float s1 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(lsum[1])));
    l_tot = (r < 16) ? s0 : s1;
  } else {
    l_tot = sum_pair32(l0 + l1);
  }
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi >= nq) return;
  __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
  if (vd == kD) {
    // every channel in range: one buffer store per value, the lane's offset in a VGPR and the
    // channel's in an SGPR (the generic form below spends a 64-bit address, a compare and an
    // exec branch on each of the 32 stores)
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(O, 2u * vd * nq);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t cst = 32u * u + (i & 3) + 8u * (i >> 2);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(o[u][i] * inv)), ors, vlane,
                                              2u * cst * (uint32_t)nq, 0);
      }
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (v < vd) O[(int64_t)v * nq + qi] = __float2half(o[u][i] * inv);
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
  if constexpr ((F & kFStampWG) != 0) {  // diagnostic build: wave 0's timeline over the block's l
    const uint64_t t3 = __builtin_amdgcn_s_memrealtime(), c3 = __builtin_amdgcn_s_memtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804), xcc = __builtin_amdgcn_s_getreg(0xF814);
    const uint32_t vals[10] = {(uint32_t)wg_t0, (uint32_t)(wg_t0 >> 32), (uint32_t)(wg_t1 - wg_t0), (uint32_t)(wg_t2 - wg_t0),
                               (uint32_t)(t3 - wg_t0), (uint32_t)(wg_c1 - wg_c0), (uint32_t)(wg_c2 - wg_c0),
                               (uint32_t)(c3 - wg_c0), hw, xcc};
    if (w == 0 && lane < 10 && q0 + lane < nq) {
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < 10; ++k) v = (lane == k) ? vals[k] : v;
      reinterpret_cast<uint32_t*>(a.l)[bi * (int64_t)nq + q0 + lane] = v;
    }
  }
  if constexpr ((F & kFStamp) != 0) {  // diagnostic build: stamps over this wave's first l entries
    if (lane < 6 && wq0 + lane < nq) {
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 6; ++k) v = (lane == k) ? st_acc[k] : v;
      static_cast<float*>(a.l)[bi * (int64_t)nq + wq0 + lane] = (float)v;
    }
  }
}

template <int F>
hipError_t launch_t(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  auto kern = a.rule.policy == 0 ? fwd_f16_pingpong_kernel<0, F> : fwd_f16_pingpong_kernel<1, F>;
  constexpr int smem = Ring<(F & kFDma) != 0>::kSmem;
  hipError_t e =
      set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool fwd_f16_pingpong_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return dm > 32 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) &&
         (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) &&
         rule_is_interval(a.rule) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

// tuned (c2, MI355X): MFMA phases at priority 1, fragment reads and staging interleaved with
// the MFMAs (full policy; 0.5526-0.5716 ms against 0.595 for 2206), row sums in running
// accumulators (0.5451 against 0.5552 ms in one process; fp32 adds instead of v_dot2c: 0.5812
// against 0.5690; the half-row rebase check kFHalfMax: 0.5464, no gain), rebase check and m on
// the packed P (0.5395-0.5441 against 0.5512-0.5553 ms in one process)
constexpr int kFDefaultR1 = kFPrio | kFStoresLate | kFInterleave | kFIlvStores;
constexpr int kFDefaultR2 = kFDefaultR1 | kFSumsAcc;
constexpr int kFDefault = kFDefaultR2 | kFPMax;

hipError_t launch_fwd_f16_pingpong(const FwdArgs& a, hipStream_t s) {
#ifdef FA_DIAG
  switch (diag_variant("FA_FWD_VARIANT")) {
    case 2200: return launch_t<0>(a, s);
    case 2203: return launch_t<kFPrio | kFStamp>(a, s);
    case 2204: return launch_t<kFPrio | kFStampWG>(a, s);
    case 2206: return launch_t<kFPrio | kFStoresLate>(a, s);
    case 2207: return launch_t<kFPrio | kFStoresLate | kFInterleave>(a, s);
    case 2208: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvFine>(a, s);
    case 2209: return launch_t<kFPrio | kFInterleave>(a, s);
    case 2210: return launch_t<kFInterleave | kFStoresLate>(a, s);
    case 2213: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores>(a, s);
    case 2214: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFIlvAt0>(a, s);
    case 2215: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFIlvAt2>(a, s);
    case 2216: return launch_t<kFStoresLate | kFInterleave | kFIlvStores>(a, s);
    case 2274: return launch_t<kFPrio | kFStampWG | kANoLoad | kANoStore | kANoFrag>(a, s);
    case 2275: return launch_t<kFPrio | kFStampWG | kANoExp | kANoMax | kANoSums>(a, s);
    case 2276: return launch_t<kFPrio | kFStampWG | kANoLoad | kANoStore | kANoFrag | kANoExp | kANoMax | kANoSums>(a, s);
    case 2277: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFStampWG>(a, s);
    case 2278: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFStampWG | kANoLoad | kANoStore | kANoFrag>(a, s);
    case 2279: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFStampWG | kANoExp | kANoMax | kANoSums>(a, s);
    case 2280: return launch_t<kFPrio | kFStoresLate | kFInterleave | kFIlvStores | kFStampWG | kANoLoad | kANoStore | kANoFrag | kANoExp | kANoMax | kANoSums>(a, s);
    case 2212: return launch_t<kFPrio | kFDma>(a, s);
    case 2217: return launch_t<kFPrio | kFDma | kFDmaAsm>(a, s);
    case 2218: return launch_t<kFPrio | kFDma | kFDmaAsm | kFSumsAcc | kFPMax>(a, s);
    case 2230: return launch_t<kFDefault | kFDma | kFDmaAsm>(a, s);
    case 2233: return launch_t<kFDefault | kFSumsMfma>(a, s);
    case 2234: return launch_t<kFDefault | kFDma | kFDmaAsm | kFSumsMfma>(a, s);
    case 2231: return launch_t<(kFDefault & ~kFIlvStores) | kFDma | kFDmaAsm>(a, s);
    case 2232: return launch_t<(kFDefault & ~kFIlvStores) | kFDma | kFDmaAsm | kFIlvFine>(a, s);
    case 2205: return launch_t<kFPrio | kFSumsLate>(a, s);
    case 2211: return launch_t<kFPrio | kFStamp | kANoExp>(a, s);
    case 2219: return launch_t<kFPrio | kFStamp | kANoMax>(a, s);
    case 2235: return launch_t<kFPrio | kFStamp | kANoSums>(a, s);
    case 2259: return launch_t<kFPrio | kFStamp | kANoExp | kANoMax | kANoSums>(a, s);
    case 2260: return launch_t<kFPrio | kANoExp | kANoMax | kANoSums>(a, s);
    case 2264: return launch_t<kFPrio | kANoLoad>(a, s);
    case 2265: return launch_t<kFPrio | kANoStore>(a, s);
    case 2266: return launch_t<kFPrio | kANoFrag>(a, s);
    case 2267: return launch_t<kFPrio | kANoLoad | kANoStore | kANoFrag>(a, s);
    case 2268: return launch_t<kFPrio | kANoLoad | kANoStore | kANoFrag | kANoExp | kANoMax | kANoSums>(a, s);
    case 2201: return launch_t<kFPrio>(a, s);
    case 2290: return launch_t<kFDefaultR1>(a, s);  // round-1 default (per-tile row-sum chains)
    case 2291: return launch_t<kFDefaultR2 | kFSumsF32>(a, s);
    case 2292: return launch_t<kFDefaultR2 | kFHalfMax>(a, s);
    case 2293: return launch_t<kFDefaultR2>(a, s);  // round-2 default (exact fp32 row max every tile)
    case 2294: return launch_t<kFDefault | kANoSums>(a, s);            // timing only: no row sums (outputs wrong)
    case 2295: return launch_t<kFDefault | kANoExp | kANoMax | kANoSums>(a, s);  // timing only: no softmax
    case 2297: return launch_t<kFDefault | kANoExp>(a, s);             // timing only: no exp2 (outputs wrong)
    case 2298: return launch_t<kFDefault | kANoLoad | kANoStore>(a, s);  // timing only: no staging
    case 2299: return launch_t<kFDefault | kFStamp>(a, s);
    case 2240: return launch_t<kFDefault | kFAsmSm>(a, s);
    case 2241: return launch_t<kFDefault | kFAsmSm2>(a, s);
    case 2242: return launch_t<kFDefault | kFAsmSm | kFStamp>(a, s);
    default: break;
  }
#endif
  return launch_t<kFDefault>(a, s);
}

}  // namespace fa
