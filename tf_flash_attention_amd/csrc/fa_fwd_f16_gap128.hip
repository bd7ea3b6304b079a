// fa_fwd_f16_gap128.hip — fp16 fused attention forward for 64 < max(d, v_d) <= 128 (BASELINE config 3's
// forward) with ONE wave per SIMD and a hand-placed gap stream: the structure of csrc/diag/fa_fwd_f16_gap.hip
// (which loses to the ping-pong at d = 64) at D = 128, where it wins.
//
// Why D = 128 is where this structure should pay: a 32 x 64 tile's softmax is the same ~16 P dwords of
// fillers as at D = 64, but a segment now has 32 MFMAs (Sᵀ 8 k-steps x 2 key halves, PV 4 k-steps x 4
// channel quarters), so one P dword fills two gaps (one v_exp_f32 a gap: inside the <= 5 fillers / one
// 8-cycle instruction a 32x32x16 gap hides, MI355X_MICROARCH.md 'one wave per SIMD'); and a wave's 64
// queries read each K / V fragment once for two query blocks, half the LDS bytes per MFMA of the two-wave
// ping-pong (fa_fwd_f16_pingpong128.hip), whose MFMA phase is LDS-bound.
//
//   segment A of step i : Sᵀ A(i+1) (16 MFMAs), PV A(i) (16)  |  softmax B(i), row sums of P_B(i-1)
//   segment B of step i : Sᵀ B(i+1) (16 MFMAs), PV B(i) (16)  |  softmax A(i+1), row sums of P_A(i)
//
// Gap g of a segment: MFMA g and its share of the other block's softmax (the table at `gap` below): in gaps
// 0-23 half of P dword g/2 a gap (one v_exp_f32, preceded by the v_sub of the running reference: the scores
// leave the MFMA relative to 0), in gaps 24-27 one whole dword each, then the last packed-max folds, the
// tile's max and the rebase predicate (an SGPR pair), so the check after a segment is one scalar branch.
//
// Registers (one wave per SIMD, 512): VGPRs hold both blocks' scores and P, and the whole K(i+1) tile's
// fragments (read once, used by both segments); AGPRs hold both blocks' O (128), Q (64) and the whole V(i)
// tile's fragments (64).  No register is left for staging, so K / V reach LDS by LDS-DMA (inline-asm
// buffer_load ... lds, two steps ahead, four-slot rings, counted vmcnt waits; the lanes' source chunks
// permuted so each wave's contiguous 1 KB is the swizzled image).  LDS: K ring 64 KB, V ring 64 KB; the Q
// image [128][256] of the prologue lies over the K ring.
//
// Memory operations per step: V(i)'s 16 fragment reads one a gap in segment A's gaps 0-15 (asm ds_read_b128
// into AGPRs, waited by lgkmcnt before the PV MFMAs that use them), K(i+2)'s 32 transposed reads in segment
// B's gaps 2-17 (each into the registers the Sᵀ MFMA two gaps back finished with), the eight DMA pieces of
// K(i+4) / V(i+2) in the four lightest gaps of each segment (28-31).  One barrier a step.
//
// Rules: the full policy and interval rules (causal, 1d local), with the heavy / light block pairing of
// fa_fwd_f16_pingpong128.hip.  Numerics as fa_fwd_f16_gap.hip.  Replaces the reference's ForwardImpl
// (flash_attention.cu:425-1077) for these shapes: the default for the full and causal policies at
// 64 < max(d, v_d) <= 128 (config 3's forward; FA_FWD_VARIANT 2700 / 2701 force it / its other layout in the
// diagnostic library).
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 128;
constexpr int kBN = 64;                 // keys per tile
constexpr int kNW = 4;                  // waves per workgroup, one per SIMD
constexpr int kBM = 64 * kNW;           // queries per workgroup (block)
constexpr int kNS = 4;                  // ring slots for K and for V
constexpr int kQRow = 2 * kBM;          // bytes per Q row in the prologue image
constexpr int kTile = kD * kBN * 2;     // 16 KB
constexpr int kOffK = 0;                // K ring (the Q image [128][256] lies over it in the prologue)
constexpr int kOffV = kNS * kTile;      // V ring
constexpr int kSmem = 2 * kNS * kTile;  // 128 KB
constexpr int kPPW = kTile / 1024 / kNW;  // DMA pieces (1 KB) per wave per tile: 4
constexpr float kRescaleThr = 8.f;

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    static_for<B + 1, E>(f);
  }
}

// query blocks a workgroup runs: one (full policy), or the heavy / light pair of an interval rule
__host__ __device__ inline int64_t gap128_groups(int64_t nqb, int pol) { return pol == 0 ? nqb : (nqb + 1) / 2; }

struct Blk {
  floatx16 s[2];   // Sᵀ (VGPR), relative to 0: register i of half t = key 32t + 16(i>>3) + 8h + (i&7)
  floatx16 o[4];   // Oᵀ (AGPR): channels 32u + 8(i>>2) + 4h + (i&3)
  half8 q[8];      // Q * scale * log2(e), k-step s = channels 16s..16s+15 (AGPR)
  uint32_t p[16];  // P (fp16 pairs): dword x of PV k-step s at 4s + x
  float l[4];      // running row sums (four chains)
  uint32_t pm;     // packed max of the tile's P (the rebase check)
  half2v pmr;      // running packed max of P over the current epoch
  half2v pmr_old;  // pmr before the segment that forms the rebase predicate
  uint32_t tm;     // the tile's P max (fp16 in the low half), formed in gap 30
  uint32_t thr_bits;  // thr_h in the low half (the compare's operand)
  uint64_t sm;     // rebase predicate of the last softmax segment (lanes whose P max passed 2^thr)
  float m_run, m_max, thr;
  _Float16 thr_h;  // 2^thr once seeded; -1 (always exceeded) before
  // interval rules: this lane's allowed keys [klo, klo + kspan), and the block's wave-uniform bounds
  int klo, kspan, wlo_min, wlo_max, whi_min, whi_max;
  bool active;
};

#define G2_MFMA_C "v_mfma_f32_32x32x16_f16 %[d], %[a], %[b], 0"
#define G2_MFMA "v_mfma_f32_32x32x16_f16 %[d], %[a], %[b], %[d]"
#define G2_EVEN                                                                                           \
  "\n\tv_sub_f32 %[t0], %[s0], %[mr]\n\tv_exp_f32 %[t0], %[t0]\n\tv_fma_mix_f32 %[la], %[pn], 1.0, %[la] op_sel_hi:[1,0,0]"
#define G2_ODD                                                                        \
  "\n\tv_sub_f32 %[t1], %[s1], %[mr]\n\tv_exp_f32 %[t1], %[t1]"                                   \
  "\n\tv_fma_mix_f32 %[lb], %[pn], 1.0, %[lb] op_sel:[1,0,0] op_sel_hi:[1,0,0]"                     \
  "\n\tv_cvt_pk_f16_f32 %[pn], %[t0], %[t1]"
#define G2_FULL                                                                                   \
  "\n\tv_sub_f32 %[t0], %[s0], %[mr]\n\tv_exp_f32 %[t0], %[t0]\n\tv_sub_f32 %[t1], %[s1], %[mr]\n\tv_exp_f32 %[t1], %[t1]" \
  "\n\tv_fma_mix_f32 %[la], %[pn], 1.0, %[la] op_sel_hi:[1,0,0]"                                     \
  "\n\tv_fma_mix_f32 %[lb], %[pn], 1.0, %[lb] op_sel:[1,0,0] op_sel_hi:[1,0,0]"                     \
  "\n\tv_cvt_pk_f16_f32 %[pn], %[t0], %[t1]"
// the tile's packed max over its two halves (tm) and the epoch max of P; then the rebase predicate
#define G2_TMAX                                                                                                  \
  "\n\tv_max_f16_sdwa %[tm], %[pm], %[pm] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" \
  "\n\tv_pk_max_f16 %[pr], %[pr], %[pm]"
#define G2_CMP "\n\tv_cmp_gt_f16_e64 %[sm], %[tm], %[th]\n\ts_nop 1"
#define G2_MAX3 "\n\tv_pk_maximum3_f16 %[pm], %[pm], %[pa], %[pb]"
#define G2_MAX2 "\n\tv_pk_max_f16 %[pm], %[pa], %[pb]"

// LAY 0: V(i)'s fragment reads one a gap over segment A's gaps 0-15, the DMA pieces in the four lightest gaps of
// each segment (28-31: folds, max, predicate), K's in segment A, V's in segment B; LAY 1 (FA_FWD_VARIANT 2701):
// the reads two a gap in gaps 0-7, the DMA pieces in segment A's gaps 8-15
template <int POL, int LAY = 0>
__global__ __launch_bounds__(kNW * 64, 1) void fwd_f16_gap128_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t ngr = (uint32_t)gap128_groups(nqb, POL);
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / ngr;
  const uint32_t jgr = bid % ngr;
  const int npass = (POL == 0 || nqb - 1 - jgr == jgr) ? 1 : 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g4 = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;

  // ---- LDS-DMA: piece j of wave w = channel rows 8(4w + j) .. +7 of a tile image, lane L the 16 B at
  //      16 L of it: row c = 8(4w + j) + L/8, position L%8, i.e. source chunk = position ^ swizzle(c)
  const int dpos = lane & 7;
  uint32_t kdoff[kPPW], vdoff[kPPW];
#pragma unroll
  for (int j = 0; j < kPPW; ++j) {
    const int c = 8 * (kPPW * w + j) + (lane >> 3);
    const int kcm = dpos ^ (4 * ((c >> 1) & 1));  // K image: 64-B halves swapped on rows with c&2
    const int vcm = dpos ^ ((c >> 1) & 7);        // V image: 16-B chunks XOR (c>>1)&7
    kdoff[j] = c < d ? (uint32_t)c * (uint32_t)nk * 2u + 16u * kcm : 0x80000000u;
    vdoff[j] = c < vd ? (uint32_t)c * (uint32_t)nk * 2u + 16u * vcm : 0x80000000u;
  }
  // one piece into LDS at lds_off + 1 KB·(4w + j); keys outside [0, nk) read as zeros.  Interior tiles
  // (wave-uniform) take the offset as it is; the others test each lane's chunk (its key chunk recomputed
  // from the lane: no register kept for it)
  auto dma = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, bool isk, int j, int k0, int lds_off) __attribute__((always_inline)) {
    const uint32_t m0v = (uint32_t)(uintptr_t)(smem + lds_off);
    // (a select, not a branch, for the tail test: with a scalar branch between the gap statements the kernel
    // lost its whole lead over the ping-pong at config 3's shape, full policy: 4.52 against 4.49 ms)
    uint32_t o = off;
    if (!(k0 >= 0 && k0 + kBN <= nk)) {
      const int c = 8 * (kPPW * w + j) + (lane >> 3);
      const int cmx = isk ? (dpos ^ (4 * ((c >> 1) & 1))) : (dpos ^ ((c >> 1) & 7));
      o = ((unsigned)(k0 + 8 * cmx) < (unsigned)nk) ? off : 0x80000000u;
    }
    // (s_nop 0: the wait state between the SALU write of M0 and an LDS-DMA that reads it)
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                 :
                 : "v"(o), "s"(rs), "s"(2 * min(max(k0, 0), nk)), "{m0}"(m0v)
                 : "memory");
  };
  auto dma_k = [&](int j, int k0, int slot) __attribute__((always_inline)) {
    dma(krs, kdoff[j], true, j, k0, kOffK + slot * kTile + 1024 * (kPPW * w + j));
  };
  auto dma_v = [&](int j, int k0, int slot) __attribute__((always_inline)) {
    dma(vrs, vdoff[j], false, j, k0, kOffV + slot * kTile + 1024 * (kPPW * w + j));
  };

  // ---- fragment read bases (lane constants; every read is base + immediate)
  //   K: lane 4q+p of a 16-lane group supplies channel row q, keys 4σ(p)..4σ(p)+3, σ swapping 1 and 2
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g4 >> 1) + tq) * 128 + (((32 * t + 16 * (g4 & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r, h) reads chunk 2s+h of channel row 32u + r (the ring's offset folded in)
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    vbase[s] = kOffV + r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));
    asm volatile("" : "+v"(vbase[s]));  // (the 64 KB offset stays in the VGPR: the immediates stay small)
  }

  half8 kf[8][2];  // K fragments of one tile: k-step s, Sᵀ half t (VGPR)
  half8 vf[4][4];  // V fragments of one tile: k-step s, O quarter u (AGPR: asm reads, waited explicitly)
  auto read_kf = [&](int slot, auto S_, auto T_) __attribute__((always_inline)) {
    constexpr int s = decltype(S_)::value, t = decltype(T_)::value;
    const lds_char_t* p = smem + kOffK + slot * kTile + kbase[t];
    kf[s][t].lo = tr_read(p + (16 * s) * 128);
    kf[s][t].hi = tr_read(p + (16 * s + 4) * 128);
  };
  auto read_vf = [&vf, &vbase](auto SLOT_, auto N_) __attribute__((always_inline)) {
    constexpr int n = decltype(N_)::value, s = n >> 2, u = n & 3;
    constexpr int off = decltype(SLOT_)::value * kTile + 32 * u * 128;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=a"(vf[s][u]) : "v"(vbase[s]), "i"(off) : "memory");
  };

  Blk A, B;

  // one query block; REV: its key tiles walked downwards (the light block of a pair)
  auto run_block = [&](auto REV_, const int q0) __attribute__((always_inline)) {
    constexpr bool rev = decltype(REV_)::value;
    // ---- key range of the block (rule-bounded)
    const int qlast = min(q0 + kBM, nq) - 1;
    int kb = 0, ke = nk;
    if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
    const int kt0 = (kb / kBN) * kBN;
    const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;
    const int kfirst = rev ? kt0 + (ntiles - 1) * kBN : kt0;
    auto tk0 = [&](int it) -> int __attribute__((always_inline)) { return rev ? kfirst - it * kBN : kfirst + it * kBN; };

    // ---- prologue: V(0), V(1) by DMA; Q through registers into the image over the K ring; the scaled
    //      Q fragments into AGPRs; then K(0..3) by DMA over the dead image
    if (rev) {
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): the first block's DMAs have landed
      __syncthreads();                     // and every wave is past its last LDS read
    }
#pragma unroll
    for (int j = 0; j < kPPW; ++j) {
      dma_v(j, tk0(0), 0);
      dma_v(j, tk0(1), 1);
    }
    {
      int tidb = tid;
      asm volatile("" : "+v"(tidb));
      constexpr int kQPT = kD * (kBM / 8) / (kNW * 64);  // 16 chunks a thread, in two rounds
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
        u32x4 qv[kQPT / 2];
#pragma unroll
        for (int jj = 0; jj < kQPT / 2; ++jj) {
          const int idx = tidb + (rd * kQPT / 2 + jj) * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
          qv[jj] = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int jj = 0; jj < kQPT / 2; ++jj) {
          const int idx = tidb + (rd * kQPT / 2 + jj) * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
          *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[jj];
        }
      }
    }
    __syncthreads();
    auto init_blk = [&](Blk& X, int blk) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int cr = 16 * s + 8 * (g4 >> 1) + 4 * e + tq;
          const int col = 64 * w + 32 * blk + 16 * (g4 & 1) + 4 * tp;
          const half4 t = tr_read(smem + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
          if (e == 0) X.q[s].lo = t; else X.q[s].hi = t;
        }
        X.q[s] = scale8(X.q[s], c2);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) X.o[u][i] = 0.f;
        X.p[i] = 0u;
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) X.l[x] = 0.f;
      X.pm = 0u;
      X.pmr = half2v{(_Float16)0.f, (_Float16)0.f};
      X.m_run = 0.f;
      X.m_max = kNegInf;
      X.thr = -__FLT_MAX__;
      X.thr_h = (_Float16)-1.f;
      X.thr_bits = (uint32_t)__builtin_bit_cast(unsigned short, X.thr_h);
      X.pmr_old = X.pmr;
      X.tm = 0u;
      X.sm = 0;
      // the block's rule bounds
      const int wq0 = q0 + 64 * w + 32 * blk;
      X.active = wq0 < nq;
      X.klo = 0; X.kspan = 0; X.wlo_min = X.wlo_max = X.whi_min = X.whi_max = 0;
      if (POL != 0 && X.active) {
        int khi;
        key_interval(a.rule, min(wq0 + r, nq - 1), &X.klo, &khi);
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
    // Q and O live in AGPRs (the MFMAs take them from there): home them once
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" : "+a"(A.q[s]), "+a"(B.q[s]));
    asm volatile("" : "+a"(A.o[0]), "+a"(A.o[1]), "+a"(A.o[2]), "+a"(A.o[3]));
    asm volatile("" : "+a"(B.o[0]), "+a"(B.o[1]), "+a"(B.o[2]), "+a"(B.o[3]));
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the image has been read
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPPW; ++j) {
      dma_k(j, tk0(0), 0);
      dma_k(j, tk0(1), 1);
      dma_k(j, tk0(2), 2);
      dma_k(j, tk0(3), 3);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();

    // tile class of block X at position it: 0 no allowed pair, 1 mixed (masked), 2 all allowed
    auto tcls = [&](const Blk& X, int it) -> int __attribute__((always_inline)) {
      if (it < 0 || it >= ntiles) return 0;
      const int k0 = tk0(it), k1 = k0 + kBN - 1;
      if (POL == 0) return (k1 < nk) ? 2 : 1;
      if (!X.active || X.wlo_min > k1 || X.whi_max < k0) return 0;
      return (X.wlo_max <= k0 && X.whi_min >= k1 && k1 < nk) ? 2 : 1;
    };
    // the scores of block X's tile at position it masked to -inf where not allowed (cls 1) / everywhere (0)
    auto mask = [&](Blk& X, int it, int cls) __attribute__((always_inline)) {
      if (cls == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          X.s[0][i] = kNegInf;
          X.s[1][i] = kNegInf;
        }
        return;
      }
      // mixed tiles, arithmetically (as fa_fwd_f16_band.hip): key k0 + 8h + off is allowed iff
      // 0 <= v < kspan, v = k0 + 8h - klo + off (POL 0: klo = 0, kspan = nk, the tail only), so
      // min(s, (v + 0.5)·2^100) (an edge below) and min(s, (kspan - v - 0.5)·2^100) (an edge above) keep an
      // allowed score and take a disallowed one to <= -2^99: one fma and one min per score and edge, no
      // compare (the select form cost a compare, a wait state and a cndmask per score)
      const int k0 = tk0(it), k1 = k0 + kBN - 1;
      const int klo = POL != 0 ? X.klo : 0, kspan = POL != 0 ? X.kspan : nk;
      const bool lo = POL != 0 && X.wlo_max > k0;
      const bool hi = POL != 0 ? (X.whi_min < k1 || k1 >= nk) : true;
      constexpr float kBig = 0x1p100f;
      const float fb = (float)(k0 + 8 * h - klo);
      if (lo) {
        const float cc = __builtin_fmaf(fb, kBig, 0.5f * kBig);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            X.s[t][i] = fminf(X.s[t][i], __builtin_fmaf(kBig, (float)(32 * t + 16 * (i >> 3) + (i & 7)), cc));
      }
      if (hi) {
        const float cc = __builtin_fmaf((float)kspan - fb, kBig, -0.5f * kBig);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            X.s[t][i] = fminf(X.s[t][i], __builtin_fmaf(-kBig, (float)(32 * t + 16 * (i >> 3) + (i & 7)), cc));
      }
    };
    auto exp_cvt = [&](Blk& X) __attribute__((always_inline)) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float s0 = X.s[g >> 3][(2 * g) & 15], s1 = X.s[g >> 3][((2 * g) & 15) + 1];
        X.p[g] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0 - X.m_run),
                                                     (_Float16)__builtin_amdgcn_exp2f(s1 - X.m_run)});
      }
    };
    // the rebase of block X (rare: the tile's packed-P max passed 2^thr, or the seed): see fa_fwd_f16_gap.hip
    auto rebase = [&](Blk& X, half2v pmr_old) __attribute__((always_inline)) {
      float mx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) mx[j] = fmaxf(X.s[j >> 1][8 * (j & 1)], X.s[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
      for (int i = 2; i < 8; i += 2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mx[j] = fmaxf(fmaxf(mx[j], X.s[j >> 1][8 * (j & 1) + i]), X.s[j >> 1][8 * (j & 1) + i + 1]);
      // (the scores are relative to 0: the tile's max relative to the running reference)
      const float mtf = max_pair32(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]))) - X.m_run;
      const float pold = (float)__builtin_elementwise_maximum(pmr_old[0], pmr_old[1]);
      X.m_max = fmaxf(X.m_max, fmaxf(X.m_run + mtf, X.m_run + __log2f(pold)));
      const bool unset = X.thr < 0.f;
      // (a masked score sits at or below -2^99: a row max below -2^98 means nothing allowed yet)
      const bool seed = unset && (mtf > -0x1p98f);
      const float delta = unset ? (seed ? mtf : 0.f) : fmaxf(mtf, 0.f);
      const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
      X.m_run += delta;
      X.thr = (unset && !seed) ? X.thr : kRescaleThr;
      X.thr_h = (unset && !seed) ? (_Float16)-1.f : (_Float16)(1 << (int)kRescaleThr);
      X.thr_bits = (uint32_t)__builtin_bit_cast(unsigned short, X.thr_h);
#pragma unroll
      for (int x = 0; x < 4; ++x) X.l[x] *= alpha;
      // O only ever appears in AGPR operands: copy out, scale, copy back, inside the branch
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        floatx16 t;
        asm volatile("; O out" : "=v"(t) : "0"(X.o[u]));
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] *= alpha;
        asm volatile("; O in" : "=a"(X.o[u]) : "0"(t));
      }
      exp_cvt(X);
      X.pmr = half2v{(_Float16)0.f, (_Float16)0.f};
      asm volatile("s_nop 4" ::: "memory");  // (VALU writes of P, then the next segment's MFMAs)
    };
    // the rebase check of block X outside the stream (the prologue's seed tile)
    auto check_now = [&](Blk& X) __attribute__((always_inline)) {
      const half2v tm = __builtin_bit_cast(half2v, X.pm);
      const _Float16 tmx = __builtin_elementwise_maximum(tm[0], tm[1]);
      const half2v pmr_old = X.pmr;
      X.pmr = __builtin_elementwise_maximum(X.pmr, tm);
      if (__any(tmx > X.thr_h)) rebase(X, pmr_old);
    };
    // the rebase check after a segment: its predicate was formed in the segment's last gaps (sm)
    auto check = [&](Blk& X) __attribute__((always_inline)) {
      if (X.sm != 0) rebase(X, X.pmr_old);
    };

    // one gap: MFMA g of block X and its share of block Y's softmax.  Fillers by gap:
    //   g < 24, even: the first exponential of Y's P dword g/2 (v_sub of the running reference, v_exp_f32)
    //                 and the first row-sum step of the dword's previous value; a packed-max fold at g % 4 == 0
    //   g < 24, odd : the second exponential, the second row-sum step, the conversion over the dword
    //   24 <= g < 28: a whole dword (12 + g - 24): both exponentials, both row-sum steps, the conversion
    //   28, 29      : the folds of dwords 12-13 and 14-15
    //   30          : the tile's max over the two halves, the epoch max of P
    //   31          : the rebase predicate (an SGPR pair): the check after the segment is one scalar branch
    float ft0 = 0.f;  // the even gap's exponential, converted in the odd gap
    int cur_it = 0;   // (the step, for segment A's DMA pieces)
    auto gap = [&](Blk& X, Blk& Y, auto G_) __attribute__((always_inline)) {
      constexpr int g = decltype(G_)::value;
      constexpr bool full = g >= 24 && g < 28;
      constexpr int j = full ? 12 + (g - 24) : (g < 24 ? g >> 1 : 15);  // Y's P dword
      constexpr int mk = (g % 4 == 0 && g >= 4 && g <= 24) ? (g / 4 - 1) : (g == 28 ? 6 : (g == 29 ? 7 : -1));
      constexpr bool fold_only = g == 28 || g == 29;
      const uint32_t pa = mk >= 0 ? Y.p[2 * mk] : 0u, pb = mk >= 0 ? Y.p[2 * mk + 1] : 0u;
      const float s0 = Y.s[j >> 3][(2 * j) & 15], s1 = Y.s[j >> 3][((2 * j) & 15) + 1];
      float& la = Y.l[j & 1];
      float& lb = Y.l[2 + (j & 1)];
      float t1;
      if constexpr (g < 16) {
        constexpr int s = g >> 1, t = g & 1;
#define G2_ST_OUT(D) [d] D(X.s[t])
#define G2_ST_IN [a] "v"(kf[s][t]), [b] "a"(X.q[s])
        if constexpr ((g & 1) == 0) {
          if constexpr (s == 0) {
            asm volatile(G2_MFMA_C G2_EVEN : G2_ST_OUT("=&v"), [t0] "=&v"(ft0), [la] "+v"(la)
                         : G2_ST_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]));
          } else if constexpr (mk == 0) {
            asm volatile(G2_MFMA G2_EVEN G2_MAX2 : G2_ST_OUT("+v"), [t0] "=&v"(ft0), [la] "+v"(la), [pm] "=&v"(Y.pm)
                         : G2_ST_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]), [pa] "v"(pa), [pb] "v"(pb));
          } else if constexpr (mk > 0) {
            asm volatile(G2_MFMA G2_EVEN G2_MAX3 : G2_ST_OUT("+v"), [t0] "=&v"(ft0), [la] "+v"(la), [pm] "+v"(Y.pm)
                         : G2_ST_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]), [pa] "v"(pa), [pb] "v"(pb));
          } else {
            asm volatile(G2_MFMA G2_EVEN : G2_ST_OUT("+v"), [t0] "=&v"(ft0), [la] "+v"(la)
                         : G2_ST_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]));
          }
        } else if constexpr (s == 0) {  // (the second key half's chain starts here too)
          asm volatile(G2_MFMA_C G2_ODD : G2_ST_OUT("=&v"), [t1] "=&v"(t1), [lb] "+v"(lb), [pn] "+v"(Y.p[j])
                       : G2_ST_IN, [s1] "v"(s1), [mr] "v"(Y.m_run), [t0] "v"(ft0));
        } else {
          asm volatile(G2_MFMA G2_ODD : G2_ST_OUT("+v"), [t1] "=&v"(t1), [lb] "+v"(lb), [pn] "+v"(Y.p[j])
                       : G2_ST_IN, [s1] "v"(s1), [mr] "v"(Y.m_run), [t0] "v"(ft0));
        }
#undef G2_ST_OUT
#undef G2_ST_IN
      } else {
        // (quarters 0-1 over gaps 16-23, 2-3 over 24-31: their V fragments are read in two waves)
        constexpr int s = ((g - 16) & 7) >> 1, u = 2 * ((g - 16) >> 3) + (g & 1);
        const u32x4 pp = {X.p[4 * s], X.p[4 * s + 1], X.p[4 * s + 2], X.p[4 * s + 3]};
#define G2_PV_OUT [d] "+a"(X.o[u])
#define G2_PV_IN [a] "a"(vf[s][u]), [b] "v"(pp)
        if constexpr (full && mk >= 0) {
          asm volatile(G2_MFMA G2_FULL G2_MAX3
                       : G2_PV_OUT, [t0] "=&v"(ft0), [t1] "=&v"(t1), [la] "+v"(la), [lb] "+v"(lb), [pn] "+v"(Y.p[j]), [pm] "+v"(Y.pm)
                       : G2_PV_IN, [s0] "v"(s0), [s1] "v"(s1), [mr] "v"(Y.m_run), [pa] "v"(pa), [pb] "v"(pb));
        } else if constexpr (full) {
          asm volatile(G2_MFMA G2_FULL
                       : G2_PV_OUT, [t0] "=&v"(ft0), [t1] "=&v"(t1), [la] "+v"(la), [lb] "+v"(lb), [pn] "+v"(Y.p[j])
                       : G2_PV_IN, [s0] "v"(s0), [s1] "v"(s1), [mr] "v"(Y.m_run));
        } else if constexpr (fold_only) {
          asm volatile(G2_MFMA G2_MAX3 : G2_PV_OUT, [pm] "+v"(Y.pm) : G2_PV_IN, [pa] "v"(pa), [pb] "v"(pb));
        } else if constexpr (g == 30) {
          asm volatile(G2_MFMA G2_TMAX : G2_PV_OUT, [tm] "=&v"(Y.tm), [pr] "+v"(Y.pmr) : G2_PV_IN, [pm] "v"(Y.pm));
        } else if constexpr (g == 31) {
          asm volatile(G2_MFMA G2_CMP : G2_PV_OUT, [sm] "=s"(Y.sm) : G2_PV_IN, [tm] "v"(Y.tm), [th] "v"(Y.thr_bits));
        } else if constexpr ((g & 1) == 0 && mk > 0) {
          asm volatile(G2_MFMA G2_EVEN G2_MAX3 : G2_PV_OUT, [t0] "=&v"(ft0), [la] "+v"(la), [pm] "+v"(Y.pm)
                       : G2_PV_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]), [pa] "v"(pa), [pb] "v"(pb));
        } else if constexpr ((g & 1) == 0) {
          asm volatile(G2_MFMA G2_EVEN : G2_PV_OUT, [t0] "=&v"(ft0), [la] "+v"(la)
                       : G2_PV_IN, [s0] "v"(s0), [mr] "v"(Y.m_run), [pn] "v"(Y.p[j]));
        } else {
          asm volatile(G2_MFMA G2_ODD : G2_PV_OUT, [t1] "=&v"(t1), [lb] "+v"(lb), [pn] "+v"(Y.p[j])
                       : G2_PV_IN, [s1] "v"(s1), [mr] "v"(Y.m_run), [t0] "v"(ft0));
        }
#undef G2_PV_OUT
#undef G2_PV_IN
      }
      (void)t1;
      // the sources of the MFMA two gaps back stay live until here: the allocator cannot see that an
      // asm statement holds an MFMA still reading them
      if constexpr (g >= 2) {
        constexpr int hh = g - 2;
        if constexpr (hh < 16) {
          asm volatile("" ::"v"(kf[hh >> 1][hh & 1]), "a"(X.q[hh >> 1]));
        } else {
          constexpr int s2 = ((hh - 16) & 7) >> 1, u2 = 2 * ((hh - 16) >> 3) + (hh & 1);
          const u32x4 pp2 = {X.p[4 * s2], X.p[4 * s2 + 1], X.p[4 * s2 + 2], X.p[4 * s2 + 3]};
          asm volatile("" ::"a"(vf[s2][u2]), "v"(pp2));
        }
      }
    };
    // after a segment: its last two MFMAs' sources stay live a little longer
    auto seg_end = [&](Blk& X) __attribute__((always_inline)) {
      const u32x4 pp3 = {X.p[12], X.p[13], X.p[14], X.p[15]};
      asm volatile("" ::"a"(vf[3][2]), "a"(vf[3][3]), "v"(pp3));
    };

    // segment A of step it (slot c = it mod 4): MFMAs of A, softmax of B(it); V(it)'s fragments one a gap
    // over gaps 0-15, quarters 0-1 first (their PV MFMAs run in gaps 16-23, quarters 2-3 in 24-31); the DMA
    // pieces of K(it+4) in gaps 28-31 (LAY 0)
    auto seg_a = [&](auto C_) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      auto body = [&](auto G_) __attribute__((always_inline)) {
        constexpr int g = decltype(G_)::value;
        if constexpr (LAY == 0) {
          if constexpr (g == 16) __builtin_amdgcn_s_waitcnt(0xC87F);  // lgkmcnt(8): quarters 0-1 of V(it)
          if constexpr (g == 24) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): quarters 2-3
          gap(A, B, G_);
          if constexpr (g < 16) read_vf(IC<c>{}, IC<(4 * ((g & 7) >> 1) + 2 * (g >> 3) + (g & 1))>{});
          if constexpr (g >= 28) dma_k(g - 28, tk0(cur_it + 4), c);
        } else {
          if constexpr (g == 16) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): V(it)
          gap(A, B, G_);
          if constexpr (g < 8) {
            read_vf(IC<c>{}, IC<2 * g>{});
            read_vf(IC<c>{}, IC<2 * g + 1>{});
          }
          if constexpr (g >= 8 && g < 12) dma_k(g - 8, tk0(cur_it + 4), c);
          if constexpr (g >= 12 && g < 16) dma_v(g - 12, tk0(cur_it + 2), (c + 2) % kNS);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      B.pmr_old = B.pmr;
      static_for<0, 32>(body);
      seg_end(A);
    };
    // segment B of step it: MFMAs of B, softmax of A(it+1); K(it+2)'s fragments in gaps 2-17, the DMA
    // pieces of V(it+2) in gaps 28-31 (LAY 0)
    auto seg_b = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;
      const int kk = tk0(it + 4), kv = tk0(it + 2);
      (void)kk; (void)kv;
      auto body = [&](auto G_) __attribute__((always_inline)) {
        constexpr int g = decltype(G_)::value;
        gap(B, A, G_);
        if constexpr (g >= 2 && g < 18) read_kf((c + 2) % kNS, IC<((g - 2) >> 1)>{}, IC<((g - 2) & 1)>{});
        if constexpr (LAY == 0 && g >= 28) dma_v(g - 28, kv, (c + 2) % kNS);
        __builtin_amdgcn_sched_barrier(0);
      };
      A.pmr_old = A.pmr;
      static_for<0, 32>(body);
      seg_end(B);
      // K(it+2)'s reads (issued 14+ gaps ago) have landed: said to the compiler, so it puts no waits for
      // them before the next segment A's MFMAs, where they would also wait for that segment's V reads
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    };

    // ---- prologue compute: Sᵀ(0) of both blocks from K(0), the softmax of A(0) (the seed), K(1)'s
    //      fragments; P_B(-1) = 0
    static_for<0, 8>([&](auto S_) __attribute__((always_inline)) {
      read_kf(0, S_, IC<0>{});
      read_kf(0, S_, IC<1>{});
    });
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (s == 0) {
          asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(A.s[t]) : "v"(kf[s][t]), "a"(A.q[s]));
          asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(B.s[t]) : "v"(kf[s][t]), "a"(B.q[s]));
        } else {
          asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(A.s[t]) : "v"(kf[s][t]), "a"(A.q[s]));
          asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(B.s[t]) : "v"(kf[s][t]), "a"(B.q[s]));
        }
      }
    // (the scores are read below and kf is overwritten: let the last MFMAs finish)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    static_for<0, 8>([&](auto S_) __attribute__((always_inline)) {
      read_kf(1, S_, IC<0>{});
      read_kf(1, S_, IC<1>{});
    });
    {
      const int cls = tcls(A, 0);
      if (cls != 2) mask(A, 0, cls);
    }
    exp_cvt(A);
    A.pm = 0u;
#pragma unroll
    for (int g = 0; g < 16; ++g)
      A.pm = __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(half2v, A.pm),
                                                                         __builtin_bit_cast(half2v, A.p[g])));
    check_now(A);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): K(1)'s fragments, before the first barrier

    // ---- steps: every step has the same straight-line shape; the last one issues the phantom Sᵀ(ntiles)
    //      (masked, never multiplied into O)
    auto step = [&](auto C_, int it) __attribute__((always_inline)) {
      cur_it = it;
      // K(it+2) and V(it) (DMA'd two steps back) have landed: only the previous step's eight may fly
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      {
        const int cls = tcls(B, it);
        if (cls != 2) mask(B, it, cls);
      }
      seg_a(C_);
      check(B);
      {
        const int cls = tcls(A, it + 1);
        if (cls != 2) mask(A, it + 1, cls);
      }
      seg_b(C_, it);
      check(A);
    };
    for (int it = 0; it < ntiles; it += kNS) {
      step(IC<0>{}, it);
      if (it + 1 < ntiles) step(IC<1>{}, it + 1);
      if (it + 2 < ntiles) step(IC<2>{}, it + 2);
      if (it + 3 < ntiles) step(IC<3>{}, it + 3);
    }

    // ---- epilogue: the row sums of P_B(ntiles-1) are still pending (P_A(ntiles) is the phantom)
    {
      const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
      for (int g = 0; g < 16; ++g)
        B.l[g & 3] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, B.p[g]), one2, B.l[g & 3], false);
    }
    __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
    float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
    __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
    auto finish = [&](Blk& X, int blk) __attribute__((always_inline)) {
      const int wq0 = q0 + 64 * w + 32 * blk;
      const int qi = wq0 + r;
      const float l0 = (X.l[0] + X.l[1]) + (X.l[2] + X.l[3]);
      const float m_max = max_pair32(fmaxf(X.m_max, X.m_run + __log2f((float)__builtin_elementwise_maximum(X.pmr[0], X.pmr[1]))));
      const float l_tot = sum_pair32(l0);
      const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
      if (wq0 >= nq || qi >= nq) return;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (v < vd) O[(int64_t)v * nq + qi] = __float2half(X.o[u][i] * inv);
        }
      if (h == 0) {
        if (l_tot > 0.f) {
          const __half mT = __float2half(m_max * kLn2);
          // l relative to the STORED (rounded) m, so exp(s - m)/l is exact downstream
          lo[qi] = l_tot * __builtin_amdgcn_exp2f(X.m_run - __half2float(mT) * kLog2e);
          mo[qi] = mT;
        } else {
          lo[qi] = 0.f;
          mo[qi] = neg_inf_approx<__half>();
        }
      }
    };
    finish(A, 0);
    finish(B, 1);
  };
  run_block(IC<false>{}, (int)(POL == 0 ? jgr : nqb - 1 - jgr) * kBM);
  if (npass == 2) {
    int q0 = (int)jgr * kBM;
    asm volatile("" : "+s"(q0));
    run_block(IC<true>{}, q0);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no DMA in flight when the workgroup ends
}

}  // namespace

bool fwd_f16_gap128_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return dm > 64 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) && (a.rule.policy == 0 || rule_is_interval(a.rule)) &&
         a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16_gap128(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const int pol = a.rule.policy == 0 ? 0 : 1;
  auto kern = pol == 0 ? fwd_f16_gap128_kernel<0> : fwd_f16_gap128_kernel<1>;
#ifdef FA_DIAG
  if (diag_variant("FA_FWD_VARIANT") == 2701) kern = pol == 0 ? fwd_f16_gap128_kernel<0, 1> : fwd_f16_gap128_kernel<1, 1>;
#endif
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * gap128_groups(nqb, pol))), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
