// fa_fwd_f16_gap.hip — fp16 fused attention forward for 32 < max(d, v_d) <= 64 under the full policy
// (BASELINE config 2, the headline) with ONE wave per SIMD and a hand-placed gap stream.
//
// Each wave owns 64 queries as two 32-query blocks A and B and the whole 512-register file (scores,
// P, -m and the K fragments in VGPRs; O, Q, the V fragments and the staging buffers in AGPRs).  A key tile (64 keys) of a step is two
// segments of 16 v_mfma_f32_32x32x16_f16 each; every segment carries the OTHER block's softmax in
// its MFMA gaps:
//
//   segment A of step i : Sᵀ A(i+1) (8 MFMAs), PV A(i) (8)  |  softmax B(i), row sums of P_B(i-1)
//   segment B of step i : Sᵀ B(i+1) (8 MFMAs), PV B(i) (8)  |  softmax A(i+1), row sums of P_A(i)
//
// A gap is ONE asm statement: the MFMA, then the fillers of one P dword of the other block — two
// v_exp_f32, the two v_fma_mix_f32 row-sum steps of the dword's previous value, a packed-max fold every
// other gap, and the v_cvt_pk_f16_f32 that overwrites the dword.  One statement per gap keeps the
// order exactly as written (the compiler's hazard checker cannot see into it, so it adds no s_nop
// between an exponential and its conversion; inside, two instructions separate them).  Row sums use
// v_fma_mix_f32, not v_dot2c: beside MFMAs of the same wave a v_dot2c costs ~20 cycles
// (tools/gap_probe.hip: 1090 cycles a segment with dot2c, 837 with fma_mix, 770 without row sums,
// 540 for the MFMAs alone; profiles/r06_gap_probe.txt).
//
// Memory operations are builtins between the gap statements (the compiler counts their waits),
// fenced into their gap by sched_barrier: the K(i+2) fragment reads fill segment B's gaps 2-9 (each
// into the registers a Sᵀ MFMA of the segment finished with two gaps earlier), V(i+1) fragments gaps
// 10-15 and the next segment A's gaps 0-1; the LDS stores of K(i+3) / V(i+2) sit in segment A, the
// global loads of K(i+6) / V(i+5) in segment B (AGPR buffers, three steps ahead).  One barrier per step.
// The rebase check (packed-P max against 2^8) closes each segment in a rare, wave-uniform branch.
//
// Numerics are those of fa_fwd_f16_pingpong.hip: fp32 accumulation, log2-domain lazy rebase at 8,
// speculative exponentials against the running reference, m from the packed P of the epoch, l
// relative to the stored fp16 m.  Replaces the reference's ForwardImpl (flash_attention.cu:425-1077)
// for these shapes.
#include "../fa_device.h"
#include "../fa_kernels.h"
#include "../fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 64;
constexpr int kBN = 64;                 // keys per tile
constexpr int kNW = 4;                  // waves per workgroup, one per SIMD
constexpr int kBM = 64 * kNW;           // queries per workgroup
constexpr int kNS = 3;                  // ring slots for K and for V
constexpr int kQRow = 2 * kBM;          // bytes per Q row in LDS (prologue)
constexpr int kTile = kD * kBN * 2;     // 8 KB
constexpr int kOffK = kD * kQRow;       // Q image [64][256] first
constexpr int kOffV = kOffK + kNS * kTile;
constexpr int kSmem = kOffV + kNS * kTile;
constexpr int kCPT = kD * 8 / (kNW * 64);  // 16-B chunks per thread per tile (2)
constexpr float kRescaleThr = 8.f;

struct Blk {
  floatx16 s[2];   // Sᵀ (VGPR): register i of half t = key 32t + 16(i>>3) + 8h + (i&7)
  floatx16 nm;     // -m_run broadcast (VGPR): the C operand of the first Sᵀ k-step
  floatx16 o[2];   // Oᵀ (AGPR): channels 32u + 8(i>>2) + 4h + (i&3)
  half8 q[4];      // Q * scale * log2(e), k-step s = channels 16s..16s+15 (AGPR)
  uint32_t p[16];  // P (fp16 pairs): dword x of PV k-step s at 4s + x
  float l[4];      // running row sums (four chains)
  uint32_t pm;     // packed max of the tile's P (the rebase check)
  half2v pmr;      // running packed max of P over the current epoch
  float m_run, m_max, thr;
  _Float16 thr_h;  // 2^thr once seeded; -1 (always exceeded) before
};

#define FG_EXP "\n\tv_exp_f32 %[t0], %[s0]\n\tv_exp_f32 %[t1], %[s1]"
#define FG_SUM                                                     \
  "\n\tv_fma_mix_f32 %[la], %[pn], 1.0, %[la] op_sel_hi:[1,0,0]" \
  "\n\tv_fma_mix_f32 %[lb], %[pn], 1.0, %[lb] op_sel:[1,0,0] op_sel_hi:[1,0,0]"
#define FG_MAX3 "\n\tv_pk_maximum3_f16 %[pm], %[pm], %[pa], %[pb]"
#define FG_MAX2 "\n\tv_pk_max_f16 %[pm], %[pa], %[pb]"
#define FG_CVT "\n\tv_cvt_pk_f16_f32 %[pn], %[t0], %[t1]"
#define FG_MFMA_C "v_mfma_f32_32x32x16_f16 %[d], %[a], %[b], %[c]"
#define FG_MFMA "v_mfma_f32_32x32x16_f16 %[d], %[a], %[b], %[d]"
// (the row sums read the dword's previous value, then the conversion overwrites it: one register)
#define FG_OUT [t0] "=&v"(t0), [t1] "=&v"(t1), [la] "+v"(Y.l[g & 1]), [lb] "+v"(Y.l[2 + (g & 1)]), [pn] "+v"(Y.p[g])
#define FG_IN [s0] "v"(Y.s[g >> 3][(2 * g) & 15]), [s1] "v"(Y.s[g >> 3][((2 * g) & 15) + 1])

// timing ablations (diagnostic library only, FA_FWD_VARIANT=2600+bits; outputs WRONG): 1 no barrier,
// 2 no staging loads / stores, 4 no fragment reads, 8 MFMAs without the softmax fillers (and no checks)
constexpr int kANoBar = 1, kANoStage = 2, kANoFrag = 4, kANoFill = 8;

template <int POL, int ABL = 0>
__global__ __launch_bounds__(kNW * 64, 1) void fwd_f16_gap_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(nqb - 1 - (bid % nqb)) * kBM;
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
  const int ntiles = (nk + kBN - 1) / kBN;

  // ---- staging: chunk j of this thread = 8 keys (16 B) of channel row (tid + 256 j) >> 3
  const int cm = tid & 7;
  uint32_t koff[kCPT], voff[kCPT], kwo[kCPT], vwo[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int c = (tid + kNW * 64 * j) >> 3;
    const uint32_t go = (uint32_t)c * (uint32_t)nk * 2u + 16u * cm;
    koff[j] = c < d ? go : 0x80000000u;  // rows past d / v_d read as zeros
    voff[j] = c < vd ? go : 0x80000000u;
    kwo[j] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));
    vwo[j] = c * 128 + 16 * (cm ^ ((c >> 1) & 7));
  }
  // branch-free chunk load: chunks past nk (the tail, tiles past the end) read as zeros
  auto load = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, int k0) -> u32x4 __attribute__((always_inline)) {
    const bool in = k0 + 8 * cm < nk;
    return __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off : 0x80000000u, 2 * min(k0, nk), 0);
  };
  auto store = [&](int off, u32x4 v) __attribute__((always_inline)) { *reinterpret_cast<lds_u32x4_t*>(smem + off) = v; };
  // staging loads of the key loop: asm, straight into AGPRs (three buffers, by ring slot: a buffer is
  // loaded in segment B of step i and stored in segment A of step i + 3).  The compiler does not count
  // them: segment A waits vmcnt(8) before its stores (the two younger buffers' eight loads may fly on)
  auto load_a = [&](u32x4& dst, __amdgpu_buffer_rsrc_t rs, uint32_t off, int k0) __attribute__((always_inline)) {
    const bool in = k0 + 8 * cm < nk;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                 : "=a"(dst)
                 : "v"(in ? off : 0x80000000u), "s"(rs), "s"(2 * min(k0, nk))
                 : "memory");
  };

  // ---- prologue: Q, K(0..2), V(0..1) into LDS; K(3..5), V(2..4) into the staging buffers
  u32x4 kr[kNS][kCPT], vr[kNS][kCPT];
  {
    constexpr int kQPT = kD * (kBM / 8) / (kNW * 64);
    u32x4 qv[kQPT];
    if (qvec) {
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
    u32x4 kp[3][kCPT], vp[2][kCPT];
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) kp[x][j] = load(krs, koff[j], x * kBN);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) vp[x][j] = load(vrs, voff[j], x * kBN);
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
      const int idx = tid + j * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
      store(c * kQRow + ((m * 16) ^ ((c & 3) << 6)), qv[j]);
    }
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) store(kOffK + x * kTile + kwo[j], kp[x][j]);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) store(kOffV + x * kTile + vwo[j], vp[x][j]);
    // (after the compiler's own loads have been waited for: its waits would also drain these)
#pragma unroll
    for (int x = 0; x < kNS; ++x)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) {
        load_a(kr[x][j], krs, koff[j], (3 + x) * kBN);
        load_a(vr[x][j], vrs, voff[j], (2 + x) * kBN);
      }
  }
  __syncthreads();

  Blk A, B;
  auto init_blk = [&](Blk& X, int blk) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
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
      X.o[0][i] = 0.f;
      X.o[1][i] = 0.f;
      X.nm[i] = 0.f;
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
  };
  init_blk(A, 0);
  init_blk(B, 1);
  // Q and O live in AGPRs (the MFMAs take them from there): home them once
#pragma unroll
  for (int s = 0; s < 4; ++s) asm volatile("" : "+a"(A.q[s]), "+a"(B.q[s]));
  asm volatile("" : "+a"(A.o[0]), "+a"(A.o[1]), "+a"(B.o[0]), "+a"(B.o[1]));

  // fragment read bases (lane constants; every read is base + immediate)
  //   K: lane 4q+p of a 16-lane group supplies channel row q, keys 4σ(p)..4σ(p)+3, σ swapping 1 and 2
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g4 >> 1) + tq) * 128 + (((32 * t + 16 * (g4 & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r, h) reads chunk 2s+h of channel row 32u + r (the ring's offset folded in: the reads'
  //   immediates stay below 64 KB)
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = kOffV + r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  half8 kf[4][2];  // K fragments: k-step s, Sᵀ half t
  half8 vf[4][2];  // V fragments: k-step s, O half u (AGPR: read by asm, waited for explicitly)
  auto read_kf = [&](auto SLOT_, auto S_, auto T_) __attribute__((always_inline)) {
    constexpr int sl = decltype(SLOT_)::value, s = decltype(S_)::value, t = decltype(T_)::value;
    const lds_char_t* p = smem + kOffK + sl * kTile + kbase[t];
    kf[s][t].lo = tr_read(p + (16 * s) * 128);
    kf[s][t].hi = tr_read(p + (16 * s + 4) * 128);
  };
  // (an asm read the compiler does not count: its own lgkmcnt waits only grow more conservative; the
  // V fragments are waited for by the lgkmcnt(0) before segment A's first PV MFMA and at its end)
  auto read_vf = [&vf, &vbase](auto SLOT_, auto S_, auto U_) __attribute__((always_inline)) {
    constexpr int off = decltype(SLOT_)::value * kTile + 32 * decltype(U_)::value * 128;
    asm volatile("ds_read_b128 %0, %1 offset:%2"
                 : "=a"(vf[decltype(S_)::value][decltype(U_)::value])
                 : "v"(vbase[decltype(S_)::value]), "i"(off)
                 : "memory");
  };

  // the tail / phantom tile at key offset k0: keys at or past nk are masked
  auto mask = [&](Blk& X, int k0) __attribute__((always_inline)) {
    const int lim = nk - k0 - 8 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = 32 * t + 16 * (i >> 3) + (i & 7);
        X.s[t][i] = (off < lim) ? X.s[t][i] : kNegInf;
      }
  };
  auto exp_cvt = [&](Blk& X) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float s0 = X.s[g >> 3][(2 * g) & 15], s1 = X.s[g >> 3][((2 * g) & 15) + 1];
      X.p[g] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0), (_Float16)__builtin_amdgcn_exp2f(s1)});
    }
  };
  // the rebase of block X (rare: the tile's packed-P max passed 2^thr, or the seed): the exact fp32
  // row max of the tile, O / l / the scores / -m rebased, P recomputed (its row sums are added in the
  // next segment, from the recomputed P)
  auto rebase = [&](Blk& X, auto XB_, half2v pmr_old) __attribute__((always_inline)) {
    constexpr int XB = decltype(XB_)::value;
    float mx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(X.s[j >> 1][8 * (j & 1)], X.s[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
    for (int i = 2; i < 8; i += 2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        mx[j] = fmaxf(fmaxf(mx[j], X.s[j >> 1][8 * (j & 1) + i]), X.s[j >> 1][8 * (j & 1) + i + 1]);
    const float mtf = max_pair32(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
    // close the epoch: its P maximum (approximate) and this tile (exact) into m_max
    const float pold = (float)__builtin_elementwise_maximum(pmr_old[0], pmr_old[1]);
    X.m_max = fmaxf(X.m_max, fmaxf(X.m_run + mtf, X.m_run + __log2f(pold)));
    const bool unset = X.thr < 0.f;
    const bool seed = unset && (mtf > X.thr);
    const float delta = unset ? (seed ? mtf : 0.f) : fmaxf(mtf, 0.f);
    const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
    X.m_run += delta;
    X.thr = (unset && !seed) ? X.thr : kRescaleThr;
    X.thr_h = (unset && !seed) ? (_Float16)-1.f : (_Float16)(1 << (int)kRescaleThr);
#pragma unroll
    for (int x = 0; x < 4; ++x) X.l[x] *= alpha;
    // O only ever appears in AGPR operands (else the allocator parks it in VGPRs around this branch and
    // copies it back and forth on the main path): copy out, scale, copy back, inside the branch
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      floatx16 t;
      asm volatile("; O out" : "=v"(t) : "0"(X.o[u]));
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] *= alpha;
      asm volatile("; O in" : "=a"(X.o[u]) : "0"(t));  // (tied: the compiler moves t into the AGPRs)
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      X.s[0][i] -= delta;
      X.s[1][i] -= delta;
      X.nm[i] = -X.m_run;
    }
    exp_cvt(X);
    X.pmr = half2v{(_Float16)0.f, (_Float16)0.f};
    asm volatile("s_nop 4" ::: "memory");  // (VALU writes of -m / P, then the next segment's MFMAs)
  };
  // the rebase check of block X after its softmax segment
  auto check = [&](Blk& X, auto XB_) __attribute__((always_inline)) {
    const half2v tm = __builtin_bit_cast(half2v, X.pm);
    const _Float16 tmx = __builtin_elementwise_maximum(tm[0], tm[1]);
    const half2v pmr_old = X.pmr;
    X.pmr = __builtin_elementwise_maximum(X.pmr, tm);
    if ((ABL & kANoFill) == 0 && __any(tmx > X.thr_h)) rebase(X, XB_, pmr_old);
  };

  // one gap: MFMA g of block X and block Y's fillers for P dword g
  auto gap = [&](Blk& X, Blk& Y, auto XB_, auto G_) __attribute__((always_inline)) {
    constexpr int g = decltype(G_)::value, XB = decltype(XB_)::value;
    constexpr int mk = (g >= 3 && (g & 1)) ? ((g - 3) >> 1) : -1;  // max fold k: pairs 2k, 2k+1
    float t0, t1;
    const uint32_t pa = mk >= 0 ? Y.p[2 * mk] : 0u, pb = mk >= 0 ? Y.p[2 * mk + 1] : 0u;
    if constexpr ((ABL & kANoFill) != 0) {
      if constexpr (g < 8) {
        constexpr int s = g >> 1, t = g & 1;
        if constexpr (s == 0) asm volatile(FG_MFMA_C : [d] "=&v"(X.s[t]) : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), [c] "v"(X.nm));
        else asm volatile(FG_MFMA : [d] "+v"(X.s[t]) : [a] "v"(kf[s][t]), [b] "a"(X.q[s]));
      } else {
        constexpr int s = (g - 8) >> 1, u = g & 1;
        const u32x4 pp = {X.p[4 * s], X.p[4 * s + 1], X.p[4 * s + 2], X.p[4 * s + 3]};
        asm volatile(FG_MFMA : [d] "+a"(X.o[u]) : [a] "a"(vf[s][u]), [b] "v"(pp));
      }
      (void)t0; (void)t1; (void)pa; (void)pb;
    } else if constexpr (g < 8) {
      constexpr int s = g >> 1, t = g & 1;
      if constexpr (s == 0) {
        if constexpr (mk < 0)
          asm volatile(FG_MFMA_C FG_EXP FG_SUM FG_CVT
                       : [d] "=&v"(X.s[t]), FG_OUT : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), [c] "v"(X.nm), FG_IN);
        else if constexpr (mk == 0)
          asm volatile(FG_MFMA_C FG_EXP FG_SUM FG_MAX2 FG_CVT
                       : [d] "=&v"(X.s[t]), FG_OUT, [pm] "=&v"(Y.pm)
                       : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), [c] "v"(X.nm), FG_IN, [pa] "v"(pa), [pb] "v"(pb));
        else
          asm volatile(FG_MFMA_C FG_EXP FG_SUM FG_MAX3 FG_CVT
                       : [d] "=&v"(X.s[t]), FG_OUT, [pm] "+v"(Y.pm)
                       : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), [c] "v"(X.nm), FG_IN, [pa] "v"(pa), [pb] "v"(pb));
      } else {
        if constexpr (mk < 0)
          asm volatile(FG_MFMA FG_EXP FG_SUM FG_CVT : [d] "+v"(X.s[t]), FG_OUT : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), FG_IN);
        else if constexpr (mk == 0)
          asm volatile(FG_MFMA FG_EXP FG_SUM FG_MAX2 FG_CVT
                       : [d] "+v"(X.s[t]), FG_OUT, [pm] "=&v"(Y.pm)
                       : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), FG_IN, [pa] "v"(pa), [pb] "v"(pb));
        else
          asm volatile(FG_MFMA FG_EXP FG_SUM FG_MAX3 FG_CVT
                       : [d] "+v"(X.s[t]), FG_OUT, [pm] "+v"(Y.pm)
                       : [a] "v"(kf[s][t]), [b] "a"(X.q[s]), FG_IN, [pa] "v"(pa), [pb] "v"(pb));
      }
    } else {
      constexpr int s = (g - 8) >> 1, u = g & 1;
      const u32x4 pp = {X.p[4 * s], X.p[4 * s + 1], X.p[4 * s + 2], X.p[4 * s + 3]};
      if constexpr (mk < 0)
        asm volatile(FG_MFMA FG_EXP FG_SUM FG_CVT : [d] "+a"(X.o[u]), FG_OUT : [a] "a"(vf[s][u]), [b] "v"(pp), FG_IN);
      else
        asm volatile(FG_MFMA FG_EXP FG_SUM FG_MAX3 FG_CVT
                     : [d] "+a"(X.o[u]), FG_OUT, [pm] "+v"(Y.pm)
                     : [a] "a"(vf[s][u]), [b] "v"(pp), FG_IN, [pa] "v"(pa), [pb] "v"(pb));
    }
    // the sources of the MFMA two gaps back stay live until here: the allocator cannot see that an
    // asm statement holds an MFMA still reading them
    if constexpr (g >= 2) {
      constexpr int hh = g - 2;
      if constexpr (hh < 8) asm volatile("" ::"v"(kf[hh >> 1][hh & 1]), "a"(X.q[hh >> 1]));
      else asm volatile("" ::"a"(vf[(hh - 8) >> 1][hh & 1]));
    }
  };
  // the segment's last max fold, after its 16 gaps
  auto seg_tail = [&](Blk& Y) __attribute__((always_inline)) {
    asm volatile("v_pk_maximum3_f16 %[pm], %[pm], %[pa], %[pb]" : [pm] "+v"(Y.pm) : [pa] "v"(Y.p[14]), [pb] "v"(Y.p[15]));
  };

  // segment A of step it (ring slot c = it mod 3): MFMAs of A, softmax of B(it); V(it) k-step 3
  // fragments in gaps 0-1, this thread's chunks of K(it+3) / V(it+2) into LDS in gaps 2-5
  auto seg_a = [&](auto C_) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    auto body = [&](auto G_) __attribute__((always_inline)) {
      constexpr int g = decltype(G_)::value;
      if constexpr (g == 8) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): V(it) for the PV MFMAs
      gap(A, B, IC<0>{}, G_);
      if constexpr (g < 2 && !(ABL & kANoFrag)) read_vf(IC<c>{}, IC<3>{}, G_);
      if constexpr (g == 2 && !(ABL & kANoStage)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // buffer c landed
      if constexpr (g >= 2 && g < 4 && !(ABL & kANoStage)) store(kOffK + c * kTile + kwo[g - 2], kr[c][g - 2]);
      if constexpr (g >= 4 && g < 6 && !(ABL & kANoStage)) store(kOffV + ((c + 2) % kNS) * kTile + vwo[g - 4], vr[c][g - 4]);
      __builtin_amdgcn_sched_barrier(0);
    };
    body(IC<0>{}); body(IC<1>{}); body(IC<2>{}); body(IC<3>{}); body(IC<4>{}); body(IC<5>{}); body(IC<6>{}); body(IC<7>{});
    body(IC<8>{}); body(IC<9>{}); body(IC<10>{}); body(IC<11>{}); body(IC<12>{}); body(IC<13>{}); body(IC<14>{}); body(IC<15>{});
    asm volatile("" ::"a"(vf[3][0]), "a"(vf[3][1]));
    seg_tail(B);
    // this step's LDS stores complete before the next barrier publishes them
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  };
  // segment B of step it: MFMAs of B, softmax of A(it+1); K(it+2) fragments in gaps 2-9, V(it+1)
  // k-steps 0-2 in gaps 10-15; global loads of K(it+4) / V(it+3) in gaps 0-1
  auto seg_b = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    auto body = [&](auto G_) __attribute__((always_inline)) {
      constexpr int g = decltype(G_)::value;
      gap(B, A, IC<1>{}, G_);
      // (segment A ended with lgkmcnt(0): its stores have read buffer c)
      if constexpr (g == 0 && !(ABL & kANoStage)) {
#pragma unroll
        for (int j = 0; j < kCPT; ++j) load_a(kr[c][j], krs, koff[j], (it + 6) * kBN);
      }
      if constexpr (g == 1 && !(ABL & kANoStage)) {
#pragma unroll
        for (int j = 0; j < kCPT; ++j) load_a(vr[c][j], vrs, voff[j], (it + 5) * kBN);
      }
      if constexpr (g >= 2 && g < 10 && !(ABL & kANoFrag)) read_kf(IC<((c + 2) % kNS)>{}, IC<((g - 2) >> 1)>{}, IC<((g - 2) & 1)>{});
      if constexpr (g >= 10 && !(ABL & kANoFrag)) read_vf(IC<((c + 1) % kNS)>{}, IC<((g - 10) >> 1)>{}, IC<(g & 1)>{});
      __builtin_amdgcn_sched_barrier(0);
    };
    body(IC<0>{}); body(IC<1>{}); body(IC<2>{}); body(IC<3>{}); body(IC<4>{}); body(IC<5>{}); body(IC<6>{}); body(IC<7>{});
    body(IC<8>{}); body(IC<9>{}); body(IC<10>{}); body(IC<11>{}); body(IC<12>{}); body(IC<13>{}); body(IC<14>{}); body(IC<15>{});
    asm volatile("" ::"a"(vf[3][0]), "a"(vf[3][1]));
    seg_tail(A);
  };

  // ---- prologue compute: Sᵀ(0) of both blocks from K(0), softmax of A(0) (the seed), K(1) and V(0)
  // fragments; P_B(-1) = 0
  read_kf(IC<0>{}, IC<0>{}, IC<0>{}); read_kf(IC<0>{}, IC<0>{}, IC<1>{}); read_kf(IC<0>{}, IC<1>{}, IC<0>{});
  read_kf(IC<0>{}, IC<1>{}, IC<1>{}); read_kf(IC<0>{}, IC<2>{}, IC<0>{}); read_kf(IC<0>{}, IC<2>{}, IC<1>{});
  read_kf(IC<0>{}, IC<3>{}, IC<0>{}); read_kf(IC<0>{}, IC<3>{}, IC<1>{});
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (s == 0) {
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(A.s[t]) : "v"(kf[s][t]), "a"(A.q[s]), "v"(A.nm));
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(B.s[t]) : "v"(kf[s][t]), "a"(B.q[s]), "v"(B.nm));
      } else {
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(A.s[t]) : "v"(kf[s][t]), "a"(A.q[s]));
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(B.s[t]) : "v"(kf[s][t]), "a"(B.q[s]));
      }
    }
  // (the scores are read below: let the last MFMAs finish)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  read_kf(IC<1>{}, IC<0>{}, IC<0>{}); read_kf(IC<1>{}, IC<0>{}, IC<1>{}); read_kf(IC<1>{}, IC<1>{}, IC<0>{});
  read_kf(IC<1>{}, IC<1>{}, IC<1>{}); read_kf(IC<1>{}, IC<2>{}, IC<0>{}); read_kf(IC<1>{}, IC<2>{}, IC<1>{});
  read_kf(IC<1>{}, IC<3>{}, IC<0>{}); read_kf(IC<1>{}, IC<3>{}, IC<1>{});
  read_vf(IC<0>{}, IC<0>{}, IC<0>{}); read_vf(IC<0>{}, IC<0>{}, IC<1>{}); read_vf(IC<0>{}, IC<1>{}, IC<0>{});
  read_vf(IC<0>{}, IC<1>{}, IC<1>{}); read_vf(IC<0>{}, IC<2>{}, IC<0>{}); read_vf(IC<0>{}, IC<2>{}, IC<1>{});
  read_vf(IC<0>{}, IC<3>{}, IC<0>{}); read_vf(IC<0>{}, IC<3>{}, IC<1>{});
  if (kBN > nk) mask(A, 0);
  exp_cvt(A);
  {
    A.pm = 0u;
#pragma unroll
    for (int g = 0; g < 16; ++g)
      A.pm = __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(half2v, A.pm),
                                                                         __builtin_bit_cast(half2v, A.p[g])));
  }
  check(A, IC<0>{});

  // ---- steps: every step has the same straight-line shape; the last one issues phantom Sᵀ(ntiles)
  // (stale or zero LDS, fully masked, never multiplied into O)
  auto step = [&](auto C_, int it) __attribute__((always_inline)) {
    if constexpr (!(ABL & kANoBar)) __builtin_amdgcn_s_barrier();
    const int k0 = it * kBN;
    if (k0 + kBN > nk) mask(B, k0);
    seg_a(C_);
    check(B, IC<1>{});
    if (k0 + 2 * kBN > nk) mask(A, k0 + kBN);
    seg_b(C_, it);
    check(A, IC<0>{});
  };
  for (int it = 0; it < ntiles; it += kNS) {
    step(IC<0>{}, it);
    if (it + 1 < ntiles) step(IC<1>{}, it + 1);
    if (it + 2 < ntiles) step(IC<2>{}, it + 2);
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
    if (wq0 >= nq) return;
    const int qi = wq0 + r;
    const float l0 = (X.l[0] + X.l[1]) + (X.l[2] + X.l[3]);
    const float m_max = max_pair32(fmaxf(X.m_max, X.m_run + __log2f((float)__builtin_elementwise_maximum(X.pmr[0], X.pmr[1]))));
    const float l_tot = sum_pair32(l0);
    const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
    if (qi >= nq) return;
    if (vd == kD) {
      const __amdgpu_buffer_rsrc_t ors = make_rsrc(O, 2u * vd * nq);
      const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t cst = 32u * u + (i & 3) + 8u * (i >> 2);
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(X.o[u][i] * inv)), ors, vlane,
                                                2u * cst * (uint32_t)nq, 0);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (v < vd) O[(int64_t)v * nq + qi] = __float2half(X.o[u][i] * inv);
        }
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
}

}  // namespace

// the full policy only (the headline): other rules go to the band, pingpong128 or fast kernels
bool fwd_f16_gap_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return a.rule.policy == 0 && dm > 32 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16_gap(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  auto kern = fwd_f16_gap_kernel<0>;
#ifdef FA_DIAG
  switch (diag_variant("FA_FWD_VARIANT") - 2600) {  // timing ablations (outputs wrong)
    case 1: kern = fwd_f16_gap_kernel<0, 1>; break;
    case 2: kern = fwd_f16_gap_kernel<0, 2>; break;
    case 4: kern = fwd_f16_gap_kernel<0, 4>; break;
    case 6: kern = fwd_f16_gap_kernel<0, 6>; break;
    case 7: kern = fwd_f16_gap_kernel<0, 7>; break;
    case 8: kern = fwd_f16_gap_kernel<0, 8>; break;
    case 15: kern = fwd_f16_gap_kernel<0, 15>; break;
    default: break;
  }
#endif
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
