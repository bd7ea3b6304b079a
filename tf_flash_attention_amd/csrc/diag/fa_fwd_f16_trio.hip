// fa_fwd_f16_trio.hip — fp16 fused attention forward for 32 < max(d, v_d) <= 64, full policy:
// twelve waves (three per SIMD) in three groups that rotate through one MFMA phase and two
// softmax half-phases ("trio").
//
// The ping-pong forward (fa_fwd_f16_pingpong.hip) pairs one wave's MFMA phase with one wave's
// softmax on each SIMD.  At d = 64 a 32-query x 64-key tile is 16 MFMAs (512 matrix cycles)
// against ~75 VALU instructions of softmax (32 v_exp_f32 among them) issued by that ONE wave:
// a wave alone issues a VALU instruction every ~4 cycles (8-10 for v_exp_f32), so the softmax
// phase (~850 cycles) and not the matrix pipe sets the interval.  Here each SIMD carries three
// waves; in every barrier interval one of them issues its tile's MFMAs and the other two each
// issue HALF of a tile's softmax, so two waves feed the SIMD's VALU at once:
//
//   interval 3i   : group 0 MFMA(i)      | group 1 softB(i-1)  | group 2 softA(i-1)
//   interval 3i+1 : group 0 softA(i)     | group 1 MFMA(i)     | group 2 softB(i-1)
//   interval 3i+2 : group 0 softB(i)     | group 1 softA(i)    | group 2 MFMA(i)
//
//   MFMA(i)  = this wave's staging share (store K(i+1) / V(i), load K(i+2) / V(i+1)), Sᵀ of
//              tile i (8 MFMAs) and PV of tile i-1 (8 MFMAs), the K / V / Q fragments read
//              from LDS inside the phase, each ahead of the MFMA pair that uses it
//   softA(i) = keys 0-31 of tile i: mask, speculative exp2 against m_run, fp16 P, row sums,
//              half the packed-P max
//   softB(i) = keys 32-63: the same, the rebase check on the whole tile's packed P (rare
//              rebase: O, l, Sᵀ, -m rescaled and both halves redone), row sums into l
//
// All three groups share one K/V stream (a K and a V tile per round of three intervals, rings of
// two slots), so a workgroup covers 384 queries.  Numerics are the ping-pong kernel's (fp32
// accumulation, log2-domain lazy rebase at 8, rebase check and m on the packed P, l relative to
// the stored fp16 m).  Replaces the reference's ForwardImpl (flash_attention.cu:425-1077) for
// these shapes.
//
// DIAGNOSTIC LIBRARY ONLY (measured and not taken): on config 2 it runs 0.58-0.61 ms
// against 0.52-0.54 for the ping-pong kernel; without its fragment reads and staging (timing
// ablations 2510-2512, outputs wrong) 0.449 ms, about what the ping-pong reaches without its LDS side.
#include "../fa_device.h"
#include "../fa_kernels.h"
#include "../fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kBN = 64;              // keys per tile
constexpr int kNW = 12;              // waves per workgroup, three per SIMD
constexpr int kBM = 32 * kNW;        // queries per workgroup
constexpr int kQRow = 2 * kBM;       // bytes per Q row in LDS
constexpr int kNS = 2;               // ring slots for K and for V
constexpr float kRescaleThr = 8.f;
// LDS layout for channel count D (32 or 64; channels past d / v_d are zero-padded)
template <int D>
struct TrioLds {
  static constexpr int kTile = D * kBN * 2;             // a K or V tile [D][64]: 8 KB at D = 64
  static constexpr int kOffK = D * kQRow;               // Q image [D][384] first (prologue only)
  static constexpr int kOffV = kOffK + kNS * kTile;
  static constexpr int kOffDummy = kOffV + kNS * kTile;  // non-staging waves' stores land here (never read)
  static constexpr int kSmem = kOffDummy + 2 * 4096;
};

constexpr int kFPrio = 1;    // s_setprio 1 over each MFMA phase
constexpr int kFStamp = 2;   // diagnostic: per-wave s_memtime sums per phase, written over l (l garbage)
constexpr int kFPin = 4;     // fragment reads pinned between the MFMA pairs (sched_group_barrier)
// the next MFMA phase's first K k-step (8 fragment registers) read at the end of softB, before the
// barrier: K(i+1) is complete by then (stored in intervals 3i and 3i+1), and its LDS latency then
// overlaps the barrier wait instead of the first Sᵀ MFMA
constexpr int kFPre = 8;
// the scaled Q fragments written back into the (dead) Q image in lane order after the prologue and
// re-read per k-step inside each MFMA phase (one ds_read_b128 each): 16 fewer live registers
// outside the MFMA phase
constexpr int kFQLds = 16;
// timing ablations (diagnostic library only; outputs WRONG): no K / V fragment reads in the MFMA
// phase (the Q fragments stand in), no staging loads / stores
constexpr int kANoFrag = 32, kANoStage = 64;

template <int D, int F>
__global__ __launch_bounds__(kNW * 64, 3) void fwd_f16_trio_kernel(FwdArgs a) {
  using L = TrioLds<D>;
  constexpr int kTile = L::kTile, kOffK = L::kOffK, kOffV = L::kOffV, kOffDummy = L::kOffDummy;
  constexpr int kKS = D / 16;  // Sᵀ k-steps (channels)
  constexpr int kU = D / 32;   // PV output blocks of 32 channels
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nqb;
  const int q0 = (int)(bid % nqb) * kBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2;  // waves w, w+4, w+8 share a SIMD
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;
  const int ntiles = (nk + kBN - 1) / kBN;

  // ---- staging: threads 0..511 own chunk tid of every K and V tile (8 keys = 16 B of channel row
  // tid / 8); group 2's threads load nothing (out-of-range offsets read zeros) and store into a
  // dummy area, so every wave runs the same branch-free code
  const int cm = tid & 7, crow = tid >> 3;
  const bool stager = tid < 8 * D;
  const uint32_t goff = (uint32_t)crow * (uint32_t)nk * 2u + 16u * cm;
  const uint32_t koff = stager && crow < d ? goff : 0x80000000u, voff = stager && crow < vd ? goff : 0x80000000u;
  const uint32_t kwo = crow * 128 + ((cm * 16) ^ ((crow & 2) << 5));
  const uint32_t vwo = crow * 128 + 16 * (cm ^ ((crow >> 1) & 7));
  const uint32_t dum = kOffDummy + 16u * (tid & 255);
  const uint32_t kdst[2] = {stager ? kOffK + kwo : dum, stager ? kOffK + kTile + kwo : dum};
  const uint32_t vdst[2] = {stager ? kOffV + vwo : dum + 4096u, stager ? kOffV + kTile + vwo : dum + 4096u};
  auto load = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, int k0) -> u32x4 __attribute__((always_inline)) {
    const bool in = k0 + 8 * cm < nk;
    return __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off : 0x80000000u, 2 * min(k0, nk), 0);
  };
  auto store = [&](uint32_t off, u32x4 v) __attribute__((always_inline)) {
    *reinterpret_cast<lds_u32x4_t*>(smem + off) = v;
  };

  // ---- prologue: Q and K(0) into LDS, V(-1)'s slot zeroed (PV(-1) adds 0 x 0); K(1), V(0) into
  // the staging registers
  u32x4 kst, vst;
  {
    const u32x4 k0v = load(krs, koff, 0);
    kst = load(krs, koff, kBN);
    vst = load(vrs, voff, 0);
    constexpr int kQPT = D * (kBM / 8) / (kNW * 64);  // 4 at D = 64
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
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
      const int idx = tid + j * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
      *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[j];
    }
    store(kdst[0], k0v);
    store(vdst[1], u32x4{0, 0, 0, 0});
  }
  __syncthreads();

  // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r]
  half8 qf[kKS];
#pragma unroll
  for (int s = 0; s < kKS; ++s) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int cr = 16 * s + 8 * (g >> 1) + 4 * e + tq;
      const int col = 32 * w + 16 * (g & 1) + 4 * tp;
      const half4 t = tr_read(smem + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
      if (e == 0) qf[s].lo = t; else qf[s].hi = t;
    }
    qf[s] = scale8(qf[s], c2);
  }
  // kFQLds: wave w's lane-ordered fragments at [4 KB * w + 1 KB * s + 16 * lane]
  const uint32_t qlo = 1024u * kKS * w + 16u * lane;
  if constexpr ((F & kFQLds) != 0) {
    __syncthreads();  // every wave has read its columns of the Q image
#pragma unroll
    for (int s = 0; s < kKS; ++s) *reinterpret_cast<lds_half8_t*>(smem + qlo + 1024 * s) = qf[s];
  }

  const int wq0 = q0 + 32 * w;
  const int qi = wq0 + r;
  // tile class: 0 past the end (P = 0), 1 holds the sequence tail (masked), 2 all in range
  auto tcls = [&](int it) -> int __attribute__((always_inline)) {
    if (it >= ntiles) return 0;
    return (it * kBN + kBN - 1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants), as fa_fwd_f16_pingpong.hip:
  //   K: register i of Sᵀ half t holds key 32t + 16(i>>3) + 8h + (i&7)
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g >> 1) + tq) * 128 + (((32 * t + 16 * (g & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  //   V: lane (r, h) reads chunk 2s+h of channel row 32u + r
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  floatx16 st[2];     // Sᵀ of the tile being softmaxed
  uint32_t pw[4][4];  // P (fp16 pairs), dword x of PV k-step s
  floatx16 o[kU];     // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
  floatx16 negm;      // -m_run broadcast: the C operand of every Sᵀ chain
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
#pragma unroll
    for (int u = 0; u < kU; ++u) o[u][i] = 0.f;
    negm[i] = 0.f;
  }
  float m_run = 0.f, m_max = kNegInf, thr = -__FLT_MAX__;
  half2v pmr = {(_Float16)0.f, (_Float16)0.f};  // running max of P over the current epoch (per lane)
  _Float16 thr_h = (_Float16)-1.f;              // 2^thr once seeded; -1 (always exceeded) before
  float lacc[4] = {0.f, 0.f, 0.f, 0.f};         // running row sums (four chains)
  float la[4];                                  // softA's row sums, folded in by softB
  half2v tma = {(_Float16)0.f, (_Float16)0.f};  // softA's packed-P max

  auto mask_half = [&](int t, int k0) __attribute__((always_inline)) {
    const int lim = nk - k0 - 8 * h;  // offset o is in range iff o < lim
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int off = 32 * t + 16 * (i >> 3) + (i & 7);
      st[t][i] = (off < lim) ? st[t][i] : kNegInf;
    }
  };
  // P k-steps 2t, 2t+1 from Sᵀ half t
  auto exp_cvt_half = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 2 * t; s < 2 * t + 2; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const float s0 = st[s >> 1][8 * (s & 1) + 2 * x], s1 = st[s >> 1][8 * (s & 1) + 2 * x + 1];
        pw[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0),
                                                       (_Float16)__builtin_amdgcn_exp2f(s1)});
      }
  };
  auto M3 = [](half2v x, half2v y, half2v z) __attribute__((always_inline)) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z);
  };
  auto H = [&](int s_, int x) __attribute__((always_inline)) { return __builtin_bit_cast(half2v, pw[s_][x]); };
  const half2v one2 = {(_Float16)1.f, (_Float16)1.f};

  // softA(i): keys 0-31
  auto soft_a = [&](int it) __attribute__((always_inline)) {
    const int cls = tcls(it);
    if (cls == 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
      return;
    }
    if (cls == 1) mask_half(0, it * kBN);
    exp_cvt_half(0);
#pragma unroll
    for (int x = 0; x < 2; ++x)
      asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
#pragma unroll
    for (int x = 0; x < 4; ++x)
      la[x] = __builtin_amdgcn_fdot2(H(1, x), one2, __builtin_amdgcn_fdot2(H(0, x), one2, 0.f, false), false);
    tma = M3(M3(H(0, 0), H(0, 1), H(0, 2)), M3(H(0, 3), H(1, 0), H(1, 1)), M3(H(1, 2), H(1, 3), H(1, 3)));
  };
  // softB(i): keys 32-63, the rebase check on the whole tile, the row sums into l
  auto soft_b = [&](int it) __attribute__((always_inline)) {
    const int cls = tcls(it);
    if (cls == 0) return;
    if (cls == 1) mask_half(1, it * kBN);
    exp_cvt_half(1);
#pragma unroll
    for (int x = 2; x < 4; ++x)
      asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
    const half2v tm = M3(M3(H(2, 0), H(2, 1), H(2, 2)), M3(H(2, 3), H(3, 0), H(3, 1)), M3(H(3, 2), H(3, 3), tma));
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
#pragma unroll
      for (int x = 0; x < 4; ++x) lacc[x] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
#pragma unroll
        for (int u = 0; u < kU; ++u) o[u][i] *= alpha;
        st[0][i] -= delta;
        st[1][i] -= delta;
        negm[i] = -m_run;
      }
      exp_cvt_half(0);
      exp_cvt_half(1);
      pmr = half2v{(_Float16)0.f, (_Float16)0.f};
#pragma unroll
      for (int x = 0; x < 4; ++x)
        la[x] = __builtin_amdgcn_fdot2(H(1, x), one2, __builtin_amdgcn_fdot2(H(0, x), one2, 0.f, false), false);
    }
#pragma unroll
    for (int x = 0; x < 4; ++x)
      lacc[x] = __builtin_amdgcn_fdot2(H(3, x), one2, __builtin_amdgcn_fdot2(H(2, x), one2, lacc[x] + la[x], false),
                                       false);
  };

  half8 kf0[2];  // kFPre: K k-step 0 of the next MFMA phase
  auto pre_read = [&](int slot) __attribute__((always_inline)) {
    if constexpr ((F & kFPre) != 0) {
      const lds_char_t* pk = smem + kOffK + slot * kTile;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kf0[t].lo = tr_read(pk + kbase[t]);
        kf0[t].hi = tr_read(pk + kbase[t] + 4 * 128);
      }
    }
  };
  // MFMA(i): staging share, Sᵀ(i) from K slot i&1, PV(i-1) from V slot (i-1)&1
  auto mfma_phase = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;  // it & 1
    if (F & kFPrio) __builtin_amdgcn_s_setprio(1);
    // K(i+1) over K(i-1) (read in the previous round), V(i) over V(i-2)
    if constexpr ((F & kANoStage) == 0) {
      store(kdst[c ^ 1], kst);
      store(vdst[c], vst);
      kst = load(krs, koff, (it + 2) * kBN);
      vst = load(vrs, voff, (it + 1) * kBN);
    }
    const lds_char_t* pk = smem + kOffK + c * kTile;
    const lds_char_t* pv = smem + kOffV + (c ^ 1) * kTile;
    half8 kf[kKS][2];
#pragma unroll
    for (int s = 0; s < kKS; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if ((F & kFPre) && s == 0) {
          kf[s][t] = kf0[t];
          continue;
        }
        if (F & kANoFrag) {
          kf[s][t] = qf[s];
          continue;
        }
        kf[s][t].lo = tr_read(pk + kbase[t] + (16 * s) * 128);
        kf[s][t].hi = tr_read(pk + kbase[t] + (16 * s + 4) * 128);
      }
    half8 vf[4][kU];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < kU; ++u) vf[s][u] = (F & kANoFrag) ? qf[(s + u) % kKS] : read_b128(pv + vbase[s] + 32 * u * 128);
#pragma unroll
    for (int s = 0; s < kKS; ++s) {
      const half8 qs = (F & kFQLds) ? read_b128(smem + qlo + 1024 * s) : qf[s];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[s][t], qs, s == 0 ? negm : st[t], 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half8 p = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
#pragma unroll
      for (int u = 0; u < kU; ++u) o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, o[u], 0, 0, 0);
    }
    if constexpr ((F & kFPin) != 0 && D == 64) {
      // staging (2 LDS stores, 2 loads), then K k-steps 0-1 read ahead; each MFMA pair followed by
      // the reads two k-steps ahead; V reads under the last Sᵀ pairs
      __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (s < 2) __builtin_amdgcn_sched_group_barrier(0x100, 0, 0);
      }
    }
    if (F & kFPrio) __builtin_amdgcn_s_setprio(0);
  };

  uint64_t st_acc[4] = {0, 0, 0, 0}, st_prev = 0;
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

  // group g enters the rotation g barriers late and leaves it 2-g barriers early, so each barrier
  // interval holds one group's MFMA phase and the other two groups' softmax halves
  pre_read(0);
  if (grp >= 1) __builtin_amdgcn_s_barrier();
  if (grp >= 2) __builtin_amdgcn_s_barrier();
  auto round = [&](auto C_, int it) __attribute__((always_inline)) {
    stamp(-1);
    __builtin_amdgcn_s_barrier();
    stamp(3);
    mfma_phase(C_, it);
    stamp(0);
    __builtin_amdgcn_s_barrier();
    stamp(3);
    soft_a(it);
    stamp(1);
    __builtin_amdgcn_s_barrier();
    stamp(3);
    soft_b(it);
    pre_read(decltype(C_)::value ^ 1);
    stamp(2);
  };
  // whole pairs of rounds (slot indices compile-time); rounds past the last tile move zeros
  for (int it = 0; it <= ntiles; it += 2) {
    round(IC<0>{}, it);
    round(IC<1>{}, it + 1);
  }
  if (grp <= 1) __builtin_amdgcn_s_barrier();
  if (grp <= 0) __builtin_amdgcn_s_barrier();

  // ---- epilogue
  if (wq0 >= nq) return;
  m_max = max_pair32(fmaxf(m_max, m_run + __log2f((float)__builtin_elementwise_maximum(pmr[0], pmr[1]))));
  const float l_tot = sum_pair32((lacc[0] + lacc[1]) + (lacc[2] + lacc[3]));
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi >= nq) return;
  __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
  if (vd == D) {
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(O, 2u * vd * nq);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t cst = 32u * u + (i & 3) + 8u * (i >> 2);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(o[u][i] * inv)), ors, vlane,
                                              2u * cst * (uint32_t)nq, 0);
      }
  } else {
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (v < vd) O[(int64_t)v * nq + qi] = __float2half(o[u][i] * inv);
      }
  }
  if (h == 0) {
    float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
    __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
    if constexpr ((F & kFStamp) != 0) {  // diagnostic build: phase cycle sums over this wave's l
      if (r < 4) lo[qi] = (float)(r == 0 ? st_acc[0] : r == 1 ? st_acc[1] : r == 2 ? st_acc[2] : st_acc[3]);
      return;
    }
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

template <int F>
hipError_t launch_t(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const bool d32 = max(a.d, a.v_d) <= 32;
  auto kern = d32 ? fwd_f16_trio_kernel<32, F> : fwd_f16_trio_kernel<64, F>;
  const int smem = d32 ? TrioLds<32>::kSmem : TrioLds<64>::kSmem;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), smem, s, a);
  return hipGetLastError();
}

}  // namespace

bool fwd_f16_trio_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return a.rule.policy == 0 && dm <= 64 && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

constexpr int kFDefault = kFPrio;

hipError_t launch_fwd_f16_trio(const FwdArgs& a, hipStream_t s) {
  switch (diag_variant("FA_FWD_VARIANT")) {
    case 2500: return launch_t<0>(a, s);
    case 2501: return launch_t<kFPrio>(a, s);
    case 2502: return launch_t<kFPin>(a, s);
    case 2503: return launch_t<kFDefault | kFStamp>(a, s);
    case 2504: return launch_t<kFPrio | kFPin>(a, s);
    case 2505: return launch_t<kFPrio | kFPre>(a, s);
    case 2506: return launch_t<kFPrio | kFPre | kFStamp>(a, s);
    case 2507: return launch_t<kFPrio | kFQLds>(a, s);
    case 2508: return launch_t<kFPrio | kFQLds | kFPre>(a, s);
    case 2509: return launch_t<kFPrio | kFQLds | kFPre | kFStamp>(a, s);
    case 2510: return launch_t<kFPrio | kANoFrag>(a, s);
    case 2511: return launch_t<kFPrio | kANoStage>(a, s);
    case 2512: return launch_t<kFPrio | kANoFrag | kANoStage>(a, s);
    case 2513: return launch_t<kFPrio | kANoFrag | kANoStage | kFStamp>(a, s);
    case 2514: return launch_t<kFStamp>(a, s);
    default: break;
  }
  return launch_t<kFDefault>(a, s);
}

}  // namespace fa
