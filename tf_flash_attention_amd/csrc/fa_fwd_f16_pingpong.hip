// fa_fwd_f16_pingpong.hip — fp16 fused attention forward for 32 < max(d, v_d) <= 64 under the full
// policy (BASELINE config 2, the headline): eight waves (two per SIMD) in two groups that alternate
// MFMA and softmax phases ("ping-pong").
//
// At d = 64 a 32-query × 64-key tile is 16 MFMAs (512 matrix cycles) against ≈ 470 cycles of
// VALU / transcendental issue.  One wave cannot overlap the two (its softmax depends on its own
// Sᵀ), and two free-running waves on a SIMD phase-lock behind the workgroup barrier so their MFMA
// and softmax phases collide.  Here the workgroup barrier itself keeps them apart: waves 0-3
// (group 0) and waves 4-7 (group 1) share the four SIMDs, and every barrier interval is an MFMA
// phase for one group and a VALU phase for the other:
//
//   interval  2i  : group 0 MFMA(i)      | group 1 VALU(i-1)
//   interval 2i+1 : group 0 VALU(i)      | group 1 MFMA(i)
//
// (both groups run the same loop; group 1 enters it one barrier late)
//
//   MFMA(i) = Sᵀ MFMAs of tile i + PV MFMAs of tile i-1 (16 MFMAs, unconditional: P is zero for a
//             skipped tile), at priority 1, each pair followed by the fragment reads it frees
//             registers for (K(i+1) after the Sᵀ pairs, V(i) after the PV pairs), one staging store
//             and one staging load pinned after the second pair of each half (sched_group_barrier)
//   VALU(i) = softmax of tile i (tail mask, speculative exp2, rebase check on the packed P, rare
//             rebase, row sums into four running accumulators)
//
// K/V tiles move global → registers (three steps ahead) → LDS; each thread owns one 16-B chunk of
// every tile and stores it in its own MFMA phase, so a tile is complete and published after the
// barrier that ends the second group's MFMA phase.  LDS images: K with 64-B halves swapped on rows
// with c&2, read transposed (ds_read_b64_tr_b16) with the key permutation that makes P's k-step
// registers contiguous keys; V plain rows, 16-B chunks XOR-swizzled by (c>>1)&7.  Rings of three
// slots for K and V.
//
// Numerics: fp32 accumulation, log2-domain lazy rebase at 8, l relative to the stored fp16 m.  The
// rebase check runs on the packed fp16 exponentials: m is exact for tiles that rebased and
// m_run + log2(max P) for the others (< 4.9e-4 from the exact max).  Replaces the reference's
// ForwardImpl (flash_attention.cu:425-1077) for these shapes.
//
// The structures measured against this one (LDS-DMA staging, row sums on the matrix pipe, the
// half-row rebase check, fp32 row sums, finer interleaves, a hand-ordered softmax stream, the
// interval-rule instance) and the stamp / ablation builds were taken out in round 5; their
// measurements are in DESIGN.md §3.0 and §6.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

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
constexpr int kNS = 3;               // ring slots for K and for V (and staging register sets)
constexpr int kOffV = kOffK + kNS * kTile;
constexpr int kSmem = kOffV + kNS * kTile;
constexpr float kRescaleThr = 8.f;

__global__ __launch_bounds__(kNW * 64, 2) void fwd_f16_pingpong_kernel(FwdArgs a) {
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
  const int grp = w >> 2;  // waves w and w+4 share a SIMD
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  const int d = a.d, vd = a.v_d;
  const __half* Q = static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(static_cast<const __half*>(a.K) + bi * (int64_t)d * nk, 2u * d * nk);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk, 2u * vd * nk);
  const bool qvec = ((nq & 7) == 0) && ((reinterpret_cast<uintptr_t>(a.Q) & 15) == 0);
  const float c2 = (float)a.scale * kLog2e;
  const int ntiles = nk > 0 ? (nk + kBN - 1) / kBN : 0;

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

  // ---- prologue: Q, K(0..2), V(0..1) into LDS; K(3..5), V(2..4) into the staging registers
  // (set j serves MFMA(i) with i mod 3 == j; loads run three steps ahead of their store)
  u32x4 kst[kNS], vst[kNS];
  {
    // every load of the prologue in flight at once (the staging registers' too): one memory
    // latency before the loop instead of two
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
    u32x4 kp[3], vp[2];
#pragma unroll
    for (int j = 0; j < 3; ++j) kp[j] = load(krs, koff, j * kBN);
#pragma unroll
    for (int j = 0; j < 2; ++j) vp[j] = load(vrs, voff, j * kBN);
    // the staging loads last: the stores below wait only for the loads before them (vmcnt drains in
    // order), so the tiles three steps ahead stay in flight over the barrier
#pragma unroll
    for (int j = 0; j < kNS; ++j) {
      kst[j] = load(krs, koff, (3 + j) * kBN);
      vst[j] = load(vrs, voff, (2 + j) * kBN);
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
  // tile class: 0 past the end (skipped), 1 the tail tile (masked), 2 every key in range
  auto tcls = [&](int it) -> int __attribute__((always_inline)) {
    if (it < 0 || it >= ntiles) return 0;
    return (it * kBN + kBN - 1 < nk) ? 2 : 1;
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
  half8 vf[4][2];  // V fragments for the next PV (zero before the first: PV(-1) runs unconditionally)
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) vf[s][u][e] = (_Float16)0.f;

  floatx16 st[2];      // Sᵀ of the tile being softmaxed
  uint32_t pw[4][4];   // P (fp16 pairs), dword x of PV k-step s (dwords: extracting them from a
                       // bit-cast half8 miscompiles with this toolchain); zero before the first PV
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
  float m_run = 0.f, m_max = kNegInf, thr = -__FLT_MAX__;
  half2v pmr = {(_Float16)0.f, (_Float16)0.f};  // running max of P over the current epoch (per lane)
  _Float16 thr_h = (_Float16)-1.f;              // 2^thr once seeded; -1 (always exceeded) before
  float lacc[4] = {0.f, 0.f, 0.f, 0.f};         // running row sums (four chains), rescaled at a rebase

  // the tail tile: key offset o of this lane's half is in range iff o < lim
  auto mask = [&](int k0) __attribute__((always_inline)) {
    const int lim = nk - k0 - 8 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = 32 * t + 16 * (i >> 3) + (i & 7);
        st[t][i] = (off < lim) ? st[t][i] : kNegInf;
      }
  };
  auto row_sums = [&]() __attribute__((always_inline)) {
    const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        lacc[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, pw[s][x]), one2, lacc[x], false);
  };
  auto exp_cvt = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const float s0 = st[s >> 1][8 * (s & 1) + 2 * x], s1 = st[s >> 1][8 * (s & 1) + 2 * x + 1];
        pw[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)__builtin_amdgcn_exp2f(s0),
                                                       (_Float16)__builtin_amdgcn_exp2f(s1)});
      }
  };
  // the tile max over the packed fp16 exponentials (8 v_pk_maximum3_f16, no cross-lane step)
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
  // softmax of tile `it`: the exponentials are computed speculatively against m_run; the rebase
  // check asks whether the tile's packed-P max exceeds 2^thr, and only a seed or such a tile (rare)
  // forms the exact fp32 row max and rebases O, l, Sᵀ, -m
  auto softmax = [&](int it, int cls) __attribute__((always_inline)) {
    if (cls == 1) mask(it * kBN);
    exp_cvt();
#pragma unroll
    for (int x = 0; x < 4; ++x)  // pinned here: else they sink past the (rare) rebase branch
      asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
    const half2v tm = pmax_tile();
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
        o[0][i] *= alpha;
        o[1][i] *= alpha;
        st[0][i] -= delta;
        st[1][i] -= delta;
        negm[i] = -m_run;
      }
      exp_cvt();
      pmr = half2v{(_Float16)0.f, (_Float16)0.f};
    }
    row_sums();
  };

  // MFMA(i): Sᵀ of tile i with the K(i+1) fragment reads; PV of tile i-1 (P from VALU(i-1)) with
  // the V(i) fragment reads; this wave's chunks of K(i+3) / V(i+2) into LDS (over K(i) / V(i-1),
  // whose fragments were read in MFMA(i-1)) and the loads of K(i+6) / V(i+5).  All LDS traffic sits
  // in the MFMA phase, beside the matrix pipe, so the VALU phase is the softmax alone.
  auto mfma_phase = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;  // it mod 3
    __builtin_amdgcn_s_setprio(1);
    const lds_char_t* pk = smem + kOffK + ((c + 1) % kNS) * kTile;
    const lds_char_t* pv = smem + kOffV + c * kTile;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qf[s], s == 0 ? negm : st[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kf[t][s].lo = tr_read(pk + kbase[t] + (16 * s) * 128);
        kf[t][s].hi = tr_read(pk + kbase[t] + (16 * s + 4) * 128);
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half8 p = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
#pragma unroll
      for (int u = 0; u < 2; ++u) o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, o[u], 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 2; ++u) vf[s][u] = read_b128(pv + vbase[s] + 32 * u * 128);
    }
    // the order: per Sᵀ k-step two MFMAs then its four K reads, per PV k-step two MFMAs then its
    // two V reads, and one staging store + one staging load after the second pair of each half
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      if (s == 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // a staging store
      if (s == 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // a staging load
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      if (s == 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      if (s == 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    // (unconditional: past the end these move zeros into slots nobody reads unmasked)
    store(kOffK + c * kTile + kwo, kst[c]);
    store(kOffV + ((c + 2) % kNS) * kTile + vwo, vst[c]);
    kst[c] = load(krs, koff, (it + 6) * kBN);
    vst[c] = load(vrs, voff, (it + 5) * kBN);
    // No lgkmcnt drain here: a wave's LDS operations complete in order, and each wave waits for
    // its fragment reads before the MFMAs that use them (MFMA(i+1)), which orders its stores of
    // this phase before any other wave reads those tiles (MFMA(i+2)) and its reads before any
    // wave overwrites their slots (MFMA(i+1) for itself, one interval later for the others).
    __builtin_amdgcn_s_setprio(0);
  };
  // VALU(i): the softmax of tile i; past the end P = 0, so the next (unconditional) PV adds nothing
  auto valu_phase = [&](int it) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staging stores landed
    const int cls = tcls(it);
    if (cls != 0) softmax(it, cls);
    if (cls == 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) pw[x][y] = 0u;
    }
  };

  // Both groups run the same loop (one code path keeps the register allocation sane); group 1
  // enters it one barrier late and group 0 leaves it one barrier late, so every barrier
  // interval pairs one group's MFMA(i) with the other's VALU phase.
  {
    const lds_char_t* p = smem + kOffK;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[t][s].lo = tr_read(p + kbase[t] + (16 * s) * 128);
        kf[t][s].hi = tr_read(p + kbase[t] + (16 * s + 4) * 128);
      }
  }
  if (grp == 1) __builtin_amdgcn_s_barrier();
  auto iter = [&](auto C_, int it) __attribute__((always_inline)) {
    __builtin_amdgcn_s_barrier();
    mfma_phase(C_, it);
    __builtin_amdgcn_s_barrier();
    valu_phase(it);
  };
  // Whole groups of three iterations, none conditional (the last ones past the end only move
  // zeros): with no control flow around the staging loads, hipcc's vmcnt waits stay exact and
  // a store waits only for the load issued three steps earlier.
  for (int it = 0; it <= ntiles; it += kNS) {
    iter(IC<0>{}, it);
    iter(IC<1>{}, it + 1);
    iter(IC<2>{}, it + 2);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();

  // ---- epilogue
  if (!wave_active) return;
  const float l0 = (lacc[0] + lacc[1]) + (lacc[2] + lacc[3]);
  m_max = max_pair32(fmaxf(m_max, m_run + __log2f((float)__builtin_elementwise_maximum(pmr[0], pmr[1]))));
  const float l_tot = sum_pair32(l0);
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
}

}  // namespace

// the full policy only: every other rule goes to the band, pingpong128 or fast kernels
bool fwd_f16_pingpong_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return a.rule.policy == 0 && dm > 32 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

// tuned (c2, MI355X): MFMA phases at priority 1, fragment reads and staging
// interleaved with the MFMAs (0.5526-0.5716 ms against 0.595 without), row sums in running
// accumulators (0.5451 against 0.5552 ms), rebase check and m on the packed P (0.5395-0.5441
// against 0.5512-0.5553 ms)
hipError_t launch_fwd_f16_pingpong(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(fwd_f16_pingpong_kernel), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fwd_f16_pingpong_kernel, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
