// fa_fwd_f16_pingpong128.hip — the ping-pong fp16 forward (fa_fwd_f16_pingpong.hip) for
// 64 < max(d, v_d) <= 128, full policy and interval rules.
//
// Same two-group structure: eight waves, waves w and w+4 share SIMD w, and every barrier
// interval is an MFMA phase for one group and the softmax phase for the other.  At d = 128 the
// MFMA phase carries 32 MFMAs (1024 matrix cycles) against the same ≈ 500-cycle softmax, so
// the matrix pipe of each SIMD is fed in every interval by one of its two waves.
//
// What changes against the d = 64 kernel is the register budget (two waves per SIMD, 256
// VGPRs each): K and V fragments are held one half (64 channels / 64 V rows) at a time, and
// the scores come out of the MFMA relative to 0 (no broadcast -m C operand; the softmax
// subtracts the running reference itself — it has slack at this d).  Inside MFMA(i), one staging
// chunk (store + next load) before each of the four MFMA blocks:
//
//   Sᵀ(i)   k-steps 0..3 (K(i) half 0 and Q half 0, read at the head of VALU(i-1))
//   read    K(i) half 1, Q half 1
//   PV(i-1) V rows 0..63 (V(i-1) half 0, read at the head of VALU(i-1))
//   read    V(i-1) half 1
//   Sᵀ(i)   k-steps 4..7;  PV(i-1) V rows 64..127
//
// and VALU(i) opens with the reads of K(i+1) half 0, Q half 0 and V(i) half 0 for MFMA(i+1) (those
// tiles were published before MFMA(i) began), then runs the softmax of tile i; the scalar tile-class
// work of MFMA(i+1) runs at its end, where the SALU is idle.
//
// Causal (interval rules, round 5): a workgroup runs two query blocks of one slice, the heavy block
// nqb-1-j with its key tiles walked upwards, then the light block j walked downwards.  Every pair of
// a slice then costs the same number of key tiles, and all pairs of a slice read key tile t at the
// same time in both passes (pass 1 of pair j starts when its pass 0 ends and reaches tile t at a time
// independent of j), so the slices in flight on an XCD share each K / V tile in its L2 instead of
// re-fetching it (the heavy-first order of one block per workgroup read 1.42x the Q / K / V bytes).
//
// LDS (160 KB): K and V rings of three 16 KB tiles, then the Q image [128][256] (in the prologue;
// then the waves' scaled Q fragments), in the d = 64 kernel's images (K: 64-B halves swapped on rows
// with c&2, transposed reads with the key permutation; V: 16-B chunks XOR-swizzled by (c>>1)&7, b128
// operand reads).  Numerics as fa_fwd_f16.hip.  Replaces the reference's ForwardImpl
// (flash_attention.cu:425-1077) for these shapes.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 128;
constexpr int kBN = 64;               // keys per tile
constexpr int kNW = 8;                // waves per workgroup, two per SIMD
constexpr int kBM = 32 * kNW;         // queries per workgroup
constexpr int kNS = 3;                // ring slots for K and for V
constexpr int kQRow = 2 * kBM;        // bytes per Q row in LDS
constexpr int kTile = kD * kBN * 2;   // 16 KB
// K ring, V ring, then the Q image [128][256] (prologue; then the scaled Q fragments): every
// fragment read and staging store is a lane-constant VGPR base (the ring's offset folded in) plus
// an immediate below 64 KB, so no address arithmetic runs in the loop
constexpr int kOffK = 0;
constexpr int kOffV = kOffK + kNS * kTile;
constexpr int kOffQ = kOffV + kNS * kTile;
constexpr int kSmem = kOffQ + kD * kQRow;  // 160 KB
constexpr int kCPT = kD * 8 / (kNW * 64);   // 16-B chunks per thread per tile (2)
constexpr float kRescaleThr = 8.f;

// query blocks a workgroup runs: one (full policy), or the heavy / light pair of an interval rule
__host__ __device__ inline int64_t pp128_groups(int64_t nqb, int pol) { return pol == 0 ? nqb : (nqb + 1) / 2; }

template <int POL>
__global__ __launch_bounds__(kNW * 64, 2) void fwd_f16_pingpong128_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;
  constexpr float kNegInf = -__builtin_huge_valf();

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nqb = (nq + kBM - 1) / kBM;
  const uint32_t ngr = (uint32_t)pp128_groups(nqb, POL);
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / ngr;
  const uint32_t j = bid % ngr;
  // full: block j (latest first); interval rules: heavy block nqb-1-j, then light block j (if distinct)
  const int npass = (POL == 0 || nqb - 1 - j == j) ? 1 : 2;
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

  // ---- staging: chunk j of this thread = 8 keys (16 B) of channel row (tid + 512 j) >> 3
  const int cm = tid & 7;
  uint32_t koff[kCPT], voff[kCPT], kwo[kCPT], vwo[kCPT];
#pragma unroll
  for (int jj = 0; jj < kCPT; ++jj) {
    const int c = (tid + kNW * 64 * jj) >> 3;
    const uint32_t go = (uint32_t)c * (uint32_t)nk * 2u + 16u * cm;
    koff[jj] = c < d ? go : 0x80000000u;
    voff[jj] = c < vd ? go : 0x80000000u;
    kwo[jj] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));
    vwo[jj] = kOffV + c * 128 + 16 * (cm ^ ((c >> 1) & 7));  // the V ring's offset folded in
    asm volatile("" : "+v"(vwo[jj]));
  }
  // fragment read bases (lane constants): K transposed reads with the key permutation σ
  // (register i of Sᵀ half t holds key 32t + 16(i>>3) + 8h + (i&7)); V chunk 2s+h of row 32u + r
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g >> 1) + tq) * 128 + (((32 * t + 16 * (g & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    vbase[s] = kOffV + r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));
    asm volatile("" : "+v"(vbase[s]));  // the V ring's offset stays in the VGPR (see kOffQ)
  }
  uint32_t qfrag = kOffQ + 8192 * w + 16 * lane;
  asm volatile("" : "+v"(qfrag));  // opaque: the 96 KB stays in the VGPR, the k-step offset in the immediate

  // one query block; REV: its key tiles walked downwards (the light block of a pair)
  auto run_block = [&](auto REV_, const int q0) __attribute__((always_inline)) {
    constexpr bool rev = decltype(REV_)::value;

    // ---- key range of the block (rule-bounded)
    const int qlast = min(q0 + kBM, nq) - 1;
    int kb = 0, ke = nk;
    if (POL != 0) k_range_for_q_block(a.rule, q0, qlast, &kb, &ke);
    const int kt0 = (kb / kBN) * kBN;
    const int ntiles = (ke > kb) ? (ke - kt0 + kBN - 1) / kBN : 0;
    // position it of the key loop -> key offset of its tile; positions past the last tile stay past
    // it (zero tiles)
    // (REV: positions past the last tile fall below kt0, to negative keys: zero tiles as well)
    const int kfirst = rev ? kt0 + (ntiles - 1) * kBN : kt0;
    auto tk0 = [&](int it) -> int __attribute__((always_inline)) { return rev ? kfirst - it * kBN : kfirst + it * kBN; };
    // branch-free (exact vmcnt waits): chunks past nk — the tail, tiles past the end — read as zeros
    auto load = [&](u32x4 (&dst)[kCPT], __amdgpu_buffer_rsrc_t rs, const uint32_t (&off)[kCPT], int k0)
        __attribute__((always_inline)) {
      const bool in = (unsigned)(k0 + 8 * cm) < (unsigned)nk;
#pragma unroll
      for (int jj = 0; jj < kCPT; ++jj)
        dst[jj] = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off[jj] : 0x80000000u, 2 * min(max(k0, 0), nk), 0);
    };
    auto store = [&](int base, const uint32_t (&wo)[kCPT], const u32x4 (&src)[kCPT]) __attribute__((always_inline)) {
#pragma unroll
      for (int jj = 0; jj < kCPT; ++jj) *reinterpret_cast<lds_u32x4_t*>(smem + base + wo[jj]) = src[jj];
    };

    // ---- prologue: Q, K(0), K(1), V(0) into LDS; K(2), V(1) into the staging registers
    if (rev) __syncthreads();  // every wave is past its last LDS read of the previous block
    // the prologue's addresses from an opaque thread id: else hipcc keeps the first block's Q-image
    // store addresses live (16 VGPRs) over its whole key loop for the second block, and spills them
    int tidb = tid;
    asm volatile("" : "+v"(tidb));
    u32x4 kst[kCPT], vst[kCPT];
    {
      u32x4 k0v[kCPT], k1v[kCPT], v0v[kCPT];
      load(k0v, krs, koff, tk0(0));
      load(k1v, krs, koff, tk0(1));
      load(v0v, vrs, voff, tk0(0));
      // Q [128][256], 64-B blocks XOR-swizzled by c&3: all of a thread's loads before its stores
      constexpr int kQPT = kD * (kBM / 8) / (kNW * 64);
      u32x4 qv[kQPT];
#pragma unroll
      for (int jj = 0; jj < kQPT; ++jj) {
        const int idx = tidb + jj * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        qv[jj] = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int jj = 0; jj < kQPT; ++jj) {
        const int idx = tidb + jj * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        *reinterpret_cast<lds_u32x4_t*>(smem + kOffQ + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[jj];
      }
      store(kOffK, kwo, k0v);
      store(kOffK + kTile, kwo, k1v);
      store(0, vwo, v0v);
      load(kst, krs, koff, tk0(2));
      load(vst, vrs, voff, tk0(1));
    }
    __syncthreads();

    // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r].
    // The scaled fragments go back into the (then dead) Q image in lane order — wave w's 8 KB, k-step
    // s at 1 KB·s, lane L at 16 L — and each MFMA phase reads the half it needs with four b128 reads:
    // holding all eight k-steps would cost 16 more VGPRs than the two-waves-per-SIMD budget has.
    {
      half8 qf[kD / 16];
#pragma unroll
      for (int s = 0; s < kD / 16; ++s) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int cr = 16 * s + 8 * (g >> 1) + 4 * e + tq;
          const int col = 32 * w + 16 * (g & 1) + 4 * tp;
          const half4 t = tr_read(smem + kOffQ + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
          if (e == 0) qf[s].lo = t; else qf[s].hi = t;
        }
        qf[s] = scale8(qf[s], c2);
      }
      __syncthreads();  // every wave has its fragments before the image is overwritten
#pragma unroll
      for (int s = 0; s < kD / 16; ++s)
        *reinterpret_cast<lds_half8_t*>(smem + kOffQ + 8192 * w + 1024 * s + 16 * lane) = qf[s];
    }
    half8 qh[4];  // Q fragments of one channel half
    auto read_q = [&](int half) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 4; ++s) qh[s] = read_b128(smem + qfrag + 1024 * (4 * half + s));
    };

    const int wq0 = q0 + 32 * w;
    const int qi = wq0 + r;
    const bool wave_active = wq0 < nq;
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
      const int k0 = tk0(it), k1 = k0 + kBN - 1;
      if (POL == 0) return (k1 < nk) ? 2 : 1;
      if (!wave_active || wlo_min > k1 || whi_max < k0) return 0;
      return (wlo_max <= k0 && whi_min >= k1 && k1 < nk) ? 2 : 1;
    };

    half8 kf[2][4];  // K fragments of one channel half: k-steps 4·half + 0..3
    half8 vf[4][2];  // V fragments of one row half: rows 64·half + 32u + r
    auto read_k = [&](int slot, int half) __attribute__((always_inline)) {
      const lds_char_t* p = smem + kOffK + slot * kTile;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ss = 4 * half + s;
          kf[t][s].lo = tr_read(p + kbase[t] + (16 * ss) * 128);
          kf[t][s].hi = tr_read(p + kbase[t] + (16 * ss + 4) * 128);
        }
    };
    auto read_v = [&](int slot, int half) __attribute__((always_inline)) {
      const lds_char_t* p = smem + slot * kTile;  // kOffV is in vbase
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) vf[s][u] = read_b128(p + vbase[s] + (64 * half + 32 * u) * 128);
    };

    floatx16 st[2];      // Sᵀ of the tile being softmaxed (relative to 0 out of the MFMA)
    uint32_t pw[4][4];   // P (fp16 pairs), dword x of PV k-step s
    floatx16 o[4];       // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[u][i] = 0.f;
    float m_run = 0.f, l0 = 0.f, l1 = 0.f, m_max = kNegInf, thr = -__FLT_MAX__;

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
    // softmax of tile `it` (see fa_fwd_f16_pingpong.hip); the scores are first moved to the running
    // reference m_run (at this d the VALU phase has room for the subtraction)
    auto softmax = [&](int it, int cls) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[0][i] -= m_run;
        st[1][i] -= m_run;
      }
      if (cls == 1) mask(tk0(it));
      float mx[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mx[jj] = fmaxf(st[jj >> 1][8 * (jj & 1)], st[jj >> 1][8 * (jj & 1) + 1]);
#pragma unroll
      for (int i = 2; i < 8; i += 2)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          mx[jj] = fmaxf(fmaxf(mx[jj], st[jj >> 1][8 * (jj & 1) + i]), st[jj >> 1][8 * (jj & 1) + i + 1]);
      const float mt = max_pair32(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
      m_max = fmaxf(m_max, m_run + mt);
      exp_cvt();
#pragma unroll
      for (int x = 0; x < 4; ++x)  // pinned here: else they sink past the (rare) rebase branch
        asm volatile("" : "+v"(pw[x][0]), "+v"(pw[x][1]), "+v"(pw[x][2]), "+v"(pw[x][3]));
      if (__any(mt > thr)) {
        const bool unset = thr < 0.f;
        const bool seed = unset && (mt > thr);
        const float delta = unset ? (seed ? mt : 0.f) : fmaxf(mt, 0.f);
        const float alpha = unset ? 1.f : __builtin_amdgcn_exp2f(-delta);
        m_run += delta;
        thr = (unset && !seed) ? thr : kRescaleThr;
        l0 *= alpha;
        l1 *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
#pragma unroll
          for (int u = 0; u < 4; ++u) o[u][i] *= alpha;
          st[0][i] -= delta;
          st[1][i] -= delta;
        }
        exp_cvt();
      }
      const half2v one2 = {(_Float16)1.f, (_Float16)1.f};
      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 4; ++x) ls[x] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2v, pw[s][x]), one2, ls[x], false);
      l0 += ls[0] + ls[2];
      l1 += ls[1] + ls[3];
    };

    auto qk = [&](int half) __attribute__((always_inline)) {
      const floatx16 zero = {};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t][s], qh[s], (half == 0 && s == 0) ? zero : st[t], 0, 0, 0);
    };
    auto pv = [&](int half) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const half8 p = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
#pragma unroll
        for (int u = 0; u < 2; ++u)
          o[2 * half + u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[s][u], p, o[2 * half + u], 0, 0, 0);
      }
    };

    // the scalar tile-class work of MFMA(it+1) runs at the end of VALU(it), where the SALU is idle
    // (wave-uniform: kept in SGPRs over the barrier)
    int cls_q = tcls(0), cls_p = 0;  // classes of the tiles of the next Sᵀ (it) and PV (it - 1)
    auto mfma_phase = [&](auto C_, int it) __attribute__((always_inline)) {
      constexpr int c = decltype(C_)::value;  // it mod 3
      // chunk q (K0, K1, V0, V1) stored and re-loaded before MFMA block q, so each group's 16 loads
      // and 16 stores reach the TA / LDS a quarter at a time under the MFMAs
      // (unconditional: past the end these move zeros into slots nobody reads unmasked)
      auto stage1 = [&](int q) __attribute__((always_inline)) {
        const int jj = q & 1;
        if (q < 2) {
          *reinterpret_cast<lds_u32x4_t*>(smem + kOffK + ((c + 2) % kNS) * kTile + kwo[jj]) = kst[jj];  // K(i+2) over K(i-1)
          const int k0 = tk0(it + 3);
          kst[jj] = __builtin_amdgcn_raw_buffer_load_b128(krs, ((unsigned)(k0 + 8 * cm) < (unsigned)nk) ? koff[jj] : 0x80000000u,
                                                          2 * min(max(k0, 0), nk), 0);
        } else {
          *reinterpret_cast<lds_u32x4_t*>(smem + ((c + 1) % kNS) * kTile + vwo[jj]) = vst[jj];  // V(i+1) over V(i-2)
          const int k0 = tk0(it + 2);
          vst[jj] = __builtin_amdgcn_raw_buffer_load_b128(vrs, ((unsigned)(k0 + 8 * cm) < (unsigned)nk) ? voff[jj] : 0x80000000u,
                                                          2 * min(max(k0, 0), nk), 0);
        }
      };
      __builtin_amdgcn_s_setprio(1);
      const bool dq = cls_q != 0, dp = cls_p != 0;
      stage1(0);
      if (dq) qk(0);
      stage1(1);
      read_k(c, 1);
      read_q(1);
      if (dp) pv(0);
      stage1(2);
      read_v((c + 2) % kNS, 1);
      if (dq) qk(1);
      stage1(3);
      if (dp) pv(1);
      // this phase's stores are complete before its barrier: the other group reads K(i+2) / V(i+1)
      // at the end of the next interval (the reads above were already waited for by the MFMAs)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_setprio(0);
    };
    auto valu_phase = [&](auto C_, int it) __attribute__((always_inline)) {
      // K(i+1) / V(i) were published before MFMA(i) began; this interval's stores (the other
      // group's MFMA phase) go to the K(i-1) / V(i-2) slots
      constexpr int c = decltype(C_)::value;
      read_k((c + 1) % kNS, 0);
      read_q(0);
      read_v(c, 0);
      const int cls = cls_q;
      if (cls != 0) softmax(it, cls);
      cls_p = cls;
      cls_q = tcls(it + 1);
    };

    // both groups run the same loop; group 1 enters it one barrier late (see fa_fwd_f16_pingpong.hip)
    read_k(0, 0);
    read_q(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (grp == 1) __builtin_amdgcn_s_barrier();
    auto iter = [&](auto C_, int it) __attribute__((always_inline)) {
      __builtin_amdgcn_s_barrier();
      mfma_phase(C_, it);
      __builtin_amdgcn_s_barrier();
      valu_phase(C_, it);
    };
    for (int it = 0; it <= ntiles; it += kNS) {
      iter(IC<0>{}, it);
      iter(IC<1>{}, it + 1);
      iter(IC<2>{}, it + 2);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();

    // ---- epilogue (no early return: a second block may follow)
    const float l_tot = sum_pair32(l0 + l1);
    const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
    if (wave_active && qi < nq) {
      __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (v < vd) O[(int64_t)v * nq + qi] = __float2half(o[u][i] * inv);
        }
      if (h == 0) {
        float* lo = static_cast<float*>(a.l) + bi * (int64_t)nq;
        __half* mo = static_cast<__half*>(a.m) + bi * (int64_t)nq;
        if (l_tot > 0.f) {
          const __half mT = __float2half(m_max * kLn2);
          lo[qi] = l_tot * __builtin_amdgcn_exp2f(m_run - __half2float(mT) * kLog2e);
          mo[qi] = mT;
        } else {
          lo[qi] = 0.f;
          mo[qi] = neg_inf_approx<__half>();
        }
      }
    }
  };
  run_block(IC<0>{}, (int)(nqb - 1 - j) * kBM);
  if (npass == 2) {
    int q0 = (int)j * kBM;
    asm volatile("" : "+s"(q0));  // keeps the light block's setup from being hoisted into the first
    run_block(IC<1>{}, q0);
  }
}

}  // namespace

bool fwd_f16_pingpong128_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  return dm > 64 && dm <= kD && (nk % 8 == 0) && nk > 0 && (int64_t)dm * nk * 2 < (1ll << 31) &&
         (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.V) % 16 == 0) &&
         rule_is_interval(a.rule) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16_pingpong128(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const int pol = a.rule.policy == 0 ? 0 : 1;
  auto kern = pol == 0 ? fwd_f16_pingpong128_kernel<0> : fwd_f16_pingpong128_kernel<1>;
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * pp128_groups(nqb, pol))), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
