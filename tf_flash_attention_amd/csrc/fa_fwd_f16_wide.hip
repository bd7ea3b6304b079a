// fa_fwd_f16_wide.hip — fp16 fused attention forward on MFMA for 128 < max(d, v_d) <= 256 (channels
// zero-padded to 256), every rule: full (POL 0), interval rules (POL 1: causal, 1d unit-stride local
// windows) and the other local windows (POL 2: strided, look-ahead, 2d; per-element order checks on
// the edge tiles).  ALN: 16-B chunk staging (nk % 8 == 0, K / V 16-B aligned); otherwise the same
// chunks are gathered element by element (zeros past nk), the LDS images unchanged.
//
// At 256 channels a 32-query x 64-key tile is 64 MFMAs (32 for Sᵀ = Kᵀ·Q over 16 channel k-steps,
// 32 for Oᵀ += V·Pᵀ over 8 blocks of 32 output channels) against the same ~120 VALU instructions of
// softmax as at d = 64, so the kernel is matrix-bound with one wave per SIMD and needs no role split:
// each wave runs Sᵀ(i) -> softmax(i) -> PV(i) on its own 32 queries, four waves (128 queries) share
// the K / V tiles of a workgroup.
//
//   registers (one wave per SIMD, 512 available): Oᵀ 128, scaled Q fragments 64 (all 16 k-steps),
//   Sᵀ 32, P 16, staging 32, K / V fragments streamed two MFMAs ahead
//   LDS: K ring 2 x 32 KB, V ring 2 x 32 KB (tile t in slot t & 1); the Q image [256][128] occupies
//   the K ring during the prologue only
//   staging: K(i+1) loaded at the head of Sᵀ(i), stored after it; V(i+1) loaded at the head of
//   softmax(i), stored after PV(i); one barrier per tile publishes both
//
// Layouts and numerics follow fa_fwd_f16_pingpong128.hip (the K image with 64-B halves swapped on
// rows with c & 2 read by transposed reads whose key columns are σ-permuted, V rows with XOR-swizzled
// 16-B chunks read as b128, scores relative to 0 out of the MFMA, exact fp32 row max, log2-domain
// lazy rebase at 8, l relative to the stored fp16 m).  Replaces the reference's ForwardImpl
// (flash_attention.cu:425-1077), whose channel count is bounded only by shared memory
// (flash_attention.cu:1977-2067), for these shapes; before round 4 they ran on the SIMT kernel.
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 256;
constexpr int kBN = 64;                // keys per tile
constexpr int kNW = 4;                 // waves per workgroup, one per SIMD
constexpr int kBM = 32 * kNW;          // queries per workgroup
constexpr int kQRow = 2 * kBM;         // bytes per Q row in LDS (prologue)
constexpr int kTile = kD * kBN * 2;    // 32 KB
constexpr int kOffV = 2 * kTile;       // K ring [0, 64 KB), V ring [64 KB, 128 KB)
constexpr int kSmem = 4 * kTile;       // 128 KB (the Q image, 64 KB, aliases the K ring)
constexpr int kCPT = kD * 8 / (kNW * 64);  // 16-B chunks of a tile per thread: 8
constexpr float kRescaleThr = 8.f;

template <int POL, bool ALN>
__global__ __launch_bounds__(kNW * 64, 1) void fwd_f16_wide_kernel(FwdArgs a) {
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

  // ---- staging: chunk j of this thread = 8 keys (16 B) of channel row (tid + 256 j) >> 3
  const int cm = tid & 7;
  uint32_t koff[kCPT], voff[kCPT], kwo[kCPT], vwo[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int c = (tid + kNW * 64 * j) >> 3;
    const uint32_t go = (uint32_t)c * (uint32_t)nk * 2u + (ALN ? 16u * cm : 0u);
    // (ALN: the row's chunk offset, 0x80000000 for a padding row; else the row start, checked per load)
    koff[j] = (!ALN || c < d) ? go : 0x80000000u;
    voff[j] = (!ALN || c < vd) ? go : 0x80000000u;
    kwo[j] = c * 128 + ((cm * 16) ^ ((c & 2) << 5));
    vwo[j] = kOffV + c * 128 + 16 * (cm ^ ((c >> 1) & 7));
  }
  // branch-free: chunks past nk (the tail, tiles past the end) read as zeros
  auto load = [&](u32x4 (&dst)[kCPT], __amdgpu_buffer_rsrc_t rs, const uint32_t (&off)[kCPT], int rows, int k0)
      __attribute__((always_inline)) {
    const bool in = k0 + 8 * cm < nk;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      if constexpr (ALN)
        dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? off[j] : 0x80000000u, 2 * min(k0, nk), 0);
      else
        dst[j] = buf_load8h(rs, off[j], k0 + 8 * cm, nk, ((tid + kNW * 64 * j) >> 3) < rows);
    }
  };
  auto store = [&](int base, const uint32_t (&wo)[kCPT], const u32x4 (&src)[kCPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) *reinterpret_cast<lds_u32x4_t*>(smem + base + wo[j]) = src[j];
  };

  // ---- prologue: the Q image [256][128] over the K ring, the scaled fragments into registers; then
  // K(0), V(0) into slot 0
  half8 qf[kD / 16];
  {
    constexpr int kQPT = kD * (kBM / 8) / (kNW * 64);  // 16 chunks a thread, in two batches
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      u32x4 qv[kQPT / 2];
#pragma unroll
      for (int j = 0; j < kQPT / 2; ++j) {
        const int idx = tid + (b2 * kQPT / 2 + j) * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        qv[j] = (c < d) ? load_chunk8(Q + (int64_t)c * nq, q0 + 8 * m, nq, qvec) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int j = 0; j < kQPT / 2; ++j) {
        const int idx = tid + (b2 * kQPT / 2 + j) * kNW * 64, c = idx / (kBM / 8), m = idx % (kBM / 8);
        *reinterpret_cast<lds_u32x4_t*>(smem + c * kQRow + ((m * 16) ^ ((c & 3) << 6))) = qv[j];
      }
    }
    __syncthreads();
    // Q*scale*log2(e) as the B operand of Sᵀ = Kᵀ·Q: lane (r,h) holds Q[c = 16s + 8h + e][q = 32w + r]
#pragma unroll
    for (int s = 0; s < kD / 16; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int cr = 16 * s + 8 * (g >> 1) + 4 * e + tq;
        const int col = 32 * w + 16 * (g & 1) + 4 * tp;
        const half4 t = tr_read(smem + cr * kQRow + ((col * 2) ^ ((cr & 3) << 6)));
        if (e == 0) qf[s].lo = t; else qf[s].hi = t;
      }
      qf[s] = scale8(qf[s], c2);
    }
    __syncthreads();  // every wave has its fragments before the K ring overwrites the image
  }
  u32x4 stg[kCPT];
  load(stg, krs, koff, d, kt0);
  store(0, kwo, stg);
  load(stg, vrs, voff, vd, kt0);
  store(0, vwo, stg);
  __syncthreads();

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
  const int qo = (POL == 2) ? seq_order(a.rule.q, a.rule, min(qi, nq - 1)) : 0;  // this lane's query order
  // tile class for this wave: 0 no allowed pair (skipped), 1 mixed (masked), 2 all allowed
  auto tcls = [&](int it) -> int __attribute__((always_inline)) {
    const int k0 = kt0 + it * kBN, k1 = k0 + kBN - 1;
    if (POL == 0) return (k1 < nk) ? 2 : 1;
    if (POL == 2) {  // (class 2 only for tiles wholly inside nk: the staged tail past nk is masked)
      if (!wave_active || k0 >= nk) return 0;
      const int c = tile_class(a.rule, wq0, min(wq0 + 31, nq - 1), k0, min(k1, nk - 1));
      return (c == 2 && k1 >= nk) ? 1 : c;
    }
    if (!wave_active || wlo_min > k1 || whi_max < k0) return 0;
    return (wlo_max <= k0 && whi_min >= k1 && k1 < nk) ? 2 : 1;
  };

  // fragment read bases (lane constants): K transposed reads with the key permutation σ
  // (register i of Sᵀ half t holds key 32t + 16(i>>3) + 8h + (i&7)); V chunk 2s+h of row 32u + r
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  uint32_t kbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    kbase[t] = (8 * (g >> 1) + tq) * 128 + (((32 * t + 16 * (g & 1) + 4 * sig) * 2) ^ ((tq & 2) << 5));
  uint32_t vbase[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) vbase[s] = kOffV + r * 128 + 16 * ((2 * s + h) ^ ((r >> 1) & 7));

  floatx16 st[2];     // Sᵀ of the tile (relative to 0 out of the MFMA)
  uint32_t pw[4][4];  // P (fp16 pairs), dword x of PV k-step s
  floatx16 o[kD / 32];  // Oᵀ: channels 32u + 8(i>>2) + 4h + (i&3)
#pragma unroll
  for (int u = 0; u < kD / 32; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[u][i] = 0.f;
  float m_run = 0.f, l0 = 0.f, l1 = 0.f, m_max = kNegInf, thr = -__FLT_MAX__;

  auto mask = [&](int k0) __attribute__((always_inline)) {
    const int lim = nk - k0 - 8 * h;    // POL 0: offset o is in range iff o < lim
    const int base = k0 + 8 * h - klo;  // POL 1: allowed iff base + o in [0, kspan)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = 32 * t + 16 * (i >> 3) + (i & 7);
        const int kk = k0 + 8 * h + off;
        const bool ok = (POL == 1)   ? ((unsigned)(base + off) < (unsigned)kspan)
                        : (POL == 2) ? (off < lim && check_orders_bf(a.rule, qo, seq_order(a.rule.k, a.rule, min(kk, nk - 1))))
                                     : (off < lim);
        st[t][i] = ok ? st[t][i] : kNegInf;
      }
  };
  auto exp_cvt = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = __builtin_amdgcn_exp2f(st[s >> 1][8 * (s & 1) + j]);
#pragma unroll
      for (int x = 0; x < 4; ++x) pw[s][x] = __builtin_bit_cast(uint32_t, half2v{(_Float16)e[2 * x], (_Float16)e[2 * x + 1]});
    }
  };
  auto softmax = [&](int it, int cls) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      st[0][i] -= m_run;
      st[1][i] -= m_run;
    }
    if (cls == 1) mask(kt0 + it * kBN);
    float mx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(st[j >> 1][8 * (j & 1)], st[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
    for (int i = 2; i < 8; i += 2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        mx[j] = fmaxf(fmaxf(mx[j], st[j >> 1][8 * (j & 1) + i]), st[j >> 1][8 * (j & 1) + i + 1]);
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
        for (int u = 0; u < kD / 32; ++u) o[u][i] *= alpha;
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

  // Sᵀ(i) from K slot c: 16 k-steps x 2 key halves, the fragments read as the MFMAs go
  auto qk = [&](int c) __attribute__((always_inline)) {
    const lds_char_t* p = smem + c * kTile;
    const floatx16 zero = {};
#pragma unroll
    for (int s = 0; s < kD / 16; ++s) {
      half8 kf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kf[t].lo = tr_read(p + kbase[t] + (16 * s) * 128);
        kf[t].hi = tr_read(p + kbase[t] + (16 * s + 4) * 128);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[t], qf[s], s == 0 ? zero : st[t], 0, 0, 0);
    }
  };
  // Oᵀ += V(i)·P(i)ᵀ from V slot c: 8 blocks of 32 channels x 4 key k-steps
  auto pv = [&](int c) __attribute__((always_inline)) {
    const lds_char_t* p = smem + c * kTile;
#pragma unroll
    for (int u = 0; u < kD / 32; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const half8 vf = read_b128(p + vbase[s] + (32 * u) * 128);
        const half8 pp = __builtin_bit_cast(half8, u32x4{pw[s][0], pw[s][1], pw[s][2], pw[s][3]});
        o[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pp, o[u], 0, 0, 0);
      }
  };

  // tile i in slot i & 1; K(i+1) / V(i+1) staged into slot (i+1) & 1, whose tile i-1 every wave
  // finished before the barrier that ended iteration i-1.  Whole pairs of iterations keep the slot
  // indices compile-time; the one past the last tile only moves zeros.
  auto iter = [&](auto C_, int it) __attribute__((always_inline)) {
    constexpr int c = decltype(C_)::value;
    const int cls = (it < ntiles) ? tcls(it) : 0;
    load(stg, krs, koff, d, kt0 + (it + 1) * kBN);
    if (cls != 0) qk(c);
    store((c ^ 1) * kTile, kwo, stg);
    load(stg, vrs, voff, vd, kt0 + (it + 1) * kBN);
    if (cls != 0) {
      softmax(it, cls);
      pv(c);
    }
    store((c ^ 1) * kTile, vwo, stg);
    __syncthreads();
  };
  for (int it = 0; it < ntiles; it += 2) {
    iter(IC<0>{}, it);
    iter(IC<1>{}, it + 1);
  }

  // ---- epilogue
  if (!wave_active) return;
  const float l_tot = sum_pair32(l0 + l1);
  const float inv = (l_tot > 0.f) ? 1.f / l_tot : 0.f;
  if (qi >= nq) return;
  __half* O = static_cast<__half*>(a.O) + bi * (int64_t)vd * nq;
  if (vd == kD) {
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(O, 2u * vd * nq);
    const uint32_t vlane = 2u * ((uint32_t)(4 * h) * (uint32_t)nq + (uint32_t)qi);
#pragma unroll
    for (int u = 0; u < kD / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t cst = 32u * u + (i & 3) + 8u * (i >> 2);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)(o[u][i] * inv)), ors, vlane,
                                              2u * cst * (uint32_t)nq, 0);
      }
  } else {
#pragma unroll
    for (int u = 0; u < kD / 32; ++u)
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

bool fwd_f16_wide_supported(const FwdArgs& a) {
  const int nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  // (32-bit buffer offsets: a slice's rows stay below 2^31 bytes, the element-wise gather included)
  return dm > 128 && dm <= kD && nk > 0 && (int64_t)dm * (nk + 8) * 2 < (1ll << 31) &&
         (int64_t)dm * a.rule.q.n * 2 < (1ll << 31) && a.b * ((a.rule.q.n + kBM - 1) / kBM) < (1ll << 31);
}

hipError_t launch_fwd_f16_wide(const FwdArgs& a, hipStream_t s) {
  const int64_t nqb = (a.rule.q.n + kBM - 1) / kBM;
  const bool aln = (a.rule.k.n % 8 == 0) && (reinterpret_cast<uintptr_t>(a.K) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(a.V) % 16 == 0);
  const int pol = a.rule.policy == 0 ? 0 : rule_is_interval(a.rule) ? 1 : 2;
  auto kern = aln ? (pol == 0 ? fwd_f16_wide_kernel<0, true> : pol == 1 ? fwd_f16_wide_kernel<1, true> : fwd_f16_wide_kernel<2, true>)
                  : (pol == 0 ? fwd_f16_wide_kernel<0, false> : pol == 1 ? fwd_f16_wide_kernel<1, false> : fwd_f16_wide_kernel<2, false>);
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nqb)), dim3(kNW * 64), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
