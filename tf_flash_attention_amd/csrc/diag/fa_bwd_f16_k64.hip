// fa_bwd_f16_k64.hip — the fp16 dK / dV pass at D = 128 with 64 keys a wave (round 6, VERDICT r5 item 2;
// diagnostic library: FA_BWD_VARIANT=1700 runs it with the shipped dQ pass).
//
// One workgroup = 4 waves, one per SIMD, 256 keys of one (batch, head) slice; a wave owns 64 keys as two
// 32-key halves and keeps dKᵀ and dVᵀ of all 64 keys in the 256 accumulator registers (asm MFMAs with
// AGPR accumulators).  Each 32-query tile (Q, dO, -lse2, -D) streams through a 2-slot LDS ring and every
// fragment read of it feeds both halves:
//     S_h  = Qᵀ·K'_h  (C = -lse2)   P_h  = exp2(S_h)           (K'_h = K·scale·log2e resident, 64 VGPRs)
//     dP_h = dOᵀ·V_h  (C = -D)      dS_h = P_h∘dP_h            (V_h read from the block's LDS image)
//     dV_h += dO·P_h,  dK_h += Q·dS_h                           (P, dS straight from the accumulators)
// so a tile's Q / dO bytes are read from LDS once per 64 keys where the producer / consumer pass reads
// them once per 32 (its LDS side was as busy as its matrix pipe).  64 MFMAs a wave a
// step against 32 transposed reads of Q / dO, 32 of V and 16 row reads.
// Shapes: max(d, v_d) in (64, 128], 16-B aligned tensors, nq % 8 == nk % 8 == 0, full and interval rules.
// Replaces the key-outer half of the reference's BackwardImpl (flash_attention.cu:1079-1967).
#include "../fa_device.h"
#include "../fa_kernels.h"
#include "../fa_mfma.h"

namespace fa {
namespace {

using namespace mf;

constexpr int kD = 128;
constexpr int kNW = 4;
constexpr int kThr = kNW * 64;
constexpr int kBK = 64 * kNW;               // keys per workgroup
constexpr int kRow = kD * kBK * 2;          // a K or V row image [128][256] fp16, 64 KB
constexpr int kQT = kD * 64;                // one [128][32] tile image
constexpr int kOffQT = 0, kOffOT = kQT, kOffLse = 2 * kQT;
constexpr int kSlot = kOffLse + 2 * 32 * 4;  // + lse2[32], D[32]
constexpr int kOffV = kRow;                  // V image (stays); the ring aliases the prologue's K image
constexpr int kSmem = 2 * kRow;
constexpr int kQChunks = kD * 4;             // 16-B chunks of one [128][32] tile
constexpr int kCPT = 2 * kQChunks / kThr;    // Q and dO chunks a thread (4)
static_assert(2 * kSlot <= kRow, "the ring fits in the K image");

// "Q16 image" [D][32] fp16 (fa_bwd_f16_fast.hip): 16-B units XOR-swizzled by (row >> 2) & 3
__device__ __forceinline__ uint32_t q16o(int row, int u, int half8 = 0) {
  return row * 64 + 16 * (u ^ ((row >> 2) & 3)) + 8 * half8;
}

#define K64_MFMA_A "v_mfma_f32_32x32x16_f16 %0, %1, %2, %0"

// timing ablations (FA_BWD_VARIANT=1700+bits, outputs WRONG): 1 no V reads (the K' fragments stand in),
// 2 no softmax (P, dS = the accumulators converted), 4 no dV / dK MFMAs, 8 no staging, 16 no S / dP MFMAs
constexpr int kANoV = 1, kANoSm = 2, kANoDvdk = 4, kANoStage = 8, kANoSdp = 16;

template <int POL, int ABL = 0>
__global__ __launch_bounds__(kThr, 1) void bwd_dkdv_k64_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char_t* smem = (lds_char_t*)smem_raw;

  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const uint32_t nkb = (nk + kBK - 1) / kBK;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t bi = bid / nkb;
  const int k0 = (int)(bid % nkb) * kBK;  // earliest (heaviest under causal) key blocks first
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int sig = ((tp & 1) << 1) | (tp >> 1);
  const float c2 = (float)a.scale * kLog2e;

  const int d = a.d, vd = a.v_d;
  const __half* K = static_cast<const __half*>(a.K) + bi * (int64_t)d * nk;
  const __half* V = static_cast<const __half*>(a.V) + bi * (int64_t)vd * nk;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(static_cast<const __half*>(a.Q) + bi * (int64_t)d * nq, 2u * d * nq);
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(static_cast<const __half*>(a.dO) + bi * (int64_t)vd * nq, 2u * vd * nq);
  const float* glse = static_cast<const float*>(a.ws_lse) + bi * (int64_t)nq;
  const float* gD = static_cast<const float*>(a.ws_D) + bi * (int64_t)nq;

  // ---- K and V row images [128][256] (64-B blocks XOR-swizzled by (row & 3)); K' resident
  // lane (r, h) of half hh holds K'[c = 16s + 8h + j][key = k0 + 64w + 32hh + r]
  half8 kb[2][kD / 16];
  auto img_off = [&](int hh, int s, int e) -> uint32_t {
    const int crow = 16 * s + 8 * (g >> 1) + 4 * e + tq;
    const int col = 64 * w + 32 * hh + 16 * (g & 1) + 4 * tp;
    return crow * (2 * kBK) + ((col * 2) ^ ((crow & 3) << 6));
  };
  {
    constexpr int kHalf = kD * (kBK / 8) / kThr;  // 16 chunks a thread per tensor
    const __amdgpu_buffer_rsrc_t krs = make_rsrc(K, 2u * d * nk), vrs = make_rsrc(V, 2u * vd * nk);
#pragma unroll
    for (int which = 0; which < 2; ++which) {  // (one tensor at a time: 16 chunks in flight, not 32)
      u32x4 rv[kHalf];
#pragma unroll
      for (int jj = 0; jj < kHalf; ++jj) {
        const int j = tid + kThr * jj, c = j / (kBK / 8), m = j % (kBK / 8);
        const bool in = c < (which ? vd : d) && k0 + 8 * m < nk;
        rv[jj] = __builtin_amdgcn_raw_buffer_load_b128(which ? vrs : krs, in ? (uint32_t)c * (uint32_t)nk * 2u + 16u * m : 0x80000000u,
                                                       2 * k0, 0);
      }
#pragma unroll
      for (int jj = 0; jj < kHalf; ++jj) {
        const int j = tid + kThr * jj, c = j / (kBK / 8), m = j % (kBK / 8);
        *reinterpret_cast<lds_u32x4_t*>(smem + which * kRow + c * (2 * kBK) + ((m * 16) ^ ((c & 3) << 6))) = rv[jj];
      }
    }
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int s = 0; s < kD / 16; ++s) {
        kb[hh][s].lo = tr_read(smem + img_off(hh, s, 0));
        kb[hh][s].hi = tr_read(smem + img_off(hh, s, 1));
        kb[hh][s] = scale8(kb[hh][s], c2);  // S in log2 units straight out of the MFMA
      }
    __syncthreads();  // the ring reuses the K image
  }

  // ---- query range of the block; per-half query intervals (POL 1)
  const int klast = min(k0 + kBK, nk) - 1;
  int qb = 0, qe = nq;
  if (POL != 0) q_range_for_k_block(a.rule, k0, klast, &qb, &qe);
  const int qt0 = (qb / 32) * 32;
  const int ntiles = (qe > qb) ? (qe - qt0 + 31) / 32 : 0;
  int qlo[2] = {0, 0}, qspan[2] = {nq, nq};
  int wlo_min[2] = {0, 0}, wlo_max[2] = {0, 0}, whi_min[2] = {nq - 1, nq - 1}, whi_max[2] = {nq - 1, nq - 1};
  bool hact[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int hk0 = k0 + 64 * w + 32 * hh, key = hk0 + r;
    hact[hh] = hk0 < nk;
    if (POL == 1 && hact[hh]) {
      int qhi;
      query_interval(a.rule, min(key, nk - 1), &qlo[hh], &qhi);
      qspan[hh] = max(qhi - qlo[hh] + 1, 0);
      const int last = min(31, nk - 1 - hk0);
      wlo_min[hh] = __builtin_amdgcn_readfirstlane(qlo[hh]);
      whi_min[hh] = __builtin_amdgcn_readfirstlane(qhi);
      wlo_max[hh] = __builtin_amdgcn_readlane(qlo[hh], last);
      whi_max[hh] = __builtin_amdgcn_readlane(qhi, last);
    }
  }
  // 0: no allowed pair for the half, 1: mixed (per-element mask), 2: all allowed
  auto tcls = [&](int hh, int qa) -> int {
    const int qz = qa + 31;
    if (!hact[hh]) return 0;
    if (POL == 0) return 2;  // q >= nq rows carry -lse2 = -inf -> P = 0; keys >= nk are never stored
    if (wlo_min[hh] > qz || whi_max[hh] < qa) return 0;
    return (wlo_max[hh] <= qa && whi_min[hh] >= qz) ? 2 : 1;
  };

  // ---- query-tile staging: chunk j = 8 queries of one channel row of Q (j < 2) or dO (j >= 2)
  uint32_t voff[kCPT];
  int crow_[kCPT], cm_[kCPT];
#pragma unroll
  for (int j = 0; j < kCPT; ++j) {
    const int idx = (tid + kThr * j) % kQChunks;
    crow_[j] = idx >> 2;
    cm_[j] = idx & 3;
    voff[j] = (uint32_t)crow_[j] * (uint32_t)nq * 2u + 16u * cm_[j];
  }
  u32x4 qr[kCPT];
  float lr = 0.f;
  auto load_tile = [&](int qa) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = j >= kCPT / 2;
      const bool out = qa + 8 * cm_[j] >= nq || crow_[j] >= (isO ? vd : d);
      qr[j] = buf_load16(isO ? ors : qrs, voff[j], 2 * qa, out);
    }
    if (w == 0) {  // lanes 0..31: -lse2, 32..63: -D (clamped load, select past nq)
      const int q = qa + (lane & 31);
      const float v = (lane < 32 ? glse : gD)[min(q, nq - 1)];
      lr = (q < nq) ? v : ((lane < 32) ? -__builtin_huge_valf() : 0.f);
    }
  };
  auto store_tile = [&](int slot) __attribute__((always_inline)) {
    lds_char_t* base = smem + slot * kSlot;
#pragma unroll
    for (int j = 0; j < kCPT; ++j) {
      const bool isO = j >= kCPT / 2;
      *reinterpret_cast<lds_u32x4_t*>(base + (isO ? kOffOT : kOffQT) + q16o(crow_[j], cm_[j])) = qr[j];
    }
    if (w == 0) reinterpret_cast<lds_f_t*>(base + kOffLse)[lane] = lr;
  };

  // dVᵀ / dKᵀ of the wave's 64 keys: [half][channel block u] (AGPRs, asm MFMAs)
  floatx16 dv[2][kD / 32], dk[2][kD / 32];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int u = 0; u < kD / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) { dv[hh][u][i] = 0.f; dk[hh][u][i] = 0.f; }
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int u = 0; u < kD / 32; ++u) asm volatile("" : "+a"(dv[hh][u]), "+a"(dk[hh][u]));

  // P = exp2(S), dS = P∘dP of one half; k-step s of the dV / dK products = registers 8s..8s+7
  auto softmax_m = [&](int hh, const floatx16& sacc, const floatx16& pacc, int qa, bool masked, half8 (&pf)[2],
                       half8 (&sf)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float pv = __builtin_amdgcn_exp2f(sacc[i]);
      if (POL == 1 && masked) {
        const int q = qa + 16 * (i >> 3) + 8 * h + (i & 7);
        pv = ((unsigned)(q - qlo[hh]) < (unsigned)qspan[hh]) ? pv : 0.f;
      }
      pf[i >> 3][i & 7] = (_Float16)pv;
      sf[i >> 3][i & 7] = (_Float16)(pv * pacc[i]);
    }
  };
  auto softmax = [&](int hh, const floatx16& sacc, const floatx16& pacc, int qa, int cls, half8 (&pf)[2], half8 (&sf)[2])
      __attribute__((always_inline)) {
    if constexpr (POL == 0) {
      softmax_m(hh, sacc, pacc, qa, false, pf, sf);
    } else if (cls != 2) {
      asm volatile("; edge tile" ::: );
      softmax_m(hh, sacc, pacc, qa, true, pf, sf);
    } else {
      asm volatile("; interior tile" ::: );
      softmax_m(hh, sacc, pacc, qa, false, pf, sf);
    }
  };

  load_tile(qt0);
  store_tile(0);
  load_tile(qt0 + 32);

  // step it: tile it in slot it&1 (complete after the barrier); tile it+1 -> slot (it+1)&1 from the
  // staging registers, which then take tile it+2
  auto step = [&](auto P_, int it) __attribute__((always_inline)) {
    constexpr int p = decltype(P_)::value;
    (void)dv; (void)dk;  // (asm operands alone do not capture them in a generic lambda)
    __syncthreads();
    const int qa = qt0 + 32 * it;
    if constexpr ((ABL & kANoStage) == 0) {
      store_tile(p ^ 1);
      load_tile(qa + 64);
    }
    const int cls0 = it < ntiles ? tcls(0, qa) : 0, cls1 = it < ntiles ? tcls(1, qa) : 0;
    if (cls0 == 0 && cls1 == 0) return;
    const lds_char_t* base = smem + p * kSlot;
    // row constants (stored negated) as the initial accumulators of both halves
    floatx16 linit, dinit;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {  // registers 4gq..4gq+3 = queries 16(gq>>1) + 8h + 4(gq&1) + 0..3
      const int q4 = 16 * (gq >> 1) + 8 * h + 4 * (gq & 1);
      const floatx4 l4 = *reinterpret_cast<const lds_f4_t*>(base + kOffLse + 4 * q4);
      const floatx4 d4 = *reinterpret_cast<const lds_f4_t*>(base + kOffLse + 128 + 4 * q4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        linit[4 * gq + j] = l4[j];
        dinit[4 * gq + j] = d4[j];
      }
    }
    // S_h = Qᵀ·K'_h, dP_h = dOᵀ·V_h: the Q / dO A operands (transposed reads, σ-permuted columns) once
    // per k-step for both halves; V_h from the block's image
    floatx16 sacc[2], pacc[2];
#pragma unroll
    for (int s = 0; s < kD / 16; ++s) {
      half8 qa8, oa8, vb8[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint32_t off = q16o(16 * s + 8 * (g >> 1) + 4 * e + tq, 2 * (g & 1) + (sig >> 1), sig & 1);
        const half4 x = tr_read(base + kOffQT + off), y = tr_read(base + kOffOT + off);
        if (e == 0) { qa8.lo = x; oa8.lo = y; } else { qa8.hi = x; oa8.hi = y; }
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if constexpr ((ABL & kANoV) != 0) {
          vb8[hh] = kb[hh][s];
        } else {
          vb8[hh].lo = tr_read(smem + kOffV + img_off(hh, s, 0));
          vb8[hh].hi = tr_read(smem + kOffV + img_off(hh, s, 1));
        }
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if constexpr ((ABL & kANoSdp) != 0) {
          if (s == 0) { sacc[hh] = linit; pacc[hh] = dinit; }
          asm volatile("" : "+v"(sacc[hh]), "+v"(pacc[hh]) : "v"(qa8), "v"(oa8), "v"(vb8[hh]), "v"(kb[hh][s]));
        } else {
          sacc[hh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(qa8, kb[hh][s], s == 0 ? linit : sacc[hh], 0, 0, 0);
          pacc[hh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(oa8, vb8[hh], s == 0 ? dinit : pacc[hh], 0, 0, 0);
        }
      }
    }
    half8 pf[2][2], sf[2][2];
    if constexpr ((ABL & kANoSm) != 0) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          pf[hh][i >> 3][i & 7] = (_Float16)sacc[hh][i];
          sf[hh][i >> 3][i & 7] = (_Float16)pacc[hh][i];
        }
    } else {
      softmax(0, sacc[0], pacc[0], qa, cls0, pf[0], sf[0]);
      softmax(1, sacc[1], pacc[1], qa, cls1, pf[1], sf[1]);
    }
    asm volatile("s_nop 2" ::: );  // (VALU writes of P / dS, then the asm MFMAs that read them)
    // dV_h += dO·P_h, dK_h += Q·dS_h: A = X[row 32u + r][queries 16s + 8h + 0..7] (b128 row reads)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int u = 0; u < kD / 32; ++u) {
        const half8 oa = read_b128(base + kOffOT + q16o(32 * u + r, 2 * s + h));
        const half8 qa_ = read_b128(base + kOffQT + q16o(32 * u + r, 2 * s + h));
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if constexpr ((ABL & kANoDvdk) != 0) {
            asm volatile("" ::"v"(oa), "v"(pf[hh][s]), "v"(qa_), "v"(sf[hh][s]));
          } else {
            asm volatile(K64_MFMA_A : "+a"(dv[hh][u]) : "v"(oa), "v"(pf[hh][s]));
            asm volatile(K64_MFMA_A : "+a"(dk[hh][u]) : "v"(qa_), "v"(sf[hh][s]));
          }
        }
      }
  };
  for (int it = 0; it < ntiles; it += 2) {
    step(IC<0>{}, it);
    step(IC<1>{}, it + 1);
  }
  // (the accumulators are read below: let the last asm MFMAs finish)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  // ---- dK = scale·Σ dS·Q, dV: rows c = 32u + (i&3) + 8(i>>2) + 4h, column = the lane's key
  __half* dK = static_cast<__half*>(a.dK) + bi * (int64_t)d * nk;
  __half* dV = static_cast<__half*>(a.dV) + bi * (int64_t)vd * nk;
  const float sc = (float)a.scale;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int key = k0 + 64 * w + 32 * hh + r;
    if (key >= nk) continue;
#pragma unroll
    for (int u = 0; u < kD / 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (c < d) dK[(int64_t)c * nk + key] = __float2half(dk[hh][u][i] * sc);
        if (c < vd) dV[(int64_t)c * nk + key] = __float2half(dv[hh][u][i]);
      }
  }
}

}  // namespace

bool bwd_dkdv_k64_supported(const BwdArgs& a) {
  const int nq = a.rule.q.n, nk = a.rule.k.n;
  const int dm = max(a.d, a.v_d);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return dm > 64 && dm <= kD && (a.rule.policy == 0 || rule_is_interval(a.rule)) && nq % 8 == 0 && nk % 8 == 0 &&
         al16(a.Q) && al16(a.K) && al16(a.V) && al16(a.dO) && (int64_t)dm * (nq + 8) * 2 < (1ll << 31) &&
         (int64_t)dm * (nk + 8) * 2 < (1ll << 31) && a.b * ((nk + kBK - 1) / kBK) < (1ll << 31);
}

hipError_t launch_dkdv_k64(const BwdArgs& a, hipStream_t s) {
  const int64_t nkb = (a.rule.k.n + kBK - 1) / kBK;
  auto kern = a.rule.policy == 0 ? bwd_dkdv_k64_kernel<0> : bwd_dkdv_k64_kernel<1>;
  if (a.rule.policy != 0) {  // timing ablations (diagnostic library, causal / interval rules; outputs wrong)
    switch (diag_variant("FA_BWD_VARIANT") - 1700) {
      case 1: kern = bwd_dkdv_k64_kernel<1, 1>; break;
      case 2: kern = bwd_dkdv_k64_kernel<1, 2>; break;
      case 4: kern = bwd_dkdv_k64_kernel<1, 4>; break;
      case 8: kern = bwd_dkdv_k64_kernel<1, 8>; break;
      case 16: kern = bwd_dkdv_k64_kernel<1, 16>; break;
      case 20: kern = bwd_dkdv_k64_kernel<1, 20>; break;
      case 11: kern = bwd_dkdv_k64_kernel<1, 11>; break;
      default: break;
    }
  }
  hipError_t e = set_smem_once(reinterpret_cast<const void*>(kern), kSmem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.b * nkb)), dim3(kThr), kSmem, s, a);
  return hipGetLastError();
}

}  // namespace fa
