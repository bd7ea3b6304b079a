// fa_rules.h — sync maps and masking rules, evaluated arithmetically on host
// and device (no mask tensor ever touches HBM).
//
// Restates, clean-room:
//   * sync methods  — /root/reference/flash_attention/kernel/sync_methods.cc:8-117
//     and the CuTe order map of sync_methods.h:56-85;
//   * policies      — flash_attention.h:45-149 (Full / Causal / Local).
//
// Index conventions (same as the reference): a sequence of rank S is stored
// row-major, flattened to n = prod(shape).  Dimension 0 of the rule is the
// LAST tensor axis (the reference pushes dims last-axis-first,
// sync_methods.cc:12-13).  For flat index x:
//     1d:  c0 = o0 + s0*x
//     2d:  c0 = o0 + s0*(x % W),  c1 = o1 + s1*(x / W)        (W = last-axis extent)
//     order = c0 + (c1 << log2R0)                                (R_i pow-2 >= max extent)
// Orders are monotone increasing in x for both Q and K, which is what makes
// index-range bounds (binary search on the order) exact.
#ifndef TF_FLASH_ATTENTION_AMD_FA_RULES_H_
#define TF_FLASH_ATTENTION_AMD_FA_RULES_H_

#include <stdint.h>

#if defined(__HIPCC__)
#define FA_HD __host__ __device__ __forceinline__
#else
#define FA_HD inline
#endif

namespace fa {

struct SeqMap {
  int32_t n;        // flattened extent
  int32_t w;        // last-axis extent (2d), n for 1d
  int32_t s0, o0;   // last axis stride / offset
  int32_t s1, o1;   // first axis stride / offset (2d)
};

struct Rule {
  int32_t policy;      // 0 full, 1 causal, 2 local
  int32_t seq_dims;    // 1 | 2
  int32_t log2R0, log2R1;
  int32_t R0, R1;
  int32_t ws;          // window_size
  int32_t ls;          // log2_stride_size
  int32_t sws;         // ws << ls (strided window size)
  int32_t look_ahead;  // 1 if causal-local, else sws (flash_attention.h:91-95)
  SeqMap q, k;
};

FA_HD int32_t seq_order(const SeqMap& m, const Rule& r, int32_t x) {
  if (r.seq_dims == 1) return m.o0 + m.s0 * x;
  const int32_t y = x / m.w;
  const int32_t xx = x - y * m.w;
  return (m.o0 + m.s0 * xx) + ((m.o1 + m.s1 * y) << r.log2R0);
}

FA_HD int32_t iabs32(int32_t v) { return v < 0 ? -v : v; }

// Per-pair rule on orders (flash_attention.h:57-60, 76-79, 119-140).
FA_HD bool check_orders(const Rule& r, int32_t qo, int32_t ko) {
  if (r.policy == 0) return true;
  if (r.policy == 1) return qo >= ko;
  if (r.look_ahead == 1 && qo < ko) return false;
  const int32_t rem = (1 << r.ls) - 1;
  // dim 0 (last axis)
  int32_t d0 = iabs32((qo & (r.R0 - 1)) - (ko & (r.R0 - 1)));
  if ((d0 & rem) != 0 || (d0 >> r.ls) >= r.ws) return false;
  if (r.seq_dims == 2) {
    int32_t d1 = iabs32(((qo >> r.log2R0) & (r.R1 - 1)) - ((ko >> r.log2R0) & (r.R1 - 1)));
    if ((d1 & rem) != 0 || (d1 >> r.ls) >= r.ws) return false;
  }
  return true;
}

// Branch-free form of check_orders for per-element use inside kernels (every
// condition evaluated, combined with bitwise &; compiles to v_cndmask, not
// exec-mask branches).  Same result as check_orders for policy 1 and 2.
FA_HD bool check_orders_bf(const Rule& r, int32_t qo, int32_t ko) {
  if (r.policy == 1) return qo >= ko;  // wave-uniform branch
  const int32_t rem = (1 << r.ls) - 1;
  const int32_t d0 = iabs32((qo & (r.R0 - 1)) - (ko & (r.R0 - 1)));
  const int32_t d1 = iabs32(((qo >> r.log2R0) & (r.R1 - 1)) - ((ko >> r.log2R0) & (r.R1 - 1)));
  bool ok = ((d0 & rem) == 0) & ((d0 >> r.ls) < r.ws);
  ok &= (r.seq_dims == 1) | (((d1 & rem) == 0) & ((d1 >> r.ls) < r.ws));
  ok &= (r.look_ahead != 1) | (qo >= ko);
  return ok;
}

FA_HD int32_t imin32(int32_t a, int32_t b) { return a < b ? a : b; }
FA_HD int32_t imax32(int32_t a, int32_t b) { return a > b ? a : b; }
// a + b for a >= 0, b >= 0, saturated at INT32_MAX (orders are < 2^30, windows up to INT32_MAX)
FA_HD int32_t sat_add32(int32_t a, int32_t b) {
  const int64_t s = (int64_t)a + (int64_t)b;
  return s > 0x7fffffff ? 0x7fffffff : (int32_t)s;
}

// Window bounding box in ORDER space for a block of partners whose orders span
// [omin, omax] (LocalAttentionPolicy::IsSkipped, flash_attention.h:100-115).
// `lo_reach`/`hi_reach` are how far (in coordinates) a partner may sit
// below/above.  Returns an order interval [*lo, *hi] containing every order
// that can pair with the block.
FA_HD void local_order_bounds(const Rule& r, int32_t omin, int32_t omax,
                              int32_t lo_reach, int32_t hi_reach,
                              int32_t* lo, int32_t* hi) {
  // a reach past the grid extent R clamps like R itself; clamping first keeps c + reach inside
  // int32 for windows up to INT32_MAX (validated: ws << ls <= INT32_MAX)
  const int32_t lr0 = imin32(lo_reach, r.R0), hr0 = imin32(hi_reach, r.R0);
  const int32_t lr1 = imin32(lo_reach, r.R1), hr1 = imin32(hi_reach, r.R1);
  const int32_t c0min = omin & (r.R0 - 1), c0max = omax & (r.R0 - 1);
  int32_t l0 = imax32(c0min - lr0, 0);
  int32_t h0 = imin32(c0max + hr0, r.R0 - 1);
  if (r.seq_dims == 1) {
    *lo = l0; *hi = h0; return;
  }
  const int32_t c1min = (omin >> r.log2R0) & (r.R1 - 1), c1max = (omax >> r.log2R0) & (r.R1 - 1);
  const int32_t l1 = imax32(c1min - lr1, 0);
  const int32_t h1 = imin32(c1max + hr1, r.R1 - 1);
  // When the row bound is clamped at the grid edge, partners of EARLIER/LATER
  // block rows can reach any column of the clamped row: widen dim 0 there.
  // (The reference's IsSkipped keeps the unclamped column bound and can skip
  // a tile holding allowed pairs in that corner case; the vanilla test oracle
  // — our parity target — attends them.)
  if (c1min - lr1 < 0) l0 = 0;
  if (c1max + hr1 > r.R1 - 1) h0 = r.R0 - 1;
  *lo = l0 + (l1 << r.log2R0);
  *hi = h0 + (h1 << r.log2R0);
}

// First index x in [0, n) with order(x) >= target (n if none).
FA_HD int32_t lower_bound_order(const SeqMap& m, const Rule& r, int32_t target) {
  int32_t lo = 0, hi = m.n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (seq_order(m, r, mid) < target) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Range [*kb, *ke) of K indices that may pair with Q indices [q0, q1] (inclusive, valid).
FA_HD void k_range_for_q_block(const Rule& r, int32_t q0, int32_t q1, int32_t* kb, int32_t* ke) {
  const int32_t nk = r.k.n;
  if (r.policy == 0) { *kb = 0; *ke = nk; return; }
  const int32_t qo_min = seq_order(r.q, r, q0), qo_max = seq_order(r.q, r, q1);
  int32_t olo = 0, ohi = qo_max;  // causal: k order <= max q order
  if (r.policy == 2) {
    // k coords in [cq - (sws-1), cq + (look_ahead-1)]
    local_order_bounds(r, qo_min, qo_max, r.sws - 1, r.look_ahead - 1, &olo, &ohi);
    if (r.look_ahead == 1) ohi = imin32(ohi, qo_max);
  }
  *kb = lower_bound_order(r.k, r, olo);
  *ke = lower_bound_order(r.k, r, ohi + 1);
  if (*ke < *kb) *ke = *kb;
}

// Range [*qb, *qe) of Q indices that may pair with K indices [k0, k1].
FA_HD void q_range_for_k_block(const Rule& r, int32_t k0, int32_t k1, int32_t* qb, int32_t* qe) {
  const int32_t nq = r.q.n;
  if (r.policy == 0) { *qb = 0; *qe = nq; return; }
  const int32_t ko_min = seq_order(r.k, r, k0), ko_max = seq_order(r.k, r, k1);
  int32_t olo = ko_min, ohi = 0x7fffffff;  // causal: q order >= min k order
  if (r.policy == 2) {
    // q coords in [ck - (look_ahead-1), ck + (sws-1)]
    local_order_bounds(r, ko_min, ko_max, r.look_ahead - 1, r.sws - 1, &olo, &ohi);
    if (r.look_ahead == 1) olo = imax32(olo, ko_min);
  }
  *qb = lower_bound_order(r.q, r, olo);
  *qe = (ohi == 0x7fffffff) ? nq : lower_bound_order(r.q, r, ohi + 1);
  if (*qe < *qb) *qe = *qb;
}

// Rules under which the keys allowed for one query form a contiguous INDEX
// interval: full, causal (any dims: orders are monotone in the index), and 1d
// local with unit stride (|dq - dk| < ws, plus qo >= ko when causal).
FA_HD bool rule_is_interval(const Rule& r) {
  return r.policy != 2 || (r.seq_dims == 1 && r.ls == 0);
}

// Inclusive key-index interval [*klo, *khi] allowed for query index qi under an
// interval rule (*khi < *klo when empty).  Both bounds are non-decreasing in qi.
FA_HD void key_interval(const Rule& r, int32_t qi, int32_t* klo, int32_t* khi) {
  const int32_t nk = r.k.n;
  if (r.policy == 0) { *klo = 0; *khi = nk - 1; return; }
  const int32_t qo = seq_order(r.q, r, qi);
  int32_t ohi = qo;  // causal: ko <= qo
  *klo = 0;
  if (r.policy == 2) {  // 1d: coordinate == order; |qo - ko| <= ws - 1
    if (r.look_ahead != 1) ohi = sat_add32(qo, r.ws - 1);
    *klo = lower_bound_order(r.k, r, qo - (r.ws - 1));
  }
  *khi = lower_bound_order(r.k, r, sat_add32(ohi, 1)) - 1;
}

// Inclusive query-index interval [*qlo, *qhi] allowed for key index ki under an
// interval rule (*qhi < *qlo when empty) — the transpose of key_interval, used by
// the key-outer backward.  Both bounds are non-decreasing in ki.
FA_HD void query_interval(const Rule& r, int32_t ki, int32_t* qlo, int32_t* qhi) {
  const int32_t nq = r.q.n;
  if (r.policy == 0) { *qlo = 0; *qhi = nq - 1; return; }
  const int32_t ko = seq_order(r.k, r, ki);
  *qlo = lower_bound_order(r.q, r, ko);  // causal (and causal-local): qo >= ko
  *qhi = nq - 1;
  if (r.policy == 2) {  // 1d: |qo - ko| <= ws - 1
    if (r.look_ahead != 1) *qlo = lower_bound_order(r.q, r, ko - (r.ws - 1));
    *qhi = lower_bound_order(r.q, r, sat_add32(ko, r.ws)) - 1;
  }
}

// Tile classification for Q rows [q0, q1] x K cols [k0, k1] (all indices valid):
//   2 = every pair allowed (no per-element check needed),
//   1 = mixed (per-element check), 0 = no pair allowed.
FA_HD int tile_class(const Rule& r, int32_t q0, int32_t q1, int32_t k0, int32_t k1) {
  if (r.policy == 0) return 2;
  const int32_t qa = seq_order(r.q, r, q0), qz = seq_order(r.q, r, q1);
  const int32_t ka = seq_order(r.k, r, k0), kz = seq_order(r.k, r, k1);
  if (r.policy == 1) {
    if (kz <= qa) return 2;
    if (ka > qz) return 0;
    return 1;
  }
  if (r.look_ahead == 1 && ka > qz) return 0;
  if (r.seq_dims == 1 && r.ls == 0) {
    // 1d contiguous window: |qo - ko| < ws for all pairs
    const int32_t far = imax32(qz - ka, kz - qa);
    const bool causal_ok = (r.look_ahead != 1) || (kz <= qa);
    if (far < r.ws && causal_ok) return 2;
    // no pair: every distance >= ws
    const int32_t near = (ka > qz) ? (ka - qz) : ((qa > kz) ? (qa - kz) : 0);
    if (near >= r.ws) return 0;
  }
  return 1;
}

}  // namespace fa

#endif  // TF_FLASH_ATTENTION_AMD_FA_RULES_H_
