// fa_api.hip — C-ABI host layer (include/fa_api.h).
//
// Replaces the reference's host side: the sync-method lookup and order-map
// construction (sync_methods.{h,cc}), the per-op validation/alloc/memset in
// FlashAttention{Forward,Backward}Base::Compute (flash_attention_forward.cc:280-386,
// flash_attention_backward.cc:181-344) and the launcher
// FlashAttentionLauncher::{Forward,Backward} (flash_attention.cu:2147-2447).
// Differences by design: no memsets (kernels write every output element), no
// Br_occupancy lock array, no shared-memory opt-in dance (gfx950 exposes
// 160 KiB LDS per workgroup), and the FLOP estimate is algorithmic.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/fa_api.h"
#include "fa_device.h"
#include "fa_kernels.h"
#include "fa_rules.h"

namespace fa {

// (kernel, device) pairs whose dynamic-LDS limit is already raised.  Readers take the shared
// lock; the first launch of a kernel on a device takes the exclusive one.  Replaces the
// reference's per-launch cudaFuncSetAttribute (flash_attention.cu:2269, which sits inside an
// assert and vanishes under NDEBUG — SURVEY N7).
hipError_t set_smem_once(const void* kern, int bytes) {
  struct Entry {
    const void* kern;
    int dev, bytes;
  };
  static std::shared_mutex mu;
  static std::vector<Entry> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    std::shared_lock<std::shared_mutex> rd(mu);
    for (const Entry& x : done)
      if (x.kern == kern && x.dev == dev && x.bytes >= bytes) return hipSuccess;
  }
  std::unique_lock<std::shared_mutex> wr(mu);
  for (const Entry& x : done)
    if (x.kern == kern && x.dev == dev && x.bytes >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.push_back({kern, dev, bytes});
  return e;
}

int device_cus() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];  // 0 = not queried yet (a benign race: same value)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < kMaxDev) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int cus = 0;
  if (dev < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (dev >= 0 && dev < kMaxDev) cache[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

// XCDs the block-placement maps assume (blocks dealt round-robin over them, 32 CUs each on gfx950).
// The count is inferred from the CUs, exact only for parts built from 32-CU XCDs; any other CU count
// returns 1, which turns the XCD-aware orders into plain ones (correct for every count: the maps are
// bijections; only their L2-locality assumption needs the true count).
int device_xcds() {
  const int cus = device_cus();
  if (cus % 32 != 0) return 1;
  const int x = cus / 32;
  return x < 1 ? 1 : (x > 8 ? 8 : x);
}

}  // namespace fa

namespace {

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int32_t next_pow2(int32_t n) {
  int32_t r = 1;
  while (r < n) r <<= 1;
  return r;
}

int32_t ilog2(int32_t n) {
  int32_t l = 0;
  while ((1 << l) < n) ++l;
  return l;
}

int64_t seq_elems(const int32_t* s, int dims) {
  int64_t n = 1;
  for (int i = 0; i < dims; ++i) n *= s[i];
  return n;
}

// Sync methods, sync_methods.cc:8-111: per dim (last axis first) the reference
// extent is the next pow2 >= max(Mq, Mk); scale modes stride by max//M;
// scale_end offsets by stride-1.
void build_rule(const fa_problem* p, fa::Rule* r) {
  memset(r, 0, sizeof(*r));
  const int S = p->seq_dims;
  int32_t R[2] = {1, 1}, sq[2] = {1, 1}, sk[2] = {1, 1}, oq[2] = {0, 0}, ok[2] = {0, 0};
  for (int i = 0; i < S; ++i) {
    const int axis = S - 1 - i;
    const int32_t mq = p->q_seq[axis], mk = p->k_seq[axis];
    const int32_t mx = mq > mk ? mq : mk;
    R[i] = next_pow2(mx < 1 ? 1 : mx);
    if (p->sync_mode != FA_NONE_FRONT) {
      sq[i] = mq > 0 ? mx / mq : 1;
      sk[i] = mk > 0 ? mx / mk : 1;
    }
    if (p->sync_mode == FA_SCALE_END) {
      oq[i] = sq[i] - 1;
      ok[i] = sk[i] - 1;
    }
  }
  r->policy = p->policy;
  r->seq_dims = S;
  r->R0 = R[0];
  r->R1 = R[1];
  r->log2R0 = ilog2(R[0]);
  r->log2R1 = ilog2(R[1]);
  r->q.n = (int32_t)seq_elems(p->q_seq, S);
  r->k.n = (int32_t)seq_elems(p->k_seq, S);
  r->q.w = S == 2 ? p->q_seq[1] : r->q.n;
  r->k.w = S == 2 ? p->k_seq[1] : r->k.n;
  r->q.s0 = sq[0]; r->q.o0 = oq[0]; r->q.s1 = sq[1]; r->q.o1 = oq[1];
  r->k.s0 = sk[0]; r->k.o0 = ok[0]; r->k.s1 = sk[1]; r->k.o1 = ok[1];
  if (p->policy == FA_LOCAL) {
    r->ws = p->window_size;
    r->ls = p->log2_stride_size;
    r->sws = p->window_size << p->log2_stride_size;
    r->look_ahead = p->is_causal ? 1 : r->sws;  // flash_attention.h:91-95
  } else {
    r->ws = 1;
    r->sws = 1;
    r->look_ahead = 1;
  }
}

size_t acc_size(int dtype) { return dtype == FA_F64 ? 8 : 4; }
size_t elem_size(int dtype) { return dtype == FA_F16 ? 2 : (dtype == FA_F32 ? 4 : 8); }

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

struct WsLayout {
  size_t dq, D, lse, total;
};

WsLayout ws_layout(const fa_problem* p) {
  const int64_t nq = seq_elems(p->q_seq, p->seq_dims);
  const size_t a = acc_size(p->dtype);
  WsLayout w;
  w.dq = 0;
  w.D = align_up(a * (size_t)p->b * (size_t)p->d * (size_t)nq);
  w.lse = w.D + align_up(a * (size_t)p->b * (size_t)nq);
  w.total = w.lse + align_up(a * (size_t)p->b * (size_t)nq);
  return w;
}

}  // namespace

extern "C" {

int fa_sync_mode_from_string(const char* name) {
  if (!name) return -1;
  if (!strcmp(name, "none_front")) return FA_NONE_FRONT;
  if (!strcmp(name, "scale_front")) return FA_SCALE_FRONT;
  if (!strcmp(name, "scale_end")) return FA_SCALE_END;
  return -1;
}

int fa_validate(const fa_problem* p) {
  if (!p) return set_error(FA_ERR_INVALID_ARGUMENT, "null problem descriptor");
  if (p->dtype < FA_F16 || p->dtype > FA_F64) return set_error(FA_ERR_INVALID_ARGUMENT, "unknown dtype");
  if (p->policy < FA_FULL || p->policy > FA_LOCAL) return set_error(FA_ERR_INVALID_ARGUMENT, "unknown attention policy");
  if (p->seq_dims != 1 && p->seq_dims != 2) return set_error(FA_ERR_INVALID_ARGUMENT, "seq_dims must be 1 or 2");
  if (p->sync_mode < FA_NONE_FRONT || p->sync_mode > FA_SCALE_END)
    return set_error(FA_ERR_INVALID_ARGUMENT, "Unsupported sync_mode");
  if (p->b < 0) return set_error(FA_ERR_INVALID_ARGUMENT, "negative batch size");
  for (int i = 0; i < p->seq_dims; ++i)
    if (p->q_seq[i] < 0 || p->k_seq[i] < 0) return set_error(FA_ERR_INVALID_ARGUMENT, "negative sequence extent");
  if (p->d < 1 || p->v_d < 1) return set_error(FA_ERR_INVALID_ARGUMENT, "channel dimensions must be >= 1");
  const int64_t nq = seq_elems(p->q_seq, p->seq_dims), nk = seq_elems(p->k_seq, p->seq_dims);
  if (nq > 0x7fffffff || nk > 0x7fffffff)
    return set_error(FA_ERR_INVALID_ARGUMENT, "sequence sizes are limited to the int32 range (sync_methods.h:12-14)");
  int64_t ref = 1;
  for (int i = 0; i < p->seq_dims; ++i) {
    const int32_t mx = p->q_seq[i] > p->k_seq[i] ? p->q_seq[i] : p->k_seq[i];
    ref *= next_pow2(mx < 1 ? 1 : mx);
  }
  if (ref > (int64_t(1) << 30)) return set_error(FA_ERR_INVALID_ARGUMENT, "reference sequence extent exceeds 2^30");
  if (p->policy == FA_LOCAL) {
    if (p->window_size < 1) return set_error(FA_ERR_INVALID_ARGUMENT, "window_size must be >= 1");
    if (p->log2_stride_size < 0 || p->log2_stride_size >= 31)
      return set_error(FA_ERR_INVALID_ARGUMENT, "log2_stride_size must be in [0, 31)");
    if ((int64_t(p->window_size) << p->log2_stride_size) > 0x7fffffff)
      return set_error(FA_ERR_INVALID_ARGUMENT,
                       "stride size is too big; please make sure the stride size/window size is within the range "
                       "representable by int32_t");
  }
  return FA_OK;
}

#ifdef FA_DIAG
// diagnostic library only: calls that reached a launch, so a test can prove which library ran them
static std::atomic<long long> g_diag_calls[2];
long long fa_diag_call_count(int which) { return (which == 0 || which == 1) ? g_diag_calls[which].load() : -1; }
#define FA_DIAG_COUNT(w) g_diag_calls[w].fetch_add(1)
#else
#define FA_DIAG_COUNT(w) ((void)0)
#endif

int fa_forward(void* stream, const fa_problem* p, const void* Q, const void* K, const void* V, void* O, void* l,
               void* m) {
  int st = fa_validate(p);
  if (st != FA_OK) return st;
  FA_DIAG_COUNT(0);
  fa::FwdArgs a;
  a.Q = Q; a.K = K; a.V = V; a.O = O; a.l = l; a.m = m;
  a.b = p->b; a.d = p->d; a.v_d = p->v_d;
  a.scale = 1.0 / sqrt((double)p->d);
  build_rule(p, &a.rule);
  if (a.b == 0 || a.rule.q.n == 0) return FA_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (p->dtype == FA_F16 && fa::fwd_f16_supported(a)) {
    e = fa::launch_fwd_f16(a, s);
  } else if (p->dtype == FA_F32 && fa::fwd_f32_supported(a)) {
    e = fa::launch_fwd_f32(a, s);
  } else if (p->dtype == FA_F64 && fa::fwd_f64_supported(a)) {
    e = fa::launch_fwd_f64(a, s);
  } else {
    if (p->d > fa::generic_max_channels(p->dtype) || p->v_d > fa::generic_max_channels(p->dtype))
      return set_error(FA_ERR_UNSUPPORTED, "channel dimension exceeds the supported maximum for this dtype");
    e = fa::launch_fwd_generic(p->dtype, a, s);
  }
  if (e != hipSuccess)
    return set_error((int)e, std::string("Failed to launch the Forward kernel: ") + hipGetErrorString(e));
  return FA_OK;
}

size_t fa_backward_workspace_bytes(const fa_problem* p) {
  if (fa_validate(p) != FA_OK) return 0;
  return ws_layout(p).total;
}

int fa_backward(void* stream, const fa_problem* p, const void* Q, const void* K, const void* V, const void* O,
                const void* l, const void* m, const void* dO, void* dQ, void* dK, void* dV, void* workspace,
                size_t workspace_bytes) {
  int st = fa_validate(p);
  if (st != FA_OK) return st;
  const WsLayout w = ws_layout(p);
  if (workspace_bytes < w.total || (!workspace && w.total > 0))
    return set_error(FA_ERR_WORKSPACE_TOO_SMALL, "backward workspace is smaller than fa_backward_workspace_bytes()");
  FA_DIAG_COUNT(1);
  fa::BwdArgs a;
  a.Q = Q; a.K = K; a.V = V; a.O = O; a.l = l; a.m = m; a.dO = dO;
  a.dQ = dQ; a.dK = dK; a.dV = dV;
  char* ws = static_cast<char*>(workspace);
  a.ws_dQ = ws + w.dq;
  a.ws_D = ws + w.D;
  a.ws_lse = ws + w.lse;
  a.b = p->b; a.d = p->d; a.v_d = p->v_d;
  a.scale = 1.0 / sqrt((double)p->d);
  build_rule(p, &a.rule);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.b == 0) return FA_OK;
  hipError_t e = hipSuccess;
  if (a.rule.q.n == 0 || a.rule.k.n == 0) {
    // nothing attends: every gradient is zero
    const size_t es = elem_size(p->dtype);
    if (a.rule.q.n) e = hipMemsetAsync(dQ, 0, es * (size_t)a.b * a.d * a.rule.q.n, s);
    if (e == hipSuccess && a.rule.k.n) e = hipMemsetAsync(dK, 0, es * (size_t)a.b * a.d * a.rule.k.n, s);
    if (e == hipSuccess && a.rule.k.n) e = hipMemsetAsync(dV, 0, es * (size_t)a.b * a.v_d * a.rule.k.n, s);
  } else if (p->dtype == FA_F16 && fa::bwd_f16_supported(a)) {
    e = fa::launch_bwd_f16(a, s);
  } else if (p->dtype == FA_F32 && fa::bwd_f32_supported(a)) {
    e = fa::launch_bwd_f32(a, s);
  } else if (p->dtype == FA_F64 && fa::bwd_f64_supported(a)) {
    e = fa::launch_bwd_f64(a, s);
  } else {
    if (p->d > fa::generic_max_channels(p->dtype) || p->v_d > fa::generic_max_channels(p->dtype))
      return set_error(FA_ERR_UNSUPPORTED, "channel dimension exceeds the supported maximum for this dtype");
    e = fa::launch_bwd_generic(p->dtype, a, s);
  }
  if (e != hipSuccess)
    return set_error((int)e, std::string("Failed to launch the Backward kernel: ") + hipGetErrorString(e));
  return FA_OK;
}

int64_t fa_allowed_pairs(const fa_problem* p) {
  if (fa_validate(p) != FA_OK) return -1;
  fa::Rule r;
  build_rule(p, &r);
  const int64_t nq = r.q.n, nk = r.k.n;
  if (r.policy == FA_FULL) return nq * nk;
  int64_t total = 0;
  for (int32_t q = 0; q < nq; ++q) {
    int32_t kb, ke;
    fa::k_range_for_q_block(r, q, q, &kb, &ke);
    if (r.policy == FA_CAUSAL) {  // the causal range is exact
      total += ke - kb;
      continue;
    }
    const int32_t qo = fa::seq_order(r.q, r, q);
    for (int32_t k = kb; k < ke; ++k) total += fa::check_orders(r, qo, fa::seq_order(r.k, r, k)) ? 1 : 0;
  }
  return total;
}

int fa_rule_mask(const fa_problem* p, uint8_t* mask) {
  int st = fa_validate(p);
  if (st != FA_OK) return st;
  if (!mask) return set_error(FA_ERR_INVALID_ARGUMENT, "null mask buffer");
  fa::Rule r;
  build_rule(p, &r);
  for (int32_t q = 0; q < r.q.n; ++q) {
    const int32_t qo = fa::seq_order(r.q, r, q);
    for (int32_t k = 0; k < r.k.n; ++k)
      mask[(int64_t)q * r.k.n + k] = fa::check_orders(r, qo, fa::seq_order(r.k, r, k)) ? 1 : 0;
  }
  return FA_OK;
}

int fa_rule_probe(const fa_problem* p, int32_t q0, int32_t q1, int32_t k0, int32_t k1, int32_t* out) {
  int st = fa_validate(p);
  if (st != FA_OK) return st;
  fa::Rule r;
  build_rule(p, &r);
  if (!out || q0 < 0 || q1 < q0 || q1 >= r.q.n || k0 < 0 || k1 < k0 || k1 >= r.k.n)
    return set_error(FA_ERR_INVALID_ARGUMENT, "probe block out of range");
  fa::k_range_for_q_block(r, q0, q1, &out[0], &out[1]);
  fa::q_range_for_k_block(r, k0, k1, &out[2], &out[3]);
  out[4] = fa::tile_class(r, q0, q1, k0, k1);
  return FA_OK;
}

double fa_estimate_forward_flops(const fa_problem* p) {
  const int64_t pairs = fa_allowed_pairs(p);
  if (pairs < 0) return -1.0;
  return 2.0 * (double)(p->d + p->v_d) * (double)pairs * (double)p->b;
}

const char* fa_error_string(int status) {
  switch (status) {
    case FA_OK: return "success";
    case FA_ERR_INVALID_ARGUMENT: return "invalid argument";
    case FA_ERR_UNSUPPORTED: return "unsupported problem";
    case FA_ERR_WORKSPACE_TOO_SMALL: return "workspace too small";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

const char* fa_last_error(void) { return g_last_error.c_str(); }

#ifndef FA_SRC_HASH
#define FA_SRC_HASH "unknown"
#endif
#ifdef FA_DIAG
#define FA_LIB_KIND "diagnostic (FA_DIAG: environment-selected variants)"
#else
#define FA_LIB_KIND "product"
#endif

const char* fa_build_info(void) {
  return "tf_flash_attention_amd: src=" FA_SRC_HASH "; lib=" FA_LIB_KIND "; gfx950; fwd={mfma_f16, mfma_f32, mfma_f64, generic(f16,f32,f64)}; bwd={mfma_f16 (two-pass / single-pass), mfma_f32 (two-pass), mfma_f64 (two-pass, d<=256), generic(f16,f32,f64)}";
}

}  // extern "C"
