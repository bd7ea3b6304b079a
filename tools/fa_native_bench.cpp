// fa_native_bench.cpp — native (no Python, no framework) driver for the C ABI
// (include/fa_api.h): the equivalent of the reference's internal_test.cu harness
// (kernel/internal_test.cu:31-66 timing, :249-317 checks), built by
// `make -C tf_flash_attention_amd native` into tools/fa_native_bench.
//
//   fa_native_bench check                       small problems vs a double-precision CPU
//                                               loop (every policy, fp16/fp32/fp64)
//   fa_native_bench time <cfg> [iters]          hipEvent-timed forward / backward of a
//                                               BASELINE config: c2 c3 c4 c5
// Prints one JSON line per result.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "fa_api.h"

#define HIP_OK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

namespace {

size_t esize(int dt) { return dt == FA_F16 ? 2 : (dt == FA_F32 ? 4 : 8); }

void to_dtype(const std::vector<double>& x, int dt, std::vector<unsigned char>* out) {
  out->resize(x.size() * esize(dt));
  for (size_t i = 0; i < x.size(); ++i) {
    if (dt == FA_F16) reinterpret_cast<__half*>(out->data())[i] = __float2half((float)x[i]);
    else if (dt == FA_F32) reinterpret_cast<float*>(out->data())[i] = (float)x[i];
    else reinterpret_cast<double*>(out->data())[i] = x[i];
  }
}
double from_dtype(const unsigned char* p, int dt, size_t i) {
  if (dt == FA_F16) return __half2float(reinterpret_cast<const __half*>(p)[i]);
  if (dt == FA_F32) return reinterpret_cast<const float*>(p)[i];
  return reinterpret_cast<const double*>(p)[i];
}

struct Dev {
  void* p = nullptr;
  explicit Dev(size_t n) { HIP_OK(hipMalloc(&p, n ? n : 1)); }
  ~Dev() { (void)hipFree(p); }
};

// Double-precision forward + backward of one slice with the library's own rule
// (fa_rule_mask) as the mask: softmax(Qᵀ K / sqrt(d)) V (tests/test_1d.py:69-76)
void cpu_reference(const fa_problem& p, const std::vector<double>& Q, const std::vector<double>& K,
                   const std::vector<double>& V, const std::vector<double>& dO, std::vector<double>* O,
                   std::vector<double>* dQ, std::vector<double>* dK, std::vector<double>* dV) {
  int nq = 1, nk = 1;
  for (int i = 0; i < p.seq_dims; ++i) { nq *= p.q_seq[i]; nk *= p.k_seq[i]; }
  const int d = p.d, vd = p.v_d;
  std::vector<uint8_t> mask((size_t)nq * nk);
  fa_rule_mask(&p, mask.data());
  const double sc = 1.0 / std::sqrt((double)d);
  O->assign((size_t)p.b * vd * nq, 0.0);
  dQ->assign((size_t)p.b * d * nq, 0.0);
  dK->assign((size_t)p.b * d * nk, 0.0);
  dV->assign((size_t)p.b * vd * nk, 0.0);
  std::vector<double> P(nk), dP(nk);
  for (int64_t b = 0; b < p.b; ++b) {
    const double* q = &Q[b * d * nq]; const double* k = &K[b * d * nk];
    const double* v = &V[b * vd * nk]; const double* g = &dO[b * vd * nq];
    for (int i = 0; i < nq; ++i) {
      double mx = -INFINITY;
      for (int j = 0; j < nk; ++j) {
        double s = 0;
        for (int c = 0; c < d; ++c) s += q[c * nq + i] * k[c * nk + j];
        P[j] = mask[(size_t)i * nk + j] ? s * sc : -INFINITY;
        mx = std::max(mx, P[j]);
      }
      double l = 0;
      for (int j = 0; j < nk; ++j) { P[j] = (mx == -INFINITY) ? 0.0 : std::exp(P[j] - mx); l += P[j]; }
      for (int j = 0; j < nk; ++j) P[j] = l > 0 ? P[j] / l : 0.0;
      double Di = 0;
      for (int c = 0; c < vd; ++c) {
        double o = 0;
        for (int j = 0; j < nk; ++j) o += P[j] * v[c * nk + j];
        (*O)[b * vd * nq + c * nq + i] = o;
        Di += o * g[c * nq + i];
      }
      for (int j = 0; j < nk; ++j) {
        double s = 0;
        for (int c = 0; c < vd; ++c) s += g[c * nq + i] * v[c * nk + j];
        dP[j] = P[j] * (s - Di) * sc;
        for (int c = 0; c < vd; ++c) (*dV)[b * vd * nk + c * nk + j] += P[j] * g[c * nq + i];
      }
      for (int j = 0; j < nk; ++j)
        for (int c = 0; c < d; ++c) {
          (*dQ)[b * d * nq + c * nq + i] += dP[j] * k[c * nk + j];
          (*dK)[b * d * nk + c * nk + j] += dP[j] * q[c * nq + i];
        }
    }
  }
}

double max_rel_err(const std::vector<unsigned char>& got, int dt, const std::vector<double>& ref) {
  double mref = 1.0, err = 0.0;
  for (double r : ref) mref = std::max(mref, std::fabs(r));
  for (size_t i = 0; i < ref.size(); ++i) err = std::max(err, std::fabs(from_dtype(got.data(), dt, i) - ref[i]));
  return err / mref;
}

int check() {
  struct Case { int dt, pol, sd, mode; int qs[2], ks[2]; int d, ws, ls, causal; };
  // every policy x dtype x seq_dims (the reference's registered op matrix,
  // flash_attention_forward.cc:548-589), sync modes and ragged extents mixed in
  const Case cases[] = {
      {FA_F16, FA_FULL, 1, FA_NONE_FRONT, {256, 1}, {192, 1}, 64, 1, 0, 0},
      {FA_F16, FA_CAUSAL, 1, FA_NONE_FRONT, {320, 1}, {320, 1}, 128, 1, 0, 0},
      {FA_F16, FA_LOCAL, 1, FA_SCALE_END, {200, 1}, {264, 1}, 64, 33, 0, 1},
      {FA_F16, FA_FULL, 2, FA_SCALE_FRONT, {12, 10}, {24, 20}, 64, 1, 0, 0},
      {FA_F16, FA_CAUSAL, 2, FA_NONE_FRONT, {16, 9}, {16, 9}, 96, 1, 0, 0},
      {FA_F16, FA_LOCAL, 2, FA_SCALE_FRONT, {10, 12}, {20, 24}, 64, 3, 1, 0},
      {FA_F32, FA_FULL, 1, FA_SCALE_FRONT, {130, 1}, {260, 1}, 64, 1, 0, 0},
      {FA_F32, FA_CAUSAL, 1, FA_SCALE_END, {150, 1}, {75, 1}, 128, 1, 0, 0},
      {FA_F32, FA_LOCAL, 1, FA_NONE_FRONT, {300, 1}, {300, 1}, 32, 17, 1, 1},
      {FA_F32, FA_FULL, 2, FA_SCALE_FRONT, {8, 8}, {16, 16}, 64, 1, 0, 0},
      {FA_F32, FA_CAUSAL, 2, FA_SCALE_END, {8, 12}, {16, 6}, 48, 1, 0, 0},
      {FA_F32, FA_LOCAL, 2, FA_NONE_FRONT, {9, 7}, {9, 7}, 32, 2, 1, 0},
      {FA_F64, FA_FULL, 1, FA_NONE_FRONT, {100, 1}, {90, 1}, 64, 1, 0, 0},
      {FA_F64, FA_CAUSAL, 1, FA_SCALE_END, {77, 1}, {130, 1}, 16, 1, 0, 0},
      {FA_F64, FA_LOCAL, 1, FA_SCALE_FRONT, {64, 1}, {128, 1}, 32, 9, 0, 0},
      {FA_F64, FA_FULL, 2, FA_SCALE_END, {6, 6}, {12, 12}, 32, 1, 0, 0},
      {FA_F64, FA_CAUSAL, 2, FA_NONE_FRONT, {7, 9}, {7, 9}, 64, 1, 0, 0},
      {FA_F64, FA_LOCAL, 2, FA_NONE_FRONT, {8, 8}, {8, 8}, 16, 2, 0, 1},
  };
  int failures = 0;
  std::mt19937_64 rng(1234);
  std::uniform_real_distribution<double> U(-2.0, 2.0);
  for (const Case& c : cases) {
    fa_problem p{};
    p.dtype = c.dt; p.policy = c.pol; p.seq_dims = c.sd; p.sync_mode = c.mode; p.b = 2;
    for (int i = 0; i < c.sd; ++i) { p.q_seq[i] = c.qs[i]; p.k_seq[i] = c.ks[i]; }
    p.d = p.v_d = c.d; p.window_size = c.ws; p.log2_stride_size = c.ls; p.is_causal = c.causal;
    if (fa_validate(&p) != FA_OK) { fprintf(stderr, "invalid case: %s\n", fa_last_error()); return 2; }
    int nq = 1, nk = 1;
    for (int i = 0; i < c.sd; ++i) { nq *= c.qs[i]; nk *= c.ks[i]; }
    auto rnd = [&](size_t n) { std::vector<double> x(n); for (auto& v : x) v = U(rng); return x; };
    std::vector<double> Q = rnd(p.b * c.d * nq), K = rnd(p.b * c.d * nk), V = rnd(p.b * c.d * nk), G = rnd(p.b * c.d * nq);
    std::vector<unsigned char> hq, hk, hv, hg;
    to_dtype(Q, c.dt, &hq); to_dtype(K, c.dt, &hk); to_dtype(V, c.dt, &hv); to_dtype(G, c.dt, &hg);
    for (auto* t : {&Q, &K, &V, &G}) {  // the reference sees the rounded inputs
      std::vector<unsigned char> tmp; to_dtype(*t, c.dt, &tmp);
      for (size_t i = 0; i < t->size(); ++i) (*t)[i] = from_dtype(tmp.data(), c.dt, i);
    }
    const size_t es = esize(c.dt), les = c.dt == FA_F16 ? 4 : es;
    Dev q(hq.size()), k(hk.size()), v(hv.size()), g(hg.size()), o(hq.size()), dq(hq.size()), dk(hk.size()), dv(hv.size());
    Dev l(p.b * nq * les), m(p.b * nq * es);
    HIP_OK(hipMemcpy(q.p, hq.data(), hq.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(k.p, hk.data(), hk.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(v.p, hv.data(), hv.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(g.p, hg.data(), hg.size(), hipMemcpyHostToDevice));
    const size_t wsb = fa_backward_workspace_bytes(&p);
    Dev ws(wsb);
    int rc = fa_forward(nullptr, &p, q.p, k.p, v.p, o.p, l.p, m.p);
    if (rc == FA_OK) rc = fa_backward(nullptr, &p, q.p, k.p, v.p, o.p, l.p, m.p, g.p, dq.p, dk.p, dv.p, ws.p, wsb);
    if (rc != FA_OK) { fprintf(stderr, "launch failed: %s\n", fa_last_error()); return 2; }
    HIP_OK(hipDeviceSynchronize());
    std::vector<double> rO, rdQ, rdK, rdV;
    cpu_reference(p, Q, K, V, G, &rO, &rdQ, &rdK, &rdV);
    std::vector<unsigned char> go(hq.size()), gdq(hq.size()), gdk(hk.size()), gdv(hv.size());
    HIP_OK(hipMemcpy(go.data(), o.p, go.size(), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(gdq.data(), dq.p, gdq.size(), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(gdk.data(), dk.p, gdk.size(), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(gdv.data(), dv.p, gdv.size(), hipMemcpyDeviceToHost));
    const double tol = c.dt == FA_F16 ? 2e-3 : (c.dt == FA_F32 ? 1e-5 : 1e-10);
    const double e[4] = {max_rel_err(go, c.dt, rO), max_rel_err(gdq, c.dt, rdQ), max_rel_err(gdk, c.dt, rdK),
                         max_rel_err(gdv, c.dt, rdV)};
    const bool ok = e[0] <= tol && e[1] <= tol && e[2] <= tol && e[3] <= tol;
    failures += !ok;
    printf("{\"check\": \"dtype=%d policy=%d seq_dims=%d sync=%d d=%d\", \"err_O\": %.3e, \"err_dQ\": %.3e, "
           "\"err_dK\": %.3e, \"err_dV\": %.3e, \"tol\": %.0e, \"ok\": %s}\n",
           c.dt, c.pol, c.sd, c.mode, c.d, e[0], e[1], e[2], e[3], tol, ok ? "true" : "false");
  }
  return failures ? 1 : 0;
}

int time_config(const std::string& cfg, int iters) {
  fa_problem p{};
  p.seq_dims = 1; p.sync_mode = FA_NONE_FRONT; p.window_size = 1;
  bool bwd = false;
  if (cfg == "c2") { p.dtype = FA_F16; p.policy = FA_FULL; p.b = 128; p.d = 64; p.q_seq[0] = p.k_seq[0] = 4096; }
  else if (cfg == "c3") { p.dtype = FA_F16; p.policy = FA_CAUSAL; p.b = 128; p.d = 128; p.q_seq[0] = p.k_seq[0] = 8192; bwd = true; }
  else if (cfg == "c4") { p.dtype = FA_F16; p.policy = FA_LOCAL; p.b = 1024; p.d = 64; p.q_seq[0] = p.k_seq[0] = 16384; p.window_size = 256; }
  else if (cfg == "c5") {
    p.dtype = FA_F32; p.policy = FA_FULL; p.seq_dims = 2; p.sync_mode = FA_SCALE_FRONT; p.b = 32; p.d = 64;
    p.q_seq[0] = p.q_seq[1] = 64; p.k_seq[0] = p.k_seq[1] = 128;
  } else { fprintf(stderr, "unknown config %s\n", cfg.c_str()); return 2; }
  p.v_d = p.d;
  if (fa_validate(&p) != FA_OK) { fprintf(stderr, "%s\n", fa_last_error()); return 2; }
  const int64_t nq = (int64_t)p.q_seq[0] * (p.seq_dims == 2 ? p.q_seq[1] : 1);
  const int64_t nk = (int64_t)p.k_seq[0] * (p.seq_dims == 2 ? p.k_seq[1] : 1);
  const size_t es = esize(p.dtype), les = p.dtype == FA_F16 ? 4 : es;
  const size_t qb = p.b * p.d * nq * es, kb = p.b * p.d * nk * es;
  Dev q(qb), k(kb), v(kb), o(qb), g(qb), dq(qb), dk(kb), dv(kb), l(p.b * nq * les), m(p.b * nq * es);
  {  // U(-2, 2) inputs (fp16 / fp32 bit patterns written on the host once)
    std::mt19937_64 rng(1234);
    std::uniform_real_distribution<double> U(-2.0, 2.0);
    std::vector<double> x(p.b * p.d * std::max(nq, nk));
    for (auto& t : x) t = U(rng);
    std::vector<unsigned char> h;
    to_dtype(x, p.dtype, &h);
    for (Dev* t : {&q, &g}) HIP_OK(hipMemcpy(t->p, h.data(), qb, hipMemcpyHostToDevice));
    for (Dev* t : {&k, &v}) HIP_OK(hipMemcpy(t->p, h.data() + es, kb - es, hipMemcpyHostToDevice));
  }
  const size_t wsb = fa_backward_workspace_bytes(&p);
  Dev ws(wsb);
  const double ffl = fa_estimate_forward_flops(&p), bfl = ffl / (2.0 * 2 * p.d) * 2.0 * 5 * p.d;
  auto run_f = [&]() { return fa_forward(nullptr, &p, q.p, k.p, v.p, o.p, l.p, m.p); };
  auto run_b = [&]() { return fa_backward(nullptr, &p, q.p, k.p, v.p, o.p, l.p, m.p, g.p, dq.p, dk.p, dv.p, ws.p, wsb); };
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0)); HIP_OK(hipEventCreate(&e1));
  auto timed = [&](auto fn) {
    for (int i = 0; i < 40; ++i) if (fn() != FA_OK) { fprintf(stderr, "%s\n", fa_last_error()); exit(2); }
    HIP_OK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < iters; ++i) fn();
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
  };
  const float fms = timed(run_f);
  printf("{\"config\": \"%s\", \"op\": \"forward\", \"ms\": %.4f, \"tflops\": %.1f}\n", cfg.c_str(), fms,
         ffl / fms / 1e9);
  if (bwd) {
    const float bms = timed(run_b);
    printf("{\"config\": \"%s\", \"op\": \"backward\", \"ms\": %.4f, \"tflops\": %.1f}\n", cfg.c_str(), bms,
           bfl / bms / 1e9);
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "check";
  if (mode == "check") return check();
  if (mode == "time" && argc > 2) return time_config(argv[2], argc > 3 ? atoi(argv[3]) : 20);
  fprintf(stderr, "usage: %s check | time <c2|c3|c4|c5> [iters]\n", argv[0]);
  return 2;
}
