// fa_tf_ops.cc — the TensorFlow-ROCm op library of the MI355X flash-attention op.
//
// Built into `flash_attention/kernel/flash_attention.so` (build_tf_op.sh), it is
// what the reference's unchanged Python module loads with tf.load_op_library
// (/root/reference/flash_attention/flash_attention.py:77-78): the same 30 op
// names, attrs, dtypes and shape functions as the reference's registrations
//   forward   flash_attention_forward.cc:144-253  (kernels :548-589)
//   backward  flash_attention_backward.cc:51-154  (kernels :385-403)
// so the wrappers and their gradient registrations (flash_attention.py:372-471)
// work as they are.  Every op kernel is a thin host shim over the C ABI of
// libfa_hip.so (include/fa_api.h); all device work is in the gfx950 kernels.
//
// Error behaviour follows the reference: shape errors are InvalidArgument with
// the reference's messages (forward.cc:100-133, backward.cc:197-258), an unknown
// sync_mode fails at construction (forward.cc:275-276), a failed launch is
// Internal("Failed to launch the Forward kernel: <str>(<code>)") (forward.cc:383-385).
// Differences: no output memsets and no Br_occupancy temp (the kernels
// write every O/l/m element); the backward scratch is an allocate_temp of
// fa_backward_workspace_bytes(); Estimate*Flops returns rule-exact algorithmic
// FLOPs instead of the reference's tile-issued count.
//
// This image has no TensorFlow, so this file is built only where one is present.
#include <string>
#include <type_traits>

#include "tensorflow/core/framework/op.h"
#include "tensorflow/core/framework/op_kernel.h"
#include "tensorflow/core/framework/shape_inference.h"
#include "tensorflow/core/framework/tensor_shape.h"

#include "fa_api.h"

using namespace tensorflow;
using GPUDevice = Eigen::GpuDevice;

namespace {

// ---------------------------------------------------------------- shape functions
// O = V's batch + channel dims ++ Q's sequence dims; l, m = Q's batch ++ sequence dims
template <int SeqDims>
absl::Status ForwardShapes(shape_inference::InferenceContext* c) {
  shape_inference::ShapeHandle q = c->input(0), k = c->input(1), v = c->input(2);
  const int rank = c->Rank(q);
  if (!(rank == c->Rank(k) && rank == c->Rank(v) && rank >= SeqDims + 2))
    return absl::InvalidArgumentError(
        "Failed to infer the shape of outputs as the shape of some inputs might be incorrect");
  const int ch = rank - SeqDims - 1;
  shape_inference::ShapeHandle v_head, q_seq, q_batch, o, lm;
  TF_RETURN_IF_ERROR(c->Subshape(v, 0, ch + 1, &v_head));
  TF_RETURN_IF_ERROR(c->Subshape(q, ch + 1, &q_seq));
  TF_RETURN_IF_ERROR(c->Subshape(q, 0, ch, &q_batch));
  TF_RETURN_IF_ERROR(c->Concatenate(v_head, q_seq, &o));
  TF_RETURN_IF_ERROR(c->Concatenate(q_batch, q_seq, &lm));
  c->set_output(0, o);
  c->set_output(1, lm);
  c->set_output(2, lm);
  return absl::OkStatus();
}

absl::Status BackwardShapes(shape_inference::InferenceContext* c) {
  for (int i = 0; i < 3; ++i) c->set_output(i, c->input(i));  // dQ, dK, dV take Q, K, V's shapes
  return absl::OkStatus();
}

absl::Status ScalarShape(shape_inference::InferenceContext* c) {
  c->set_output(0, c->Scalar());
  return absl::OkStatus();
}

}  // namespace

// ---------------------------------------------------------------- op registrations
#define FA_LOCAL_ATTRS .Attr("window_size: int >= 1").Attr("log2_stride_size: int >= 0").Attr("is_causal: bool")

#define FA_REGISTER_FORWARD_OP(op, sd, extra)                                                                 \
  REGISTER_OP(op #sd "dFloat16")                                                                              \
      .Attr("T: {float16}").Input("q: T").Input("k: T").Input("v: T").Attr("sync_mode: string") extra        \
      .Output("o: T").Output("l: float").Output("m: T").SetShapeFn(&ForwardShapes<sd>);                      \
  REGISTER_OP(op #sd "d")                                                                                     \
      .Attr("T: {float, double}").Input("q: T").Input("k: T").Input("v: T").Attr("sync_mode: string") extra  \
      .Output("o: T").Output("l: T").Output("m: T").SetShapeFn(&ForwardShapes<sd>);

#define FA_REGISTER_BACKWARD_OP(op, sd, extra)                                                                 \
  REGISTER_OP(op #sd "dFloat16")                                                                               \
      .Attr("T: {float16}").Input("q: T").Input("k: T").Input("v: T").Input("o: T").Input("l: float")         \
      .Input("m: T").Input("d_o: T").Attr("sync_mode: string") extra                                          \
      .Output("d_q: T").Output("d_k: T").Output("d_v: T").SetShapeFn(&BackwardShapes);                        \
  REGISTER_OP(op #sd "d")                                                                                      \
      .Attr("T: {float, double}").Input("q: T").Input("k: T").Input("v: T").Input("o: T").Input("l: T")       \
      .Input("m: T").Input("d_o: T").Attr("sync_mode: string") extra                                          \
      .Output("d_q: T").Output("d_k: T").Output("d_v: T").SetShapeFn(&BackwardShapes);

#define FA_REGISTER_FLOPS_OP(op, sd, extra)                                                                   \
  REGISTER_OP("Estimate" op #sd "dFlops")                                                                     \
      .Attr("q_shape: shape").Attr("k_shape: shape").Attr("v_shape: shape")                                  \
      .Attr("dtype: {float16, float, double}").Attr("sync_mode: string") extra                               \
      .Output("flops: float").SetShapeFn(&ScalarShape);

#define FA_REGISTER_OPS(sd)                                          \
  FA_REGISTER_FORWARD_OP("FullAttentionForward", sd, )               \
  FA_REGISTER_FORWARD_OP("CausalAttentionForward", sd, )             \
  FA_REGISTER_FORWARD_OP("LocalAttentionForward", sd, FA_LOCAL_ATTRS) \
  FA_REGISTER_BACKWARD_OP("FullAttentionBackward", sd, )             \
  FA_REGISTER_BACKWARD_OP("CausalAttentionBackward", sd, )           \
  FA_REGISTER_BACKWARD_OP("LocalAttentionBackward", sd, FA_LOCAL_ATTRS) \
  FA_REGISTER_FLOPS_OP("FullAttentionForward", sd, )                 \
  FA_REGISTER_FLOPS_OP("CausalAttentionForward", sd, )               \
  FA_REGISTER_FLOPS_OP("LocalAttentionForward", sd, FA_LOCAL_ATTRS)

FA_REGISTER_OPS(1)
FA_REGISTER_OPS(2)

namespace {

// ---------------------------------------------------------------- host helpers
template <typename T>
constexpr int32_t fa_dtype_of() {
  return std::is_same<T, Eigen::half>::value ? FA_F16 : (std::is_same<T, float>::value ? FA_F32 : FA_F64);
}

// The op's rule attrs, read once at construction (immutable afterwards, so Compute is reentrant)
struct RuleAttrs {
  int32_t sync_mode = FA_NONE_FRONT;
  int32_t window_size = 1, log2_stride_size = 0, is_causal = 0;
};

template <int Policy>
void ReadRuleAttrs(OpKernelConstruction* ctx, RuleAttrs* r) {
  std::string sync;
  OP_REQUIRES_OK(ctx, ctx->GetAttr("sync_mode", &sync));
  r->sync_mode = fa_sync_mode_from_string(sync.c_str());
  OP_REQUIRES(ctx, r->sync_mode >= 0, errors::InvalidArgument("Unsupported sync_mode: ", sync));
  if (Policy == FA_LOCAL) {
    int ws = 1, ls = 0;
    bool causal = false;
    OP_REQUIRES_OK(ctx, ctx->GetAttr("window_size", &ws));
    OP_REQUIRES_OK(ctx, ctx->GetAttr("log2_stride_size", &ls));
    OP_REQUIRES_OK(ctx, ctx->GetAttr("is_causal", &causal));
    r->window_size = ws;
    r->log2_stride_size = ls;
    r->is_causal = causal ? 1 : 0;
  }
}

TensorShape SubShape(const TensorShape& s, int begin, int end) {
  TensorShape out;
  for (int i = begin; i < end; ++i) out.AddDim(s.dim_size(i));
  return out;
}

// Forward shape checks with the reference's messages (flash_attention_forward.cc:97-140);
// fills the problem and the output shapes.
template <int SeqDims>
absl::Status ForwardProblem(const TensorShape& q, const TensorShape& k, const TensorShape& v, fa_problem* p,
                            TensorShape* o_shape, TensorShape* lm_shape) {
  if (q.dims() != k.dims() || k.dims() != v.dims())
    return errors::InvalidArgument("The number of dimensions of Q, K, and V should be equal");
  if (q.dims() < SeqDims + 2)
    return errors::InvalidArgument("The number of dimensions of Q, K, and V should be >= ", SeqDims + 2);
  const int ch = q.dims() - SeqDims - 1, rank = q.dims();
  const TensorShape qb = SubShape(q, 0, ch), kb = SubShape(k, 0, ch), vb = SubShape(v, 0, ch);
  const TensorShape qs = SubShape(q, ch + 1, rank), ks = SubShape(k, ch + 1, rank), vs = SubShape(v, ch + 1, rank);
  if (q.dim_size(ch) != k.dim_size(ch)) return errors::InvalidArgument("The channel dimension of Q and K should be equal");
  if (qb != kb || qb != vb)
    return errors::InvalidArgument("The batch shape of all inputs should be equal, but Q_batch_shape = ",
                                   qb.DebugString(), ", K_batch_shape = ", kb.DebugString(),
                                   ", V_batch_shape = ", vb.DebugString(), " were received");
  if (ks != vs)
    return errors::InvalidArgument("The sequence shape of K and V are expected to be equal, but K_seq_shape = ",
                                   ks.DebugString(), ", V_seq_shape = ", vs.DebugString(), " are detected");
  p->seq_dims = SeqDims;
  p->b = qb.num_elements();
  for (int i = 0; i < SeqDims; ++i) {
    p->q_seq[i] = static_cast<int32_t>(qs.dim_size(i));
    p->k_seq[i] = static_cast<int32_t>(ks.dim_size(i));
  }
  p->d = static_cast<int32_t>(q.dim_size(ch));
  p->v_d = static_cast<int32_t>(v.dim_size(ch));
  if (o_shape) {
    *o_shape = SubShape(v, 0, ch + 1);
    o_shape->AppendShape(qs);
    *lm_shape = qb;
    lm_shape->AppendShape(qs);
  }
  if (fa_validate(p) != FA_OK) return errors::InvalidArgument(fa_last_error());
  return absl::OkStatus();
}

void* StreamOf(OpKernelContext* ctx) { return reinterpret_cast<void*>(ctx->eigen_device<GPUDevice>().stream()); }

// ---------------------------------------------------------------- op kernels
// Replaces FlashAttentionForwardBase::Compute (flash_attention_forward.cc:280-386)
template <typename T, int SeqDims, int Policy>
class FaForwardOp : public OpKernel {
 public:
  explicit FaForwardOp(OpKernelConstruction* ctx) : OpKernel(ctx) { ReadRuleAttrs<Policy>(ctx, &rule_); }

  void Compute(OpKernelContext* ctx) override {
    const Tensor &Q = ctx->input(0), &K = ctx->input(1), &V = ctx->input(2);
    fa_problem p{};
    p.dtype = fa_dtype_of<T>();
    p.policy = Policy;
    p.sync_mode = rule_.sync_mode;
    p.window_size = rule_.window_size;
    p.log2_stride_size = rule_.log2_stride_size;
    p.is_causal = rule_.is_causal;
    TensorShape o_shape, lm_shape;
    OP_REQUIRES_OK(ctx, ForwardProblem<SeqDims>(Q.shape(), K.shape(), V.shape(), &p, &o_shape, &lm_shape));
    Tensor *O = nullptr, *l = nullptr, *m = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, o_shape, &O));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, lm_shape, &l));  // float for the Float16 ops, else T
    OP_REQUIRES_OK(ctx, ctx->allocate_output(2, lm_shape, &m));
    const int rc = fa_forward(StreamOf(ctx), &p, Q.data(), K.data(), V.data(), O->data(), l->data(), m->data());
    OP_REQUIRES(ctx, rc == FA_OK,
                errors::Internal("Failed to launch the Forward kernel: ", fa_error_string(rc), "(", rc, ")"));
  }

 private:
  RuleAttrs rule_;
};

// Replaces FlashAttentionBackwardBase::Compute (flash_attention_backward.cc:181-344)
template <typename T, int SeqDims, int Policy>
class FaBackwardOp : public OpKernel {
 public:
  explicit FaBackwardOp(OpKernelConstruction* ctx) : OpKernel(ctx) { ReadRuleAttrs<Policy>(ctx, &rule_); }

  void Compute(OpKernelContext* ctx) override {
    const Tensor &Q = ctx->input(0), &K = ctx->input(1), &V = ctx->input(2), &O = ctx->input(3);
    const Tensor &l = ctx->input(4), &m = ctx->input(5), &dO = ctx->input(6);
    // the reference's backward checks and messages (flash_attention_backward.cc:197-258)
    OP_REQUIRES(ctx, Q.dims() == K.dims() && K.dims() == V.dims() && V.dims() == O.dims() && O.dims() == dO.dims(),
                errors::InvalidArgument("The number of dimensions of Q, K, V, O, and dO should be equal"));
    OP_REQUIRES(ctx, l.dims() == m.dims() && m.dims() == Q.dims() - 1,
                errors::InvalidArgument("The number of dimensions of l and m should be equal to the one of Q minus 1"));
    OP_REQUIRES(ctx, Q.dims() >= SeqDims + 2,
                errors::InvalidArgument("The number of dimensions of Q, K, V, O, and dO should be >= ", SeqDims + 2));
    const int rank = Q.dims(), ch = rank - SeqDims - 1;
    OP_REQUIRES(ctx, Q.dim_size(ch) == K.dim_size(ch),
                errors::InvalidArgument("The channel dimension of Q and K should be equal"));
    OP_REQUIRES(ctx, V.dim_size(ch) == O.dim_size(ch),
                errors::InvalidArgument("The channel dimension of V and O should be equal"));
    const TensorShape qb = SubShape(Q.shape(), 0, ch), kb = SubShape(K.shape(), 0, ch), vb = SubShape(V.shape(), 0, ch);
    const TensorShape ob = SubShape(O.shape(), 0, ch), lb = SubShape(l.shape(), 0, ch), mb = SubShape(m.shape(), 0, ch);
    const TensorShape db = SubShape(dO.shape(), 0, ch);
    OP_REQUIRES(ctx, qb == kb && qb == vb && vb == ob && ob == lb && lb == mb && mb == db,
                errors::InvalidArgument("The batch shape of all inputs should be equal, but Q_batch_shape = ",
                                        qb.DebugString(), ", K_batch_shape = ", kb.DebugString(),
                                        ", V_batch_shape = ", vb.DebugString(), ", O_batch_shape = ", ob.DebugString(),
                                        ", l_batch_shape = ", lb.DebugString(), ", m_batch_shape = ", mb.DebugString(),
                                        ", dO_batch_shape = ", db.DebugString(), " are received"));
    const TensorShape qs = SubShape(Q.shape(), ch + 1, rank), ks = SubShape(K.shape(), ch + 1, rank);
    const TensorShape vs = SubShape(V.shape(), ch + 1, rank), os = SubShape(O.shape(), ch + 1, rank);
    const TensorShape ls = SubShape(l.shape(), ch, rank - 1), ms = SubShape(m.shape(), ch, rank - 1);
    const TensorShape ds = SubShape(dO.shape(), ch + 1, rank);
    OP_REQUIRES(ctx, ks == vs,
                errors::InvalidArgument("The sequence shape of K and V should be equal, but K_seq_shape = ",
                                        ks.DebugString(), ", V_seq_shape = ", vs.DebugString(), " were received"));
    OP_REQUIRES(ctx, qs == os && os == ls && ls == ms && ms == ds,
                errors::InvalidArgument("The sequence shape of Q, O, l, m, and dO should be equal, but Q_seq_shape = ",
                                        qs.DebugString(), ", O_seq_shape = ", os.DebugString(),
                                        ", l_seq_shape = ", ls.DebugString(), ", m_seq_shape = ", ms.DebugString(),
                                        ", dO_seq_shape = ", ds.DebugString(), " were received"));
    fa_problem p{};
    p.dtype = fa_dtype_of<T>();
    p.policy = Policy;
    p.sync_mode = rule_.sync_mode;
    p.window_size = rule_.window_size;
    p.log2_stride_size = rule_.log2_stride_size;
    p.is_causal = rule_.is_causal;
    OP_REQUIRES_OK(ctx, ForwardProblem<SeqDims>(Q.shape(), K.shape(), V.shape(), &p, nullptr, nullptr));

    Tensor *dQ = nullptr, *dK = nullptr, *dV = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, Q.shape(), &dQ));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(1, K.shape(), &dK));
    OP_REQUIRES_OK(ctx, ctx->allocate_output(2, V.shape(), &dV));
    const size_t ws_bytes = fa_backward_workspace_bytes(&p);
    Tensor ws;
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_UINT8, TensorShape({static_cast<int64_t>(ws_bytes > 0 ? ws_bytes : 1)}), &ws));
    const int rc = fa_backward(StreamOf(ctx), &p, Q.data(), K.data(), V.data(), O.data(), l.data(), m.data(),
                               dO.data(), dQ->data(), dK->data(), dV->data(), ws.data(), ws_bytes);
    OP_REQUIRES(ctx, rc == FA_OK,
                errors::Internal("Failed to launch the Backward kernel: ", fa_error_string(rc), "(", rc, ")"));
  }

 private:
  RuleAttrs rule_;
};

// Replaces FlashAttentionForwardFlopsEstimationBase (flash_attention_forward.cc:390-474):
// host-only, rule-exact algorithmic FLOPs 2*(d+v_d)*P
template <typename T, int SeqDims, int Policy>
class FaFlopsOp : public OpKernel {
 public:
  explicit FaFlopsOp(OpKernelConstruction* ctx) : OpKernel(ctx) {
    ReadRuleAttrs<Policy>(ctx, &rule_);
    OP_REQUIRES_OK(ctx, ctx->GetAttr("q_shape", &q_shape_));
    OP_REQUIRES_OK(ctx, ctx->GetAttr("k_shape", &k_shape_));
    OP_REQUIRES_OK(ctx, ctx->GetAttr("v_shape", &v_shape_));
  }

  void Compute(OpKernelContext* ctx) override {
    fa_problem p{};
    p.dtype = fa_dtype_of<T>();
    p.policy = Policy;
    p.sync_mode = rule_.sync_mode;
    p.window_size = rule_.window_size;
    p.log2_stride_size = rule_.log2_stride_size;
    p.is_causal = rule_.is_causal;
    OP_REQUIRES_OK(ctx, ForwardProblem<SeqDims>(q_shape_, k_shape_, v_shape_, &p, nullptr, nullptr));
    Tensor* flops = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({}), &flops));  // HostMemory("flops")
    flops->flat<float>()(0) = static_cast<float>(fa_estimate_forward_flops(&p));
  }

 private:
  RuleAttrs rule_;
  TensorShape q_shape_, k_shape_, v_shape_;
};

}  // namespace

// ---------------------------------------------------------------- kernel registrations
#define FA_REGISTER_KERNELS(op, policy, sd)                                                                          \
  REGISTER_KERNEL_BUILDER(Name(op "Forward" #sd "dFloat16").Device(DEVICE_GPU).TypeConstraint<Eigen::half>("T"),  \
                          FaForwardOp<Eigen::half, sd, policy>);                                                  \
  REGISTER_KERNEL_BUILDER(Name(op "Forward" #sd "d").Device(DEVICE_GPU).TypeConstraint<float>("T"),               \
                          FaForwardOp<float, sd, policy>);                                                        \
  REGISTER_KERNEL_BUILDER(Name(op "Forward" #sd "d").Device(DEVICE_GPU).TypeConstraint<double>("T"),              \
                          FaForwardOp<double, sd, policy>);                                                       \
  REGISTER_KERNEL_BUILDER(Name(op "Backward" #sd "dFloat16").Device(DEVICE_GPU).TypeConstraint<Eigen::half>("T"), \
                          FaBackwardOp<Eigen::half, sd, policy>);                                                 \
  REGISTER_KERNEL_BUILDER(Name(op "Backward" #sd "d").Device(DEVICE_GPU).TypeConstraint<float>("T"),              \
                          FaBackwardOp<float, sd, policy>);                                                       \
  REGISTER_KERNEL_BUILDER(Name(op "Backward" #sd "d").Device(DEVICE_GPU).TypeConstraint<double>("T"),             \
                          FaBackwardOp<double, sd, policy>);                                                      \
  REGISTER_KERNEL_BUILDER(Name("Estimate" op "Forward" #sd "dFlops").Device(DEVICE_GPU)                           \
                              .TypeConstraint<Eigen::half>("dtype").HostMemory("flops"),                          \
                          FaFlopsOp<Eigen::half, sd, policy>);                                                    \
  REGISTER_KERNEL_BUILDER(Name("Estimate" op "Forward" #sd "dFlops").Device(DEVICE_GPU)                           \
                              .TypeConstraint<float>("dtype").HostMemory("flops"),                                \
                          FaFlopsOp<float, sd, policy>);                                                          \
  REGISTER_KERNEL_BUILDER(Name("Estimate" op "Forward" #sd "dFlops").Device(DEVICE_GPU)                           \
                              .TypeConstraint<double>("dtype").HostMemory("flops"),                               \
                          FaFlopsOp<double, sd, policy>);

FA_REGISTER_KERNELS("FullAttention", FA_FULL, 1)
FA_REGISTER_KERNELS("CausalAttention", FA_CAUSAL, 1)
FA_REGISTER_KERNELS("LocalAttention", FA_LOCAL, 1)
FA_REGISTER_KERNELS("FullAttention", FA_FULL, 2)
FA_REGISTER_KERNELS("CausalAttention", FA_CAUSAL, 2)
FA_REGISTER_KERNELS("LocalAttention", FA_LOCAL, 2)
