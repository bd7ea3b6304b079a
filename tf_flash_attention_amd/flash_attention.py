"""Drop-in mirror of the reference's ``flash_attention/flash_attention.py`` on MI355X.

Public API (same names, argument meaning, defaults and return convention as
``/root/reference/flash_attention/flash_attention.py:80-370``)::

    full_1d(Q, K, V, sync_mode='none_front', returning_l_m=False)
    causal_1d(Q, K, V, sync_mode, returning_l_m=False)
    local_1d(Q, K, V, window_size, log2_stride_size, is_causal, sync_mode, returning_l_m=False)
    full_2d / causal_2d / local_2d   (same, for 2-D sequences)

Tensors are ``torch`` tensors on a ROCm device in the reference's channel-first
layout ``batch_shape + (C, *seq_shape)``.  Each call returns ``O`` or
``(O, l, m)``; autograd flows through ``O`` only (gradients of ``l``/``m`` are
ignored, as in ``flash_attention.py:382-384``).

``_fa_kernel`` exposes the op-level entry points under the snake_case names
TF generates for the reference's registered ops
(``flash_attention_forward.cc:144-253``, ``flash_attention_backward.cc:51-154``),
e.g. ``_fa_kernel.full_attention_forward1d_float16(q, k, v, sync_mode=...)`` and
``_fa_kernel.local_attention_backward2d(q, k, v, o, l, m, d_o, sync_mode=...,
window_size=..., log2_stride_size=..., is_causal=...)``.  They validate shapes
with the reference's exact messages (``flash_attention_forward.cc:97-140``,
``flash_attention_backward.cc:197-258``) and call the C ABI (``include/fa_api.h``)
on the current HIP stream.  There is no CPU / eager fallback.
"""

from __future__ import annotations

import re
from types import SimpleNamespace

import torch

from . import _lib

__all__ = [
    "full_1d", "causal_1d", "local_1d", "full_2d", "causal_2d", "local_2d",
    "InvalidArgumentError", "InternalError", "estimate_forward_flops",
]


class InvalidArgumentError(ValueError):
    """Mirror of tf.errors.InvalidArgumentError raised by the reference op kernels."""


class InternalError(RuntimeError):
    """Mirror of tf.errors.InternalError (kernel launch failures)."""


_DTYPES = {torch.float16: _lib.F16, torch.float32: _lib.F32, torch.float64: _lib.F64}
_POLICIES = {"full": _lib.FULL, "causal": _lib.CAUSAL, "local": _lib.LOCAL}


def _shape_str(shape) -> str:
    # TensorShape::DebugString() format
    return "[" + ",".join(str(int(s)) for s in shape) + "]"


def _sync_mode_id(sync_mode) -> int:
    if isinstance(sync_mode, bytes):
        sync_mode = sync_mode.decode()
    sid = {"none_front": _lib.NONE_FRONT, "scale_front": _lib.SCALE_FRONT,
           "scale_end": _lib.SCALE_END}.get(sync_mode, -1)
    if sid < 0:
        # FlashAttentionForwardBase ctor, flash_attention_forward.cc:274-276
        raise InvalidArgumentError(f"Unsupported sync_mode: {sync_mode}")
    return sid


def verify_and_extract_shapes(seq_dims, Q_shape, K_shape, V_shape):
    """VerifyAndExtractShapes<SequenceDims> (flash_attention_forward.cc:97-140)."""
    Q_shape, K_shape, V_shape = tuple(Q_shape), tuple(K_shape), tuple(V_shape)
    if not (len(Q_shape) == len(K_shape) == len(V_shape)):
        raise InvalidArgumentError("The number of dimensions of Q, K, and V should be equal")
    if len(Q_shape) < seq_dims + 2:
        raise InvalidArgumentError(f"The number of dimensions of Q, K, and V should be >= {seq_dims + 2}")
    ch = len(Q_shape) - seq_dims - 1
    Q_ch, K_ch, V_ch = Q_shape[ch], K_shape[ch], V_shape[ch]
    Qb, Qs = Q_shape[:ch], Q_shape[ch + 1:]
    Kb, Ks = K_shape[:ch], K_shape[ch + 1:]
    Vb, Vs = V_shape[:ch], V_shape[ch + 1:]
    if Q_ch != K_ch:
        raise InvalidArgumentError("The channel dimension of Q and K should be equal")
    if Qb != Kb or Qb != Vb:
        raise InvalidArgumentError(
            "The batch shape of all inputs should be equal, but Q_batch_shape = " + _shape_str(Qb)
            + ", K_batch_shape = " + _shape_str(Kb) + ", V_batch_shape = " + _shape_str(Vb) + " were received")
    if Ks != Vs:
        raise InvalidArgumentError(
            "The sequence shape of K and V are expected to be equal, but K_seq_shape = " + _shape_str(Ks)
            + ", V_seq_shape = " + _shape_str(Vs) + " are detected")
    return Qb, Qs, Q_ch, Kb, Ks, K_ch, Vb, Vs, V_ch


def verify_backward_shapes(seq_dims, Q, K, V, O, l, m, dO):
    """Checks of FlashAttentionBackwardBase::Compute (flash_attention_backward.cc:197-258)."""
    shapes = [tuple(t.shape) for t in (Q, K, V, O, l, m, dO)]
    Qs_, Ks_, Vs_, Os_, ls_, ms_, dOs_ = shapes
    if not (len(Qs_) == len(Ks_) == len(Vs_) == len(Os_) == len(dOs_)):
        raise InvalidArgumentError("The number of dimensions of Q, K, V, O, and dO should be equal")
    if not (len(ls_) == len(ms_) == len(Qs_) - 1):
        raise InvalidArgumentError("The number of dimensions of l and m should be equal to the one of Q minus 1")
    if len(Qs_) < seq_dims + 2:
        raise InvalidArgumentError(f"The number of dimensions of Q, K, V, O, and dO should be >= {seq_dims + 2}")
    ch = len(Qs_) - seq_dims - 1
    Q_ch, K_ch, V_ch, O_ch = Qs_[ch], Ks_[ch], Vs_[ch], Os_[ch]

    def split(s, lm=False):
        return s[:ch], (s[ch:] if lm else s[ch + 1:])

    (Qb, Qq), (Kb, Kk), (Vb, Vk), (Ob, Oq) = split(Qs_), split(Ks_), split(Vs_), split(Os_)
    (lb, lq), (mb, mq), (dOb, dOq) = split(ls_, True), split(ms_, True), split(dOs_)
    if Q_ch != K_ch:
        raise InvalidArgumentError("The channel dimension of Q and K should be equal")
    if V_ch != O_ch:
        raise InvalidArgumentError("The channel dimension of V and O should be equal")
    if not (Qb == Kb == Vb == Ob == lb == mb == dOb):
        raise InvalidArgumentError(
            "The batch shape of all inputs should be equal, but Q_batch_shape = " + _shape_str(Qb)
            + ", K_batch_shape = " + _shape_str(Kb) + ", V_batch_shape = " + _shape_str(Vb)
            + ", O_batch_shape = " + _shape_str(Ob) + ", l_batch_shape = " + _shape_str(lb)
            + ", m_batch_shape = " + _shape_str(mb) + ", dO_batch_shape = " + _shape_str(dOb) + " are received")
    if Kk != Vk:
        raise InvalidArgumentError(
            "The sequence shape of K and V should be equal, but K_seq_shape = " + _shape_str(Kk)
            + ", V_seq_shape = " + _shape_str(Vk) + " were received")
    if not (Qq == Oq == lq == mq == dOq):
        raise InvalidArgumentError(
            "The sequence shape of Q, O, l, m, and dO should be equal, but Q_seq_shape = " + _shape_str(Qq)
            + ", O_seq_shape = " + _shape_str(Oq) + ", l_seq_shape = " + _shape_str(lq)
            + ", m_seq_shape = " + _shape_str(mq) + ", dO_seq_shape = " + _shape_str(dOq) + " were received")
    return Qb, Qq, Q_ch, Kk, V_ch


def _prod(xs) -> int:
    n = 1
    for x in xs:
        n *= int(x)
    return n


def _check_device_tensors(*ts):
    dev = ts[0].device
    if dev.type != "cuda":
        raise InvalidArgumentError("flash attention tensors must live on a ROCm (cuda) device; there is no CPU kernel")
    for t in ts:
        if t.device != dev:
            raise InvalidArgumentError("all inputs must be on the same device")


def _dtype_id(t: torch.Tensor, float16_op: bool) -> int:
    dt = _DTYPES.get(t.dtype)
    if dt is None:
        raise TypeError(f"unsupported dtype {t.dtype}; expected float16, float32 or float64")
    if float16_op != (dt == _lib.F16):
        raise TypeError(f"op {'...Float16' if float16_op else '{float,double}'} does not accept {t.dtype}")
    return dt


def _raise_status(st: int, what: str):
    msg = _lib.last_error()
    if st == _lib.FA_ERR_INVALID_ARGUMENT:
        raise InvalidArgumentError(msg)
    if st == _lib.FA_ERR_UNSUPPORTED:
        raise InvalidArgumentError(msg)
    raise InternalError(msg or f"Failed to launch the {what} kernel ({st})")


def _stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def attention_forward(policy: str, seq_dims: int, Q, K, V, sync_mode, window_size=1, log2_stride_size=0,
                      is_causal=False, float16_op=None):
    """Op-level forward: returns (O, l, m).  Mirrors FlashAttentionForwardBase::Compute."""
    sid = _sync_mode_id(sync_mode)
    Qb, Qs, Q_ch, _, Ks, _, _, _, V_ch = verify_and_extract_shapes(seq_dims, Q.shape, K.shape, V.shape)
    if float16_op is None:
        float16_op = Q.dtype == torch.float16
    dt = _dtype_id(Q, float16_op)
    if K.dtype != Q.dtype or V.dtype != Q.dtype:
        raise TypeError("Q, K and V must share one dtype")
    _check_device_tensors(Q, K, V)
    Q, K, V = Q.contiguous(), K.contiguous(), V.contiguous()
    l_dtype = torch.float32 if dt == _lib.F16 else Q.dtype
    O = torch.empty(Qb + (V_ch,) + Qs, dtype=Q.dtype, device=Q.device)
    l = torch.empty(Qb + Qs, dtype=l_dtype, device=Q.device)
    m = torch.empty(Qb + Qs, dtype=Q.dtype, device=Q.device)
    prob = _lib.make_problem(dt, _POLICIES[policy], seq_dims, sid, _prod(Qb), Qs, Ks, Q_ch, V_ch,
                             window_size, log2_stride_size, is_causal)
    L = _lib.lib()
    with torch.cuda.device(Q.device):
        st = L.fa_forward(_stream_handle(Q.device), prob, Q.data_ptr(), K.data_ptr(), V.data_ptr(),
                          O.data_ptr(), l.data_ptr(), m.data_ptr())
    if st != _lib.FA_OK:
        _raise_status(st, "Forward")
    return O, l, m


def attention_backward(policy: str, seq_dims: int, Q, K, V, O, l, m, dO, sync_mode, window_size=1,
                       log2_stride_size=0, is_causal=False, float16_op=None):
    """Op-level backward: returns (dQ, dK, dV).  Mirrors FlashAttentionBackwardBase::Compute."""
    sid = _sync_mode_id(sync_mode)
    Qb, Qs, Q_ch, Ks, V_ch = verify_backward_shapes(seq_dims, Q, K, V, O, l, m, dO)
    if float16_op is None:
        float16_op = Q.dtype == torch.float16
    dt = _dtype_id(Q, float16_op)
    # the typed op inputs of flash_attention_backward.cc:51-154: q, k, v, o, m: T; l: float for the
    # Float16 ops, T otherwise (a mismatched l would be read at the wrong width)
    for name, t in (("K", K), ("V", V), ("O", O), ("m", m)):
        if t.dtype != Q.dtype:
            raise TypeError(f"{name} must have Q's dtype {Q.dtype}, got {t.dtype}")
    l_dtype = torch.float32 if dt == _lib.F16 else Q.dtype
    if l.dtype != l_dtype:
        raise TypeError(f"l must be {l_dtype} for this op, got {l.dtype}")
    _check_device_tensors(Q, K, V, O, l, m, dO)
    Q, K, V, O, l, m, dO = (t.contiguous() for t in (Q, K, V, O, l, m, dO))
    dO = dO.to(Q.dtype)
    dQ = torch.empty_like(Q)
    dK = torch.empty_like(K)
    dV = torch.empty_like(V)
    prob = _lib.make_problem(dt, _POLICIES[policy], seq_dims, sid, _prod(Qb), Qs, Ks, Q_ch, V_ch,
                             window_size, log2_stride_size, is_causal)
    L = _lib.lib()
    ws_bytes = L.fa_backward_workspace_bytes(prob)
    ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=Q.device)
    with torch.cuda.device(Q.device):
        st = L.fa_backward(_stream_handle(Q.device), prob, Q.data_ptr(), K.data_ptr(), V.data_ptr(),
                           O.data_ptr(), l.data_ptr(), m.data_ptr(), dO.data_ptr(), dQ.data_ptr(),
                           dK.data_ptr(), dV.data_ptr(), ws.data_ptr(), ws_bytes)
    if st != _lib.FA_OK:
        _raise_status(st, "Backward")
    return dQ, dK, dV


class _AttentionFn(torch.autograd.Function):
    """Forward op + its registered gradient (flash_attention.py:392-471)."""

    @staticmethod
    def forward(ctx, Q, K, V, policy, seq_dims, sync_mode, window_size, log2_stride_size, is_causal):
        O, l, m = attention_forward(policy, seq_dims, Q, K, V, sync_mode, window_size, log2_stride_size, is_causal)
        ctx.save_for_backward(Q, K, V, O, l, m)
        ctx.attrs = (policy, seq_dims, sync_mode, window_size, log2_stride_size, is_causal)
        ctx.mark_non_differentiable(l, m)
        return O, l, m

    @staticmethod
    def backward(ctx, dO, dl, dm):
        # only the gradient w.r.t. O is propagated (flash_attention.py:382-384)
        Q, K, V, O, l, m = ctx.saved_tensors
        policy, seq_dims, sync_mode, ws, ls, causal = ctx.attrs
        if dO is None:
            dO = torch.zeros_like(O)
        dQ, dK, dV = attention_backward(policy, seq_dims, Q, K, V, O, l, m, dO, sync_mode, ws, ls, causal)
        return dQ, dK, dV, None, None, None, None, None, None


def _attend(policy, seq_dims, Q, K, V, sync_mode, returning_l_m, window_size=1, log2_stride_size=0,
            is_causal=False):
    results = _AttentionFn.apply(Q, K, V, policy, seq_dims, sync_mode, window_size, log2_stride_size, is_causal)
    return results if returning_l_m else results[0]


def full_1d(Q, K, V, sync_mode="none_front", returning_l_m=False):
    """Full attention on 1d sequences (flash_attention.py:80-119)."""
    return _attend("full", 1, Q, K, V, sync_mode, returning_l_m)


def causal_1d(Q, K, V, sync_mode, returning_l_m=False):
    """Causal attention on 1d sequences (flash_attention.py:122-160)."""
    return _attend("causal", 1, Q, K, V, sync_mode, returning_l_m)


def local_1d(Q, K, V, window_size, log2_stride_size, is_causal, sync_mode, returning_l_m=False):
    """Local attention on 1d sequences (flash_attention.py:163-216)."""
    return _attend("local", 1, Q, K, V, sync_mode, returning_l_m, window_size, log2_stride_size, is_causal)


def full_2d(Q, K, V, sync_mode="none_front", returning_l_m=False):
    """Full attention on 2d sequences (flash_attention.py:219-263)."""
    return _attend("full", 2, Q, K, V, sync_mode, returning_l_m)


def causal_2d(Q, K, V, sync_mode, returning_l_m=False):
    """Causal attention on 2d sequences (flash_attention.py:266-309)."""
    return _attend("causal", 2, Q, K, V, sync_mode, returning_l_m)


def local_2d(Q, K, V, window_size, log2_stride_size, is_causal, sync_mode, returning_l_m=False):
    """Local attention on 2d sequences (flash_attention.py:312-370)."""
    return _attend("local", 2, Q, K, V, sync_mode, returning_l_m, window_size, log2_stride_size, is_causal)


# ----------------------------------------------------------------------------
# Op-name mirror of the TF-generated wrappers (REGISTER_OP names, snake_cased)
# ----------------------------------------------------------------------------
def _make_forward_op(policy, seq_dims, float16):
    def op(q, k, v, sync_mode, window_size=1, log2_stride_size=0, is_causal=False):
        return attention_forward(policy, seq_dims, q, k, v, sync_mode, window_size, log2_stride_size, is_causal,
                                 float16_op=float16)
    return op


def _make_backward_op(policy, seq_dims, float16):
    def op(q, k, v, o, l, m, d_o, sync_mode, window_size=1, log2_stride_size=0, is_causal=False):
        return attention_backward(policy, seq_dims, q, k, v, o, l, m, d_o, sync_mode, window_size,
                                  log2_stride_size, is_causal, float16_op=float16)
    return op


def estimate_forward_flops(policy, seq_dims, q_shape, k_shape, v_shape, sync_mode="none_front", window_size=1,
                           log2_stride_size=0, is_causal=False) -> float:
    """Estimate{Full,Causal,Local}AttentionForward{1,2}dFlops (flash_attention_forward.cc:217-245):
    algorithmic 2*(d+v_d)*allowed_pairs (not tile-issued work)."""
    sid = _sync_mode_id(sync_mode)
    Qb, Qs, Q_ch, _, Ks, _, _, _, V_ch = verify_and_extract_shapes(seq_dims, q_shape, k_shape, v_shape)
    prob = _lib.make_problem(_lib.F32, _POLICIES[policy], seq_dims, sid, _prod(Qb), Qs, Ks, Q_ch, V_ch,
                             window_size, log2_stride_size, is_causal)
    return float(_lib.lib().fa_estimate_forward_flops(prob))


def _make_flops_op(policy, seq_dims):
    def op(q_shape, k_shape, v_shape, dtype=None, sync_mode="none_front", window_size=1, log2_stride_size=0,
           is_causal=False):
        return estimate_forward_flops(policy, seq_dims, q_shape, k_shape, v_shape, sync_mode, window_size,
                                      log2_stride_size, is_causal)
    return op


_ops = {}
for _pol in ("full", "causal", "local"):
    for _sd in (1, 2):
        for _f16 in (True, False):
            suffix = "_float16" if _f16 else ""
            _ops[f"{_pol}_attention_forward{_sd}d{suffix}"] = _make_forward_op(_pol, _sd, _f16)
            _ops[f"{_pol}_attention_backward{_sd}d{suffix}"] = _make_backward_op(_pol, _sd, _f16)
        _ops[f"estimate_{_pol}_attention_forward{_sd}d_flops"] = _make_flops_op(_pol, _sd)
_fa_kernel = SimpleNamespace(**_ops)

# gradient dispatch table, as registered with @ops.RegisterGradient (flash_attention.py:392-471)
_OP_RE = re.compile(r".+(?P<ndim>\dd)(?P<f16>Float16)?$")


def gradient_op_for(op_type: str):
    """Maps a forward op type name (e.g. 'CausalAttentionForward1dFloat16') to its backward op."""
    m = re.match(r"(Full|Causal|Local)AttentionForward", op_type)
    match = _OP_RE.match(op_type)
    if not m or not match:
        raise ValueError(f'Unsupported op "{op_type}"')
    g = match.groupdict()
    name = f"{m.group(1).lower()}_attention_backward{g['ndim']}{'_float16' if g['f16'] else ''}"
    return getattr(_fa_kernel, name)


# ----------------------------------------------------------------------------
# The 'flops' statistic of each forward op (flash_attention.py:475-562 registers these with
# ops.RegisterStatistics, so TF's profiler reports the op's algorithmic FLOPs)
# ----------------------------------------------------------------------------
_STAT_OPS = tuple(f"{p}AttentionForward{n}d{f}" for p in ("Full", "Causal", "Local") for n in (1, 2)
                  for f in ("", "Float16"))


def forward_flops_statistics(op_type: str, q_shape, k_shape, v_shape, attrs) -> float:
    """The statistic the reference computes for a forward node (_estimate_{full,causal,local}_attention_
    forward_flops, flash_attention.py:498-562): the op's Estimate*Flops over the node's Q/K/V shapes with
    its sync_mode attr, and window_size / log2_stride_size / is_causal for the local ops.  Raises
    ValueError('Unsupported op "..."') for any other op name, as the reference does."""
    m = re.match(r"(Full|Causal|Local)AttentionForward(\d)d(Float16)?$", op_type)
    if not m or m.group(2) not in ("1", "2"):
        raise ValueError(f'Unsupported op "{op_type}"')
    policy, seq_dims = m.group(1).lower(), int(m.group(2))
    kw = {"sync_mode": attrs["sync_mode"]}
    if policy == "local":
        kw.update(window_size=int(attrs["window_size"]), log2_stride_size=int(attrs["log2_stride_size"]),
                  is_causal=bool(attrs["is_causal"]))
    return estimate_forward_flops(policy, seq_dims, tuple(q_shape), tuple(k_shape), tuple(v_shape), **kw)


def register_tf_statistics() -> bool:
    """With TensorFlow importable (the TF-ROCm op library of tf_op/ loaded), register
    forward_flops_statistics as the 'flops' statistic of the 12 forward ops, as importing the
    reference module does.  Returns False (nothing registered) when TensorFlow is absent."""
    try:
        from tensorflow.python.framework import ops as tf_ops  # noqa: WPS433 (optional dependency)
    except ImportError:
        return False

    def _stat(graph, node):
        def tensor(name):
            return graph.get_tensor_by_name(name if ":" in name else name + ":0")
        q, k, v = (tensor(node.input[i]) for i in range(3))
        attrs = {"sync_mode": node.attr["sync_mode"].s.decode()}
        if node.op.startswith("Local"):
            attrs.update(window_size=node.attr["window_size"].i, log2_stride_size=node.attr["log2_stride_size"].i,
                         is_causal=node.attr["is_causal"].b)
        flops = forward_flops_statistics(node.op, q.shape.as_list(), k.shape.as_list(), v.shape.as_list(), attrs)
        return tf_ops.OpStats("flops", flops)

    for name in _STAT_OPS:
        tf_ops.RegisterStatistics(name, "flops")(_stat)
    return True

