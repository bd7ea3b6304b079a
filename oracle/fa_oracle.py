"""CPU oracle for the fused flash-attention hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``tf_flash_attention_amd``) must never route through it.

What it restates (reference = nothingstopsme/tf_flash_attention, read-only at
/root/reference; citations are ``path:line`` relative to that tree):

* Sync methods (Q<->K sequence alignment): ``flash_attention/kernel/sync_methods.cc:8-111``
  (per-dim reference extent R_i = next pow2 >= max(Mq_i, Mk_i), strides
  ``max//M``, ``scale_end`` offsets ``stride-1``; dims pushed last-axis-first)
  and the order map ``sync_methods.h:56-85`` (order = sum_i c_i * prod_{j<i} R_j).
* Mask rules: ``flash_attention/kernel/flash_attention.h:45-149`` (Full, Causal,
  Local(window, log2_stride, is_causal)), plus out-of-range masking of padded
  rows/cols (``flash_attention.cu:927-932``).
* The reference's unit-test oracle ("vanilla attention"):
  ``flash_attention/tests/test_1d.py:69-76`` / ``tests/test_2d.py:97-109``:
  einsum(Q,K)/sqrt(C) -> where(mask, logit, min) -> softmax -> where(mask, p, 0)
  -> einsum(p, V); gradients are TF autodiff of that graph.  Its mask
  generators ``tests/test_base.py:33-67`` and coordinates ``tests/test_1d.py:9-50``,
  ``tests/test_2d.py:11-78`` are restated in :func:`vanilla_mask` as an
  independent second formulation of the rules.
* l / m outputs (not exposed by the vanilla path): ``flash_attention.cu:974-1035``
  (m = row max of scaled logits stored in T, l = sum exp(s - m), l in fp32 for
  fp16 inputs, ``flash_attention_forward.cc:152``), fully-masked rows keep the
  memset values O=0, l=0, m=bytes 0xFA (``flash_attention_forward.cc:352-365``,
  ``type_util.h:43-45``).
* Backward: D = rowsum(dO*O), dS = P*(dP - D)*scale
  (``flash_attention.cu:1544-1546``, ``internal_test.cu:381-513``).

Pinning: the reference ships no numeric golden vectors and cannot run here
(TensorFlow and CUDA are absent).  The sync maps and mask rules
are pinned to the known-answer examples the reference itself publishes (the
module docstring of ``flash_attention/flash_attention.py:1-70`` and the figures
under ``images/``), committed under ``tests/golden/`` and checked by
``tests/test_oracle.py``; the two reference formulations of the rules (kernel
rule + vanilla test generator) are cross-checked against each other.  The
attention numerics themselves are the textbook softmax-attention restated in
float64 — exact values at the TF boundary are "parity unpinned" (SURVEY §8c).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

SYNC_MODES = ("none_front", "scale_front", "scale_end")
POLICIES = ("full", "causal", "local")


# ----------------------------------------------------------------------------
# NegInfApprox: every byte 0xFA (type_util.h:43-45)
# ----------------------------------------------------------------------------
def neg_inf_approx(dtype) -> np.generic:
    dtype = np.dtype(dtype)
    raw = np.frombuffer(b"\xfa" * dtype.itemsize, dtype=dtype)
    return raw[0]


def l_dtype_for(dtype) -> np.dtype:
    """L_T: float32 for float16 inputs, T otherwise (flash_attention.h:181-185)."""
    dtype = np.dtype(dtype)
    return np.dtype(np.float32) if dtype == np.float16 else dtype


# ----------------------------------------------------------------------------
# Sync methods (sync_methods.cc:8-111)
# ----------------------------------------------------------------------------
@dataclass
class SyncPack:
    """Per-dimension description, index 0 = LAST sequence axis (sync_methods.cc:12-13)."""

    ref_shape: List[int]     # R_i (powers of two)
    q_shape: List[int]
    q_stride: List[int]
    q_offset: List[int]
    k_shape: List[int]
    k_stride: List[int]
    k_offset: List[int]


def _next_pow2(n: int) -> int:
    # host log2i is floor-log2 (cute_ext/algorithms.h:14); ref = 1<<log2i, doubled if short
    r = 1 << (max(int(n), 1).bit_length() - 1)
    if r < n:
        r <<= 1
    return r


def sync_pack(q_seq: Sequence[int], k_seq: Sequence[int], mode: str) -> SyncPack:
    if mode not in SYNC_MODES:
        raise ValueError(f"Unsupported sync_mode: {mode}")
    if len(q_seq) != len(k_seq):
        raise ValueError("Q and K sequence ranks differ")
    p = SyncPack([], [], [], [], [], [], [])
    for dim in reversed(range(len(q_seq))):
        mq, mk = int(q_seq[dim]), int(k_seq[dim])
        mx = max(mq, mk)
        p.ref_shape.append(_next_pow2(mx))
        if mode == "none_front":
            sq, sk = 1, 1
        else:
            sq, sk = mx // mq, mx // mk
        oq, ok = (sq - 1, sk - 1) if mode == "scale_end" else (0, 0)
        p.q_shape.append(mq); p.q_stride.append(sq); p.q_offset.append(oq)
        p.k_shape.append(mk); p.k_stride.append(sk); p.k_offset.append(ok)
    return p


def seq_coords(shape_rev: Sequence[int], stride: Sequence[int], offset: Sequence[int]) -> np.ndarray:
    """Reference-space coordinates of every flat (row-major) index.

    Returns int64 array [n, ndim] with column 0 = last axis.  The flat index is
    decomposed row-major over the sequence's own shape; c_i = idx_i*s_i + o_i
    (zipped_divide by stride then by shape, sync_methods.h:82-84)."""
    nd = len(shape_rev)
    n = int(np.prod(shape_rev))
    flat = np.arange(n, dtype=np.int64)
    coords = np.empty((n, nd), dtype=np.int64)
    rem = flat
    for i in range(nd):  # dim 0 (last axis) varies fastest
        idx = rem % shape_rev[i]
        rem = rem // shape_rev[i]
        coords[:, i] = idx * stride[i] + offset[i]
    return coords


def coords_to_order(coords: np.ndarray, ref_shape: Sequence[int]) -> np.ndarray:
    """order = sum_i c_i * prod_{j<i} R_j (AttentionPolicy::MapToOrder, flash_attention.h:27-41)."""
    order = np.zeros(coords.shape[0], dtype=np.int64)
    mult = 1
    for i, r in enumerate(ref_shape):
        order += coords[:, i] * mult
        mult *= r
    return order


def order_to_coords(order: np.ndarray, ref_shape: Sequence[int]) -> np.ndarray:
    """Shift/mask decomposition over pow-2 extents (MapToCoords, flash_attention.h:11-25)."""
    out = np.empty((order.shape[0], len(ref_shape)), dtype=np.int64)
    shift = 0
    for i, r in enumerate(ref_shape):
        out[:, i] = (order >> shift) & (r - 1)
        shift += int(r).bit_length() - 1
    return out


def seq_orders(q_seq, k_seq, mode) -> Tuple[np.ndarray, np.ndarray, SyncPack]:
    p = sync_pack(q_seq, k_seq, mode)
    qc = seq_coords(p.q_shape, p.q_stride, p.q_offset)
    kc = seq_coords(p.k_shape, p.k_stride, p.k_offset)
    return coords_to_order(qc, p.ref_shape), coords_to_order(kc, p.ref_shape), p


# ----------------------------------------------------------------------------
# Mask rules (flash_attention.h:45-149)
# ----------------------------------------------------------------------------
class RuleEval:
    """Evaluates the rule for arbitrary row/column sub-blocks (bounded memory)."""

    def __init__(self, q_seq, k_seq, mode, policy, window_size=1, log2_stride_size=0, is_causal=False):
        if policy not in POLICIES:
            raise ValueError(policy)
        self.qo, self.ko, self.p = seq_orders(q_seq, k_seq, mode)
        self.policy = policy
        self.ws, self.ls = int(window_size), int(log2_stride_size)
        strided = self.ws << self.ls
        self.look_ahead = 1 if is_causal else strided  # flash_attention.h:91-95
        if policy == "local":
            self.qc = order_to_coords(self.qo, self.p.ref_shape)
            self.kc = order_to_coords(self.ko, self.p.ref_shape)

    def block(self, r0, r1, c0=0, c1=None) -> np.ndarray:
        c1 = self.ko.size if c1 is None else c1
        qo, ko = self.qo[r0:r1], self.ko[c0:c1]
        if self.policy == "full":
            return np.ones((qo.size, ko.size), dtype=bool)
        if self.policy == "causal":
            return qo[:, None] >= ko[None, :]
        ok = np.ones((qo.size, ko.size), dtype=bool)
        if self.look_ahead == 1:
            ok &= qo[:, None] >= ko[None, :]
        rem_mask = (1 << self.ls) - 1
        for i in range(len(self.p.ref_shape)):
            diff = np.abs(self.qc[r0:r1, i][:, None] - self.kc[c0:c1, i][None, :])
            ok &= ((diff & rem_mask) == 0) & ((diff >> self.ls) < self.ws)
        return ok


def rule_mask(q_seq, k_seq, mode, policy, window_size=1, log2_stride_size=0, is_causal=False) -> np.ndarray:
    """bool [Nq, Nk]: True where the (q, k) pair is attended."""
    ev = RuleEval(q_seq, k_seq, mode, policy, window_size, log2_stride_size, is_causal)
    return ev.block(0, ev.qo.size)


def vanilla_coords(q_seq, k_seq, mode):
    """The unit-test coordinate generators (tests/test_1d.py:9-50, tests/test_2d.py:11-78).

    Returns (Q_coords [Nq, nd] in (y, x) order, K_coords, Q_l, K_l) where l is the
    causality index y*max_width + x."""
    nd = len(q_seq)
    maxes = [max(a, b) for a, b in zip(q_seq, k_seq)]

    def one(shape):
        grids = np.meshgrid(*[np.arange(s, dtype=np.int64) for s in shape], indexing="ij")
        cs = []
        for i, g in enumerate(grids):
            step = 1 if mode == "none_front" else maxes[i] // shape[i]
            c = g * step if mode != "scale_end" else (g + 1) * step - 1
            cs.append(c.reshape(-1))
        coords = np.stack(cs, axis=-1)
        if nd == 1:
            l_idx = coords[:, 0]
        else:
            l_idx = coords[:, 0] * maxes[-1] + coords[:, 1]
        return coords, l_idx

    qc, ql = one(q_seq)
    kc, kl = one(k_seq)
    return qc, kc, ql, kl


def vanilla_mask(q_seq, k_seq, mode, policy, window_size=1, log2_stride_size=0, is_causal=False) -> np.ndarray:
    """Mask exactly as the reference's test generators build it (tests/test_base.py:33-67),
    generalised to an explicit window/stride (the tests fix window = max(diff.shape))."""
    qc, kc, ql, kl = vanilla_coords(q_seq, k_seq, mode)
    idx_diff = ql[:, None] - kl[None, :]
    if policy == "full":
        return np.ones_like(idx_diff, dtype=bool)
    if policy == "causal":
        return idx_diff >= 0
    diff = np.abs(qc[:, None, :] - kc[None, :, :])
    pred = idx_diff >= 0 if is_causal else np.ones_like(idx_diff, dtype=bool)
    stride = 2 ** int(log2_stride_size)
    if stride > 1:
        return pred & np.all(((diff % stride) == 0) & (diff // stride < window_size), axis=-1)
    return pred & np.all(diff < window_size, axis=-1)


# ----------------------------------------------------------------------------
# Forward / backward restatement (float64 math on dtype-rounded inputs)
# ----------------------------------------------------------------------------
@dataclass
class Problem:
    policy: str
    seq_dims: int
    sync_mode: str = "none_front"
    window_size: int = 1
    log2_stride_size: int = 0
    is_causal: bool = False


def _split(shape, seq_dims):
    ch = len(shape) - seq_dims - 1
    return tuple(shape[:ch]), int(shape[ch]), tuple(shape[ch + 1:])


def problem_mask(prob: Problem, q_seq, k_seq) -> np.ndarray:
    return rule_mask(q_seq, k_seq, prob.sync_mode, prob.policy,
                     prob.window_size, prob.log2_stride_size, prob.is_causal)


def _evaluator(prob: Problem, q_seq, k_seq) -> RuleEval:
    return RuleEval(q_seq, k_seq, prob.sync_mode, prob.policy, prob.window_size, prob.log2_stride_size,
                    prob.is_causal)


ROW_CHUNK = 512


def _row_chunks(ev: RuleEval, nq: int):
    """Yields (r0, r1, c0, c1, mask[r1-r0, c1-c0]) with [c0,c1) the column band that
    holds every attended key of rows [r0,r1) — row-exact, memory-bounded."""
    for r0 in range(0, nq, ROW_CHUNK):
        r1 = min(nq, r0 + ROW_CHUNK)
        full = ev.block(r0, r1)
        cols = np.nonzero(full.any(axis=0))[0]
        if cols.size == 0:
            yield r0, r1, 0, 0, full[:, :0]
        else:
            c0, c1 = int(cols[0]), int(cols[-1]) + 1
            yield r0, r1, c0, c1, full[:, c0:c1]


def _flat(Q, K, V, prob):
    bq, d, q_seq = _split(Q.shape, prob.seq_dims)
    bk, dk, k_seq = _split(K.shape, prob.seq_dims)
    bv, vd, v_seq = _split(V.shape, prob.seq_dims)
    assert bq == bk == bv and d == dk and k_seq == v_seq
    b = int(np.prod(bq)) if bq else 1
    nq, nk = int(np.prod(q_seq)), int(np.prod(k_seq))
    return bq, q_seq, k_seq, b, d, vd, nq, nk


def forward_f64(Q, K, V, prob: Problem, slices=None):
    """Float64 forward on dtype-rounded inputs (the parity reference).

    Returns (O [*, vd, *q_seq], L, M, has_any[nq]) — L = sum exp(s - M), M = row max of
    scaled logits (both float64, unrounded).  ``slices`` restricts the flattened batch
    slices computed (outputs then have leading dim len(slices))."""
    bq, q_seq, k_seq, b, d, vd, nq, nk = _flat(Q, K, V, prob)
    sl = list(range(b)) if slices is None else list(slices)
    ev = _evaluator(prob, q_seq, k_seq)
    q = Q.reshape(b, d, nq)
    k = K.reshape(b, d, nk)
    v = V.reshape(b, vd, nk)
    scale = 1.0 / math.sqrt(d)
    O = np.zeros((len(sl), vd, nq))
    M = np.zeros((len(sl), nq))
    L = np.zeros((len(sl), nq))
    has_any = np.zeros(nq, dtype=bool)
    for r0, r1, c0, c1, mk in _row_chunks(ev, nq):
        has_any[r0:r1] = mk.any(axis=1)
        if c1 == c0:
            continue
        ha = has_any[r0:r1]
        for j, i in enumerate(sl):
            s = np.where(mk, (q[i, :, r0:r1].astype(np.float64).T @ k[i, :, c0:c1].astype(np.float64)) * scale,
                         -np.inf)
            mrow = np.where(ha, s.max(axis=1), 0.0)
            p = np.exp(s - mrow[:, None])
            lrow = p.sum(axis=1)
            o = v[i, :, c0:c1].astype(np.float64) @ (p / np.where(ha, lrow, 1.0)[:, None]).T
            o[:, ~ha] = 0.0
            O[j, :, r0:r1] = o
            M[j, r0:r1] = mrow
            L[j, r0:r1] = np.where(ha, lrow, 0.0)
    lead = bq if slices is None else (len(sl),)
    return O.reshape(lead + (vd,) + q_seq), L.reshape(lead + q_seq), M.reshape(lead + q_seq), has_any


def forward(Q: np.ndarray, K: np.ndarray, V: np.ndarray, prob: Problem):
    """Returns (O, l, m) with the reference's output dtypes and shapes.

    O: batch ++ [v_d] ++ q_seq (T); l, m: batch ++ q_seq (L_T / T).  m is the row max
    rounded to T; l is sum exp(s - m_T) (relative to the STORED m); rows attending
    nothing get O=0, l=0, m=NegInfApprox."""
    T = Q.dtype
    LT = l_dtype_for(T)
    O64, L64, M64, has_any = forward_f64(Q, K, V, prob)
    m_t = M64.astype(T)
    l_rel = L64 * np.exp(M64 - m_t.astype(np.float64))
    ha = np.broadcast_to(has_any.reshape((1,) * (M64.ndim - prob.seq_dims) + M64.shape[M64.ndim - prob.seq_dims:]),
                         M64.shape)
    l_out = np.where(ha, l_rel, 0.0).astype(LT)
    m_out = np.where(ha, m_t, neg_inf_approx(T)).astype(T)
    return O64.astype(T), l_out, m_out


def backward_f64(Q, K, V, dO, prob: Problem, slices=None):
    """Gradients of the vanilla path w.r.t. Q, K, V in float64 (autodiff of
    tests/test_1d.py:69-76 restated analytically; fully-masked rows give 0).
    D = rowsum(dO*O), dS = P*(dP-D)*scale (flash_attention.cu:1544-1546)."""
    bq, q_seq, k_seq, b, d, vd, nq, nk = _flat(Q, K, V, prob)
    sl = list(range(b)) if slices is None else list(slices)
    ev = _evaluator(prob, q_seq, k_seq)
    q = Q.reshape(b, d, nq)
    k = K.reshape(b, d, nk)
    v = V.reshape(b, vd, nk)
    do = dO.reshape(b, vd, nq)
    scale = 1.0 / math.sqrt(d)
    dQ = np.zeros((len(sl), d, nq)); dK = np.zeros((len(sl), d, nk)); dV = np.zeros((len(sl), vd, nk))
    for r0, r1, c0, c1, mk in _row_chunks(ev, nq):
        if c1 == c0:
            continue
        ha = mk.any(axis=1)
        for j, i in enumerate(sl):
            qi = q[i, :, r0:r1].astype(np.float64)
            ki = k[i, :, c0:c1].astype(np.float64)
            vi = v[i, :, c0:c1].astype(np.float64)
            doi = do[i, :, r0:r1].astype(np.float64)
            s = np.where(mk, (qi.T @ ki) * scale, -np.inf)
            mrow = np.where(ha, s.max(axis=1), 0.0)
            p = np.exp(s - mrow[:, None])
            p = p / np.where(ha, p.sum(axis=1), 1.0)[:, None]   # 0 where masked
            o = vi @ p.T
            dV[j, :, c0:c1] += doi @ p
            dp = doi.T @ vi
            D = np.sum(doi * o, axis=0)
            ds = p * (dp - D[:, None]) * scale
            dQ[j, :, r0:r1] = ki @ ds.T
            dK[j, :, c0:c1] += qi @ ds
    if slices is None:
        return dQ.reshape(Q.shape), dK.reshape(K.shape), dV.reshape(V.shape)
    n = len(sl)
    return (dQ.reshape((n, d) + q_seq), dK.reshape((n, d) + k_seq), dV.reshape((n, vd) + k_seq))


def backward_rounding_scale_f64(Q, K, V, dO, prob: Problem, u_t: float, u_acc: float, slices=None):
    """Per-element rounding-error scale of the gradients (test infrastructure: the parity tests'
    tolerance model, not a reference algorithm).  Each gradient is a sum of per-pair terms
    (dQ = K·dSᵀ, dK = Q·dS, dV = dO·P, the same contractions as backward_f64); a term carries the
    rounding of its factor dS (or P), and the returned scale is the root-sum-square over the sum
    of |other factor| × that factor's error bound, the usual probabilistic bound for independent
    roundings.  The error bound of one dS = P·(dP − D)·scale is
        P·scale·( u_t·(1 + |s|_rss)·|dP − D| + u_t·|dO∘O|_rss + u_acc·Σ_c|dO_c·V_c| ),
    with |s|_rss = scale·(Σ_c (q_c·k_c)²)^½ the scale of a score's rounding (Q is rounded to the tensor
    type after scaling; the error scales P), |dO∘O|_rss the same for D (O is rounded to the tensor
    type), u_t the tensor type's unit roundoff (dS and P are rounded to it) and u_acc that of the
    accumulation: it grows where dP and D cancel, which a relative tolerance on the (small) result
    cannot see.  P's error bound is u_t·(1 + |s|_rss)·P."""
    bq, q_seq, k_seq, b, d, vd, nq, nk = _flat(Q, K, V, prob)
    sl = list(range(b)) if slices is None else list(slices)
    ev = _evaluator(prob, q_seq, k_seq)
    q = Q.reshape(b, d, nq)
    k = K.reshape(b, d, nk)
    v = V.reshape(b, vd, nk)
    do = dO.reshape(b, vd, nq)
    scale = 1.0 / math.sqrt(d)
    eQ = np.zeros((len(sl), d, nq)); eK = np.zeros((len(sl), d, nk)); eV = np.zeros((len(sl), vd, nk))
    for r0, r1, c0, c1, mk in _row_chunks(ev, nq):
        if c1 == c0:
            continue
        ha = mk.any(axis=1)
        for j, i in enumerate(sl):
            qi = q[i, :, r0:r1].astype(np.float64)
            ki = k[i, :, c0:c1].astype(np.float64)
            vi = v[i, :, c0:c1].astype(np.float64)
            doi = do[i, :, r0:r1].astype(np.float64)
            s = np.where(mk, (qi.T @ ki) * scale, -np.inf)
            mrow = np.where(ha, s.max(axis=1), 0.0)
            p = np.exp(s - mrow[:, None])
            p = p / np.where(ha, p.sum(axis=1), 1.0)[:, None]
            o = vi @ p.T
            dp = doi.T @ vi
            D = np.sum(doi * o, axis=0)
            s_rss = np.sqrt((qi * qi).T @ (ki * ki)) * scale
            e_p = u_t * (1.0 + s_rss) * p
            e_ds = scale * (e_p * np.abs(dp - D[:, None])
                            + p * (u_t * np.sqrt(np.sum((doi * o) ** 2, axis=0))[:, None]
                                   + u_acc * (np.abs(doi).T @ np.abs(vi))))
            eV[j, :, c0:c1] += (doi * doi) @ (e_p * e_p)
            eQ[j, :, r0:r1] = (ki * ki) @ (e_ds * e_ds).T
            eK[j, :, c0:c1] += (qi * qi) @ (e_ds * e_ds)
    eQ, eK, eV = np.sqrt(eQ), np.sqrt(eK), np.sqrt(eV)
    if slices is None:
        return eQ.reshape(Q.shape), eK.reshape(K.shape), eV.reshape(V.shape)
    n = len(sl)
    return (eQ.reshape((n, d) + q_seq), eK.reshape((n, d) + k_seq), eV.reshape((n, vd) + k_seq))


# ----------------------------------------------------------------------------
# Algorithmic FLOP counts — allowed pairs from the rule
# ----------------------------------------------------------------------------
def allowed_pairs(prob: Problem, q_seq, k_seq) -> int:
    ev = _evaluator(prob, q_seq, k_seq)
    return int(sum(int(mk.sum()) for _, _, _, _, mk in _row_chunks(ev, ev.qo.size)))


def forward_flops(b, d, vd, pairs) -> float:
    return 2.0 * (d + vd) * pairs * b


def backward_flops(b, d, vd, pairs) -> float:
    return 2.0 * (3 * d + 2 * vd) * pairs * b


# ----------------------------------------------------------------------------
# CPU baseline: the reference's "naive TF attention" (tests/test_1d.py:69-76)
# restated in numpy fp32, one (b,h) slice at a time (bounded memory).
# ----------------------------------------------------------------------------
def naive_attention_slice_f32(q: np.ndarray, k: np.ndarray, v: np.ndarray, mask=None) -> np.ndarray:
    """q [d, nq], k [d, nk], v [vd, nk] -> o [vd, nq], all float32."""
    d = q.shape[0]
    logit = (q.T @ k) / np.float32(math.sqrt(d))
    if mask is not None:
        logit = np.where(mask, logit, np.finfo(np.float32).min)
    logit -= logit.max(axis=1, keepdims=True)
    p = np.exp(logit)
    p /= p.sum(axis=1, keepdims=True)
    if mask is not None:
        p = np.where(mask, p, np.float32(0))
    return v @ p.T


def naive_attention_backward_slice_f32(q, k, v, do, mask=None):
    """The gradients TF's autodiff takes through the naive graph of tests/test_1d.py:69-76
    (einsum -> where -> softmax -> where -> einsum), restated in numpy float32 for one slice:
    the CPU leg of a forward+backward step.  Recomputes P like the graph's saved activations
    would hold it.  q [d, nq], k [d, nk], v [vd, nk], do [vd, nq] -> (dq, dk, dv)."""
    d = q.shape[0]
    sc = np.float32(1.0 / math.sqrt(d))
    logit = (q.T @ k) * sc
    if mask is not None:
        logit = np.where(mask, logit, np.finfo(np.float32).min)
    logit -= logit.max(axis=1, keepdims=True)
    p = np.exp(logit)
    p /= p.sum(axis=1, keepdims=True)
    if mask is not None:
        p = np.where(mask, p, np.float32(0))
    dv = do @ p                                   # [vd, nk]
    dp = do.T @ v                                 # [nq, nk]
    ds = p * (dp - np.sum(dp * p, axis=1, keepdims=True)) * sc
    return k @ ds.T, q @ ds, dv


def forward_rows_f64(q, k, v, prob: Problem, q_seq, k_seq, r0: int, r1: int, k0: int = 0, k1=None):
    """Float64 forward of query rows [r0, r1) of ONE slice (q [d, nq], k [d, nk], v [vd, nk]):
    the same math as :func:`forward_f64`, for sequences too long to walk whole.  The rule is
    evaluated for those rows against keys [k0, k1) (default: every key); a caller narrows the
    range only where the rule provably allows nothing outside it (a 1d window around the rows).
    Returns (O [vd, r1-r0], L, M, has_any)."""
    ev = _evaluator(prob, q_seq, k_seq)
    d = q.shape[0]
    scale = 1.0 / math.sqrt(d)
    k1 = k.shape[1] if k1 is None else k1
    mk_full = np.zeros((r1 - r0, k.shape[1]), dtype=bool)
    mk_full[:, k0:k1] = ev.block(r0, r1, k0, k1)
    cols = np.nonzero(mk_full.any(axis=0))[0]
    ha = mk_full.any(axis=1)
    vd = v.shape[0]
    if cols.size == 0:
        return np.zeros((vd, r1 - r0)), np.zeros(r1 - r0), np.zeros(r1 - r0), ha
    c0, c1 = int(cols[0]), int(cols[-1]) + 1
    mk = mk_full[:, c0:c1]
    s = np.where(mk, (q[:, r0:r1].astype(np.float64).T @ k[:, c0:c1].astype(np.float64)) * scale, -np.inf)
    mrow = np.where(ha, s.max(axis=1), 0.0)
    p = np.exp(s - mrow[:, None])
    lrow = p.sum(axis=1)
    o = v[:, c0:c1].astype(np.float64) @ (p / np.where(ha, lrow, 1.0)[:, None]).T
    o[:, ~ha] = 0.0
    return o, np.where(ha, lrow, 0.0), mrow, ha
