"""CPU tests that pin the oracle (oracle/fa_oracle.py) before it is trusted.

* Sync maps vs the reference's published alignment examples
  (flash_attention.py:29-70 docstring, images/*_1d.jpg, *_2d.jpg) -> tests/golden/sync_examples.json
* Mask rules vs the reference's masking figure (images/masking_rule_examples.jpg)
  -> tests/golden/mask_examples.json
* Kernel rule formulation (flash_attention.h) == unit-test generator formulation
  (tests/test_base.py:33-67 + tests/test_1d.py / test_2d.py coordinates) on many shapes.
* Forward/backward numerics vs torch float64 autograd of the vanilla path
  (tests/test_1d.py:69-76), and vs the committed config-1 fixture.
"""

import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_sync_examples_match_reference_docstring():
    cases = json.load(open(os.path.join(GOLDEN, "sync_examples.json")))["cases"]
    for c in cases:
        qo, ko, _ = O.seq_orders(c["a_shape"], c["b_shape"], c["mode"])
        assert [int(ko[i]) for i in range(len(ko))] == [int(qo[j]) for j in c["b_aligned_to"]], c
        # symmetric roles: B as the query sequence
        qo2, ko2, _ = O.seq_orders(c["b_shape"], c["a_shape"], c["mode"])
        assert [int(x) for x in qo2] == [int(ko2[j]) for j in c["b_aligned_to"]], c


def test_mask_examples_match_reference_figure():
    cases = json.load(open(os.path.join(GOLDEN, "mask_examples.json")))["cases"]
    for c in cases:
        shape = [6] if c["dims"] == 1 else [6, 6]
        qi = 3 if c["dims"] == 1 else 3 * 6 + 3
        m = O.rule_mask(shape, shape, "none_front", c["policy"], c["window_size"], c["log2_stride_size"],
                        c["is_causal"])
        active = sorted(np.nonzero(m[qi])[0].tolist())
        expect = list(range(int(np.prod(shape)))) if c["active"] == "all" else c["active"]
        assert active == expect, c
        vm = O.vanilla_mask(shape, shape, "none_front", c["policy"], c["window_size"], c["log2_stride_size"],
                            c["is_causal"])
        assert (vm == m).all(), c


def _random_cases(seed, n, dims):
    rng = np.random.default_rng(seed)
    for _ in range(n):
        if dims == 1:
            qs = [int(rng.integers(1, 40))]
            ks = [int(rng.integers(1, 40))]
        else:
            qs = [int(rng.integers(1, 9)), int(rng.integers(1, 9))]
            ks = [int(rng.integers(1, 9)), int(rng.integers(1, 9))]
        yield qs, ks, str(rng.choice(O.SYNC_MODES)), int(rng.integers(1, 6)), int(rng.integers(0, 3)), bool(
            rng.integers(0, 2))


@pytest.mark.parametrize("dims", [1, 2])
def test_rule_formulations_agree(dims):
    """Kernel rule (pow-2 orders, shifts) == the unit-test generator (max_width orders, % and //)."""
    for qs, ks, mode, ws, ls, causal in _random_cases(7 + dims, 250, dims):
        for policy in ("full", "causal", "local"):
            a = O.rule_mask(qs, ks, mode, policy, ws, ls, causal)
            b = O.vanilla_mask(qs, ks, mode, policy, ws, ls, causal)
            assert (a == b).all(), (qs, ks, mode, policy, ws, ls, causal)


def test_reference_test_windows_are_trivial():
    """The reference tests set window = max(diff.shape) (test_base.py:54), i.e. local == full in 1d;
    documents why our suite adds small windows."""
    qs, ks = [37], [29]
    ws = max(qs[0], ks[0])
    assert (O.rule_mask(qs, ks, "none_front", "local", ws, 0, False) == O.rule_mask(qs, ks, "none_front", "full")).all()


def test_neg_inf_approx_bytes():
    for dt in (np.float16, np.float32, np.float64):
        v = O.neg_inf_approx(dt)
        assert np.array([v], dtype=dt).tobytes() == b"\xfa" * np.dtype(dt).itemsize
    assert float(O.neg_inf_approx(np.float16)) == -57152.0


def _vanilla_torch(Q, K, V, mask, seq_dims):
    """tests/test_1d.py:69-76 / test_2d.py:97-109 restated in torch float64 (flattened sequences)."""
    b = Q.shape[:-seq_dims - 1]
    d = Q.shape[-seq_dims - 1]
    q = Q.reshape(-1, d, mask.shape[0])
    k = K.reshape(-1, d, mask.shape[1])
    v = V.reshape(-1, V.shape[-seq_dims - 1], mask.shape[1])
    logit = torch.einsum("bcq,bck->bqk", q, k) / math.sqrt(d)
    mk = torch.from_numpy(mask)[None]
    logit = torch.where(mk, logit, torch.finfo(logit.dtype).min)
    p = torch.softmax(logit, dim=-1)
    p = torch.where(mk, p, torch.zeros((), dtype=p.dtype))
    o = torch.einsum("bqk,bck->bcq", p, v)
    return o.reshape(b + (v.shape[1],) + Q.shape[len(b) + 1:])


@pytest.mark.parametrize("seq_dims,policy,mode,ws,ls,causal", [
    (1, "full", "none_front", 1, 0, False),
    (1, "causal", "scale_front", 1, 0, False),
    (1, "causal", "scale_end", 1, 0, False),
    (1, "local", "none_front", 3, 0, False),
    (1, "local", "scale_end", 2, 1, True),
    (2, "full", "scale_front", 1, 0, False),
    (2, "causal", "scale_end", 1, 0, False),
    (2, "local", "none_front", 2, 1, False),
    (2, "local", "scale_front", 2, 0, True),
])
def test_oracle_forward_backward_vs_torch_autograd(seq_dims, policy, mode, ws, ls, causal):
    rng = np.random.default_rng(3)
    if seq_dims == 1:
        qs, ks = (23,), (17,)
    else:
        qs, ks = (5, 6), (3, 7)
    d, vd = 6, 5
    Q = rng.uniform(-2, 2, (2, d) + qs)
    K = rng.uniform(-2, 2, (2, d) + ks)
    V = rng.uniform(-2, 2, (2, vd) + ks)
    dO = rng.uniform(-2, 2, (2, vd) + qs)
    prob = O.Problem(policy, seq_dims, mode, ws, ls, causal)
    mask = O.problem_mask(prob, list(qs), list(ks))
    Ot, Lt, Mt, has_any = O.forward_f64(Q, K, V, prob)
    tq, tk, tv = (torch.tensor(x, requires_grad=True) for x in (Q, K, V))
    to = _vanilla_torch(tq, tk, tv, mask, seq_dims)
    np.testing.assert_allclose(Ot, to.detach().numpy(), rtol=1e-12, atol=1e-12)
    to.backward(torch.tensor(dO))
    dQ, dK, dV = O.backward_f64(Q, K, V, dO, prob)
    np.testing.assert_allclose(dQ, tq.grad.numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(dK, tk.grad.numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(dV, tv.grad.numpy(), rtol=1e-10, atol=1e-12)
    # l/m definitions: O = sum_k exp(s-m)/l * v  (flash_attention.cu:974-1035)
    Oo, lo, mo = O.forward(Q.astype(np.float64), K, V, prob)
    np.testing.assert_allclose(lo.reshape(2, -1)[:, has_any], Lt.reshape(2, -1)[:, has_any], rtol=1e-12)
    np.testing.assert_allclose(mo.reshape(2, -1)[:, has_any], Mt.reshape(2, -1)[:, has_any], rtol=0)


def test_fully_masked_rows_conventions():
    """Rows that attend nothing: O=0, l=0, m=0xFA bytes (flash_attention_forward.cc:352-365)."""
    prob = O.Problem("local", 2, "scale_end", 1, 2, True)
    qs, ks = (4, 6), (6, 4)
    mask = O.problem_mask(prob, list(qs), list(ks))
    empty = ~mask.any(axis=1)
    assert empty.any()
    rng = np.random.default_rng(0)
    for dt in (np.float16, np.float32, np.float64):
        Q = rng.uniform(-2, 2, (1, 3) + qs).astype(dt)
        K = rng.uniform(-2, 2, (1, 3) + ks).astype(dt)
        V = rng.uniform(-2, 2, (1, 2) + ks).astype(dt)
        Oo, lo, mo = O.forward(Q, K, V, prob)
        assert lo.dtype == (np.float32 if dt == np.float16 else dt)
        assert (Oo.reshape(1, 2, -1)[:, :, empty] == 0).all()
        assert (lo.reshape(1, -1)[:, empty] == 0).all()
        assert (mo.reshape(1, -1)[:, empty].tobytes() == b"\xfa" * (empty.sum() * np.dtype(dt).itemsize))


def test_config1_fixture_regression():
    """Config 1 (full_1d fp32 B=2 H=4 d=32 N=128): oracle == committed fixture (tests/golden/make_golden.py)."""
    f = np.load(os.path.join(GOLDEN, "config1_full1d_f32.npz"))
    prob = O.Problem("full", 1, "none_front")
    Oo, lo, mo = O.forward(f["Q"], f["K"], f["V"], prob)
    np.testing.assert_allclose(Oo, f["O"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(lo, f["l"], rtol=1e-6)
    np.testing.assert_array_equal(mo, f["m"])
    dQ, dK, dV = O.backward_f64(f["Q"], f["K"], f["V"], f["dO"], prob)
    np.testing.assert_allclose(dQ, f["dQ"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dK, f["dK"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dV, f["dV"], rtol=1e-6, atol=1e-6)


def test_flop_counts():
    # SURVEY.md §8d closed forms
    assert O.allowed_pairs(O.Problem("full", 1), [128], [128]) == 128 * 128
    assert O.allowed_pairs(O.Problem("causal", 1), [100], [100]) == 100 * 101 // 2
    n, ws = 300, 16
    assert O.allowed_pairs(O.Problem("local", 1, "none_front", ws), [n], [n]) == n * (2 * ws - 1) - ws * (ws - 1)


def test_naive_backward_matches_f64_backward():
    """The CPU baseline's fp32 naive backward (the autodiff of tests/test_1d.py:69-76) agrees with
    the float64 oracle's analytic gradients."""
    rng = np.random.default_rng(11)
    d, nq, nk = 16, 70, 90
    q, k, v, do = (rng.uniform(-2, 2, s).astype(np.float32) for s in ((d, nq), (d, nk), (d, nk), (d, nq)))
    prob = O.Problem("causal", 1, "scale_end")
    mask = O.problem_mask(prob, [nq], [nk])
    dq, dk, dv = O.naive_attention_backward_slice_f32(q, k, v, do, mask)
    rq, rk, rv = O.backward_f64(q[None], k[None], v[None], do[None], prob)
    for got, ref in ((dq, rq[0]), (dk, rk[0]), (dv, rv[0])):
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


def _bwd_f32_kernel_form(q, k, v, do):
    """fp32 gradients in the kernels' formulation (Q pre-scaled, D = rowsum(dO*O) from the rounded O)."""
    sc = np.float32(1.0 / math.sqrt(q.shape[0]))
    s = (q * sc).astype(np.float32).T @ k
    p = np.exp(s - s.max(axis=1, keepdims=True))
    p /= p.sum(axis=1, keepdims=True)
    D = np.sum(do * (v @ p.T), axis=0)
    ds = p * (do.T @ v - D[:, None])
    return (k @ ds.T) * sc, (q @ ds) * sc, do @ p


@pytest.mark.parametrize("d,vd,nq,nk,seed", [(48, 48, 504, 1, 0), (8, 48, 200, 1, 5), (3, 200, 80, 2, 1),
                                              (1, 128, 354, 2, 2), (16, 16, 70, 90, 3), (64, 64, 300, 300, 4)])
def test_gradient_rounding_scale_covers_fp32(d, vd, nq, nk, seed):
    """The gradient tolerance of the GPU parity tests (tests/test_gpu_parity.py: rtol/atol plus KAPPA x
    backward_rounding_scale_f64) holds for a plain fp32 computation of the gradients in the kernels'
    formulation, including the cancelling sums of a single key (dK analytically 0 from terms of size
    ~|dP|), where that computation exceeds the rtol/atol part alone (checked: the model is needed)."""
    from tests.test_gpu_parity import KAPPA, TOL, U_ROUND
    rng = np.random.default_rng(seed)
    q, k, v, do = (rng.uniform(-2, 2, s).astype(np.float32) for s in ((d, nq), (d, nk), (vd, nk), (vd, nq)))
    prob = O.Problem("full", 1, "none_front")
    got = _bwd_f32_kernel_form(q, k, v, do)
    ref = O.backward_f64(q[None], k[None], v[None], do[None], prob)
    esc = O.backward_rounding_scale_f64(q[None], k[None], v[None], do[None], prob, *U_ROUND[np.float32])
    rtol, atol = TOL[np.float32]["bwd"]
    base_ok = []
    for g, r, e in zip(got, ref, esc):
        r, e = r[0], e[0]
        base = atol * max(np.abs(r).max(), 1.0) + rtol * np.abs(r)
        assert (np.abs(g - r) <= base + KAPPA * e).all(), np.max(np.abs(g - r) / (base + KAPPA * e))
        base_ok.append(bool((np.abs(g - r) <= base).all()))
    if nk == 1:
        assert not base_ok[1]   # dK of a single key: rtol/atol alone rejects a correct fp32 result


def test_forward_rows_matches_forward():
    """forward_rows_f64 (row ranges of one long slice) equals forward_f64 on those rows."""
    rng = np.random.default_rng(12)
    d, nq, nk = 8, 300, 260
    q, k, v = (rng.uniform(-2, 2, s) for s in ((d, nq), (d, nk), (d, nk)))
    prob = O.Problem("local", 1, "scale_front", 37, 0, True)
    Of, Lf, Mf, haf = O.forward_f64(q[None], k[None], v[None], prob)
    for r0, r1 in ((0, 5), (100, 180), (290, 300)):
        o, l, m, ha = O.forward_rows_f64(q, k, v, prob, [nq], [nk], r0, r1)
        np.testing.assert_allclose(o, Of[0][:, r0:r1], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(l, Lf[0][r0:r1], rtol=1e-12)
        np.testing.assert_allclose(m, Mf[0][r0:r1], rtol=1e-12)
        assert (ha == haf[r0:r1]).all()
