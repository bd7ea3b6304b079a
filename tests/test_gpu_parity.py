"""GPU parity: the HIP path (through the C ABI, via the reference-API mirror) vs
the float64 oracle on identical dtype-rounded inputs.

Tolerances (stated here, checked per element: |got - ref| <= ATOL*S + RTOL*|ref|, with
S = max(max|ref|, 1): inputs are U(-2,2), so 1 is the natural magnitude floor for
outputs that vanish analytically, e.g. dQ when a row attends a single key):
  fp16: forward O rtol 1e-3 / atol 1e-3*max|O|  (BASELINE.json north_star rtol=1e-3);
        backward rtol 1e-3 / atol 2e-3*max|grad|
  fp32: rtol 1e-5 / atol 1e-5*max  (north_star rtol=1e-5)
  fp64: rtol 1e-10 / atol 1e-10*max
l is checked with the same rtol (l for fp16 is fp32), m to two units in the last
place of T (it is the rounded row max) — for fp16 plus rtol 1e-3 / atol 1e-3*max(|m|,1),
since the fp16 kernel scores with Q pre-scaled by scale*log2(e) in fp16; for fp32 / fp64 plus
1e-6*|m| and the larger of 1e-6 (1e-12) and 2 eps of the score's rounding bound scale*|q|_1*max|k|.
Gradients add KAPPA x the oracle's per-element rounding scale (capped in fp16 where the element does
not cancel) and must pass the whole-gradient scale-slope check (tests/gate.py).
The reference's own gate (rtol=atol=1e-3*N for fp16, 1e-6*N otherwise, N the K or Q entries;
tests/test_base.py:198-226) is far looser at its tests' sizes; at N < 10 it is tighter than any
of these and would reject a correct fp32 dQ of one or two keys (an analytic 0 formed from
dP - D at ~1e-5), so it is not used as a cap.  Rows that attend nothing must be exactly O=0, l=0,
m=bytes 0xFA.
"""

import json
import math
import os
import zlib

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu

# TOL, U_ROUND, KAPPA and the gradient bound live in tests/gate.py (one definition for these tests and
# for the CPU checks of the gate itself, tests/test_gate_mutations.py)
from tests.gate import KAPPA, TOL, U_ROUND  # noqa: E402
from tests import gate  # noqa: E402
TORCH = {np.float16: torch.float16, np.float32: torch.float32, np.float64: torch.float64}


def _fa():
    from tf_flash_attention_amd import flash_attention as fa
    return fa


def _close(name, got, ref, rtol, atol_rel, extra=0.0):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    scale = max(float(np.max(np.abs(ref))) if ref.size else 0.0, 1.0)
    atol = atol_rel * scale
    err = np.abs(got - ref)
    bad = err > atol + rtol * np.abs(ref) + extra
    assert np.isfinite(got).all(), f"{name}: non-finite output"
    assert not bad.any(), (f"{name}: {bad.sum()} / {bad.size} elements off; max abs err {err.max():.3e}, "
                           f"max|ref| {scale:.3e}, worst idx {np.unravel_index(np.argmax(err - rtol * np.abs(ref)), err.shape)}")
    return float(err.max() / max(scale, 1e-30))


def _call(policy, seq_dims, tq, tk, tv, mode, ws, ls, causal):
    fa = _fa()
    if policy == "full":
        f = fa.full_1d if seq_dims == 1 else fa.full_2d
        return f(tq, tk, tv, sync_mode=mode, returning_l_m=True)
    if policy == "causal":
        f = fa.causal_1d if seq_dims == 1 else fa.causal_2d
        return f(tq, tk, tv, mode, returning_l_m=True)
    f = fa.local_1d if seq_dims == 1 else fa.local_2d
    return f(tq, tk, tv, ws, ls, causal, mode, returning_l_m=True)


def _to_dev(x, dev, bwd, misalign):
    t = torch.from_numpy(x).to(dev)
    if misalign:  # same values at a data pointer one element past an aligned allocation
        buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=dev)
        buf[1:].copy_(t.reshape(-1))
        t = buf[1:].view(t.shape)
        assert t.is_contiguous() and t.data_ptr() % 16 != 0
    return t.requires_grad_(bwd)


def run_case(dtype, policy, seq_dims, mode, batch, d, vd, qs, ks, ws=1, ls=0, causal=False, seed=0, bwd=True,
             slices=None, inputs=None, misalign=False):
    rng = np.random.default_rng(seed)
    qs, ks = tuple(qs), tuple(ks)
    if inputs is None:
        Q = rng.uniform(-2, 2, tuple(batch) + (d,) + qs).astype(dtype)
        K = rng.uniform(-2, 2, tuple(batch) + (d,) + ks).astype(dtype)
        V = rng.uniform(-2, 2, tuple(batch) + (vd,) + ks).astype(dtype)
        dO = rng.uniform(-2, 2, tuple(batch) + (vd,) + qs).astype(dtype)
    else:
        Q, K, V, dO = inputs
    dev = torch.device("cuda:0")
    tq, tk, tv = (_to_dev(x, dev, bwd, misalign) for x in (Q, K, V))
    o, l, m = _call(policy, seq_dims, tq, tk, tv, mode, ws, ls, causal)
    if bwd:
        o.backward(torch.from_numpy(dO).to(dev))
    torch.cuda.synchronize()
    prob = O.Problem(policy, seq_dims, mode, ws, ls, causal)
    b = int(np.prod(batch))
    flat = lambda x: x.reshape((b,) + x.shape[len(batch):])  # noqa: E731
    sl = list(range(b)) if slices is None else list(slices)
    Qf, Kf, Vf, dOf = flat(Q), flat(K), flat(V), flat(dO)
    O64, L64, M64, has_any = O.forward_f64(Qf, Kf, Vf, prob, slices=sl)
    rtol, atol = TOL[dtype]["fwd"]
    og = flat(o.detach().cpu().numpy())[sl]
    res = {"O": _close("O", og, O64, rtol, atol)}
    # l, m
    nq = int(np.prod(qs))
    lg = flat(l.cpu().numpy()).reshape(b, nq)[sl].astype(np.float64)
    mg = flat(m.cpu().numpy()).reshape(b, nq)[sl]
    M64 = M64.reshape(len(sl), nq)
    L64 = L64.reshape(len(sl), nq)
    ha = has_any
    if ha.any():
        m_f = mg[:, ha].astype(np.float64)
        ulp = np.abs(np.spacing(np.abs(M64[:, ha]).astype(dtype))).astype(np.float64)
        # m: 2 ulp of T, plus (fp16) the same rtol/atol-with-floor-1 as the other outputs — the
        # fp16 kernel forms its scores from Q pre-scaled by scale*log2(e) in fp16 (~1e-4 abs)
        # fp32 / fp64: m is a score, a d-term dot product rounded in T (Q pre-scaled, then the MFMA's
        # fma chain), so its absolute error scales with scale·Σ|q_c·k_c| <= scale·|q|_1·max|k|, not
        # with |m| (a row max near 0 can come from large, cancelling terms); allow 2 units of T's
        # rounding of that bound
        eps = float(np.finfo(dtype).eps)
        qn1 = np.abs(Qf[sl].astype(np.float64)).sum(axis=1).reshape(len(sl), nq)[:, ha]
        kmax = max(float(np.abs(Kf[sl]).max()), 1e-30)
        dot_bound = qn1 * kmax / math.sqrt(d)
        # fp16: the kernels score with Q·scale·log2(e) rounded to fp16 (relative error <= 2^-11 per
        # element), so a score may sit up to 2^-11·scale·Σ_c|q_c·k_c| from the exact one (plus the f32
        # accumulation, <= d·2^-24 of the same sum), and the row max up to the largest of these over the
        # row's allowed keys (round 6: per key, not |q|_1·max|k|, about half as wide at d = 32);
        # plus the packed-P max approximation (< 4.9e-4); that bound matters at the
        # reference's own shapes (N up to 4096, d = 8..32) for rows whose max is small
        if dtype == np.float16:
            rowdot = gate.max_abs_dot(Qf[sl].reshape(len(sl), d, nq), Kf[sl].reshape(len(sl), d, -1),
                                      O.problem_mask(prob, qs, ks))[:, ha] / math.sqrt(d)
            f16_dot = (2.0 ** -11 + d * 2.0 ** -24) * rowdot + 4.9e-4
        m_tol = 2 * ulp + (np.maximum(1e-3 * np.maximum(np.abs(M64[:, ha]), 1.0), f16_dot)
                           if dtype == np.float16
                           else 1e-6 * np.abs(M64[:, ha]) + np.maximum(1e-6 if dtype != np.float64 else 1e-12,
                                                                      2 * eps * dot_bound))
        assert (np.abs(m_f - M64[:, ha]) <= m_tol).all(), f"m: max err {np.abs(m_f - M64[:, ha]).max():.3e}"
        l_ref = L64[:, ha] * np.exp(M64[:, ha] - m_f)    # relative to the stored m
        _close("l", lg[:, ha], l_ref, max(rtol, 1e-6 if dtype == np.float16 else rtol), atol)
    if (~ha).any():
        assert (og.reshape(len(sl), vd, nq)[:, :, ~ha] == 0).all()
        assert (lg[:, ~ha] == 0).all()
        assert mg[:, ~ha].tobytes() == b"\xfa" * (mg[:, ~ha].size * np.dtype(dtype).itemsize)
    if bwd:
        dQ, dK, dV = O.backward_f64(Qf, Kf, Vf, dOf, prob, slices=sl)
        eQ, eK, eV = O.backward_rounding_scale_f64(Qf, Kf, Vf, dOf, prob, *U_ROUND[dtype], slices=sl)
        rtol, atol = TOL[dtype]["bwd"]
        grads = {"dQ": (flat(tq.grad.cpu().numpy())[sl], dQ, eQ), "dK": (flat(tk.grad.cpu().numpy())[sl], dK, eK),
                 "dV": (flat(tv.grad.cpu().numpy())[sl], dV, eV)}
        stats_file = os.environ.get("FA_GATE_STATS")
        if stats_file:  # gate statistics for DESIGN §4 (not part of the verdict)
            with open(stats_file, "a") as f:
                for name, (got, ref, e) in grads.items():
                    st = gate.grad_stats(got, ref, e, dtype)
                    st.update(grad=name, dtype=np.dtype(dtype).name, policy=policy, seq_dims=seq_dims, d=d, vd=vd,
                              qs=list(qs), ks=list(ks), seed=seed)
                    f.write(json.dumps(st) + "\n")
        for name, (got, ref, e) in grads.items():
            res[name] = _close(name, got, ref, rtol, atol, gate.grad_extra(ref, e, dtype))
            # whole-gradient scale: catches a defect scaling a gradient by ~2^-8 in fp16 that the
            # per-element bound cannot see (tests/gate.py, tests/test_gate_mutations.py)
            ch = got.shape[1]  # [batch, channels, positions...]: the channels of one row
            assert gate.slope_ok(got, ref, e, dtype, d, ch), (
                f"{name}: scale slope {gate.scale_slope(got, ref):.3e} > "
                f"{gate.slope_tol_eff(ref, e, dtype, d, ch):.3e}")
    return res


DTYPES = [np.float16, np.float32, np.float64]


# ---------------------------------------------------------------- config 1
def test_config1_fixture():
    import os
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1_full1d_f32.npz"))
    fa = _fa()
    dev = torch.device("cuda:0")
    tq, tk, tv = (torch.from_numpy(f[n]).to(dev).requires_grad_(True) for n in ("Q", "K", "V"))
    o, l, m = fa.full_1d(tq, tk, tv, returning_l_m=True)
    o.backward(torch.from_numpy(f["dO"]).to(dev))
    _close("O", o.detach().cpu().numpy(), f["O"], 1e-5, 1e-5)
    _close("l", l.cpu().numpy(), f["l"], 1e-5, 1e-5)
    _close("m", m.cpu().numpy(), f["m"], 1e-5, 1e-6)
    for g, n in ((tq.grad, "dQ"), (tk.grad, "dK"), (tv.grad, "dV")):
        _close(n, g.cpu().numpy(), f[n], 1e-5, 1e-5)


# ------------------------------------------ the reference's test matrix
# 15 registered cases + the unregistered CausalAttentionSyncModeNoneFront (tests/test_base.py:314-385)
REF_CASES = [
    ("full", "none_front", False, False),
    ("causal", "none_front", False, False),
    ("causal", "scale_front", False, False),
    ("causal", "scale_end", False, False),
] + [("local", mode, stride, causal) for stride, causal in ((False, False), (True, False), (False, True), (True, True))
     for mode in ("none_front", "scale_front", "scale_end")]


def _ref_window(seq_dims, qs, ks, stride):
    # VanillaLocalPolicy: window = max(diff.shape) (tests/test_base.py:54-58)
    window = max((1,) + tuple(qs) + tuple(ks) + (seq_dims,))
    ls = int(np.log2(window)) if stride else 0
    return window, ls


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("seq_dims", [1, 2])
@pytest.mark.parametrize("case", REF_CASES, ids=lambda c: f"{c[0]}-{c[1]}-s{int(c[2])}-c{int(c[3])}")
def test_reference_matrix(dtype, seq_dims, case):
    policy, mode, stride, causal = case
    rng = np.random.default_rng(zlib.crc32(repr((seq_dims,) + case).encode()))
    d = int(rng.integers(8, 33))
    if seq_dims == 1:
        qs = (int(rng.integers(40, 400)),)
        ks = (int(rng.integers(40, 400)),)
        if dtype == np.float16:  # fp16 tests round the last seq dim to even (test_base.py:148-149)
            qs, ks = (qs[0] // 2 * 2,), (ks[0] // 2 * 2,)
    else:
        qs = (int(rng.integers(4, 20)), int(rng.integers(4, 20)))
        ks = (int(rng.integers(4, 20)), int(rng.integers(4, 20)))
    ws, ls = _ref_window(seq_dims, qs, ks, stride)
    run_case(dtype, policy, seq_dims, mode, (1, 3), d, d, qs, ks, ws, ls, causal, seed=1)


# The same 16-case matrix at the reference's own shape ranges (tests/test_1d.py:57-66,
# tests/test_2d.py:85-94): [B, H, C, *seq] from [1, 8, 8, 256] to [1, 8, 32, N_max] in 1d with
# N_max = 4096 / 2048 / 1024 for fp16 / fp32 / fp64, and from [1, 8, 8, 16, 16] to
# [1, 8, 32, 64, 64] / [.., 32, 64] / [.., 32, 32] in 2d.  Two draws per case, as the reference's
# test_base.py:148-176 makes them: 'max' (Q = K = V = the max shape) and 'random' (C and the K
# sequence drawn in range, the Q sequence drawn separately, so Nq != Nk; fp16 rounds the last
# sequence dim to even).  The oracle checks the first and last of the 8 slices.
REF_SHAPES = {
    1: {np.float16: (256, 4096), np.float32: (256, 2048), np.float64: (256, 1024)},
    2: {np.float16: ((16, 16), (64, 64)), np.float32: ((16, 16), (32, 64)), np.float64: ((16, 16), (32, 32))},
}


def _ref_draw(dtype, seq_dims, case, draw):
    if draw == "max":
        mx = REF_SHAPES[seq_dims][dtype][1]
        qs = ks = (mx,) if seq_dims == 1 else tuple(mx)
        return 32, qs, ks
    rng = np.random.default_rng(zlib.crc32(repr((np.dtype(dtype).name, seq_dims) + case).encode()))
    lo, hi = REF_SHAPES[seq_dims][dtype]
    lo, hi = ((lo,), (hi,)) if seq_dims == 1 else (lo, hi)
    d = int(rng.integers(8, 33))
    ks = tuple(int(rng.integers(a, b + 1)) for a, b in zip(lo, hi))
    qs = tuple(int(rng.integers(a, b + 1)) for a, b in zip(lo, hi))
    if dtype == np.float16:
        ks, qs = ks[:-1] + (ks[-1] // 2 * 2,), qs[:-1] + (qs[-1] // 2 * 2,)
    return d, qs, ks


@pytest.mark.parametrize("draw", ["max", "random"])
@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("seq_dims", [1, 2])
@pytest.mark.parametrize("case", REF_CASES, ids=lambda c: f"{c[0]}-{c[1]}-s{int(c[2])}-c{int(c[3])}")
def test_reference_matrix_reference_shapes(draw, dtype, seq_dims, case):
    policy, mode, stride, causal = case
    d, qs, ks = _ref_draw(dtype, seq_dims, case, draw)
    ws, ls = _ref_window(seq_dims, qs, ks, stride)
    run_case(dtype, policy, seq_dims, mode, (1, 8), d, d, qs, ks, ws, ls, causal, seed=2, slices=[0, 7])


# ------------------------------------------------- small windows / strides
@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("seq_dims,qs,ks", [(1, (300,), (300,)), (1, (257,), (130,)), (1, (130,), (517,)),
                                            (2, (12, 13), (12, 13)), (2, (16, 8), (8, 16))])
@pytest.mark.parametrize("ws,ls,causal", [(1, 0, False), (2, 0, False), (8, 0, True), (37, 0, False), (2, 1, True),
                                          (3, 3, False)])
@pytest.mark.parametrize("mode", ["none_front", "scale_end"])
def test_small_windows(dtype, seq_dims, qs, ks, ws, ls, causal, mode):
    run_case(dtype, "local", seq_dims, mode, (2,), 16, 16, qs, ks, ws, ls, causal, seed=ws + ls)


# ------------------------------------------- fp16 / fp32 MFMA-path shapes
@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("policy", ["full", "causal", "local"])
@pytest.mark.parametrize("nq,nk", [(256, 256), (320, 192), (130, 1000)])
def test_f16_mfma_shapes(d, policy, nq, nk):
    run_case(np.float16, policy, 1, "none_front", (2, 2), d, d, (nq,), (nk,), ws=33, ls=0, causal=False, seed=d)


# fp16 streamlined forward / two-pass backward (d in {64, 128}, nq % 8 == nk % 8 == 0): ragged
# last tiles on both axes, every interval rule, sync maps, and 2d causal orders
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("policy,ws,causal,seq_dims,mode,qs,ks", [
    ("full", 1, False, 1, "none_front", (264,), (136,)),
    ("causal", 1, False, 1, "none_front", (392,), (392,)),
    ("causal", 1, False, 1, "scale_end", (200,), (520,)),
    ("local", 33, False, 1, "none_front", (456,), (456,)),
    ("local", 70, True, 1, "scale_front", (240,), (480,)),
    ("causal", 1, False, 2, "scale_front", (8, 24), (16, 16)),
    ("full", 1, False, 2, "none_front", (16, 16), (8, 40)),
])
def test_f16_fast_paths(d, policy, ws, causal, seq_dims, mode, qs, ks):
    run_case(np.float16, policy, seq_dims, mode, (2, 2), d, d, qs, ks, ws=ws, ls=0, causal=causal, seed=d + ws)


# the two-pass fp16 backward beyond the interval rules and aligned lengths: strided and 2d local
# windows (per-element order check), lengths that are not multiples of 8 and data pointers that are
# not 16-B aligned (element-wise staging), at the MFMA tile sizes
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("policy,ws,ls,causal,seq_dims,mode,qs,ks,misalign", [
    ("local", 20, 2, False, 1, "none_front", (520,), (520,), False),
    ("local", 9, 1, True, 1, "scale_front", (300,), (600,), False),
    ("local", 5, 0, False, 2, "none_front", (24, 20), (24, 20), False),
    ("local", 3, 1, True, 2, "scale_end", (16, 24), (20, 12), False),
    ("full", 1, 0, False, 1, "none_front", (263,), (517,), False),
    ("causal", 1, 0, False, 1, "scale_end", (333,), (199,), False),
    ("local", 45, 0, False, 1, "none_front", (301,), (301,), False),
    ("full", 1, 0, False, 1, "none_front", (256,), (192,), True),
    ("local", 7, 1, False, 2, "scale_front", (15, 17), (13, 19), True),
])
def test_f16_fast_bwd_general(d, policy, ws, ls, causal, seq_dims, mode, qs, ks, misalign):
    run_case(np.float16, policy, seq_dims, mode, (2, 2), d, d, qs, ks, ws=ws, ls=ls, causal=causal, seed=d + ws + ls,
             misalign=misalign)


# channel counts below the kernel's D (zero-padded rows) and d != v_d on the streamlined paths
@pytest.mark.parametrize("d,vd", [(96, 96), (40, 64), (64, 48), (128, 72), (33, 100)])
@pytest.mark.parametrize("policy", ["full", "causal"])
def test_f16_fast_paths_padded_channels(d, vd, policy):
    run_case(np.float16, policy, 1, "none_front", (2,), d, vd, (200,), (136,), seed=d + vd)


@pytest.mark.parametrize("d", [16, 32, 48, 64, 96, 128])
@pytest.mark.parametrize("policy", ["full", "causal", "local"])
@pytest.mark.parametrize("nq,nk", [(256, 256), (130, 1001)])
def test_f32_mfma_shapes(d, policy, nq, nk):
    run_case(np.float32, policy, 1, "scale_end", (2, 1), d, d, (nq,), (nk,), ws=41, ls=0, causal=True, seed=d + 1)


# fp64 MFMA path (fa_f64.hip): forward any d, v_d <= 128, backward d, v_d <= 64 (generic above)
@pytest.mark.parametrize("d", [16, 32, 48, 64, 96, 128])
@pytest.mark.parametrize("policy", ["full", "causal", "local"])
@pytest.mark.parametrize("nq,nk", [(256, 256), (130, 1001)])
def test_f64_mfma_shapes(d, policy, nq, nk):
    run_case(np.float64, policy, 1, "scale_front", (2, 1), d, d, (nq,), (nk,), ws=41, ls=0, causal=True, seed=d + 2)


# 1d local bands at MFMA sizes: the interval-rule path (per-lane key interval, empty tiles skipped)
@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("ws,causal", [(64, False), (100, True), (256, False), (300, True)])
@pytest.mark.parametrize("mode,nq,nk", [("none_front", 1500, 1500), ("scale_front", 700, 1500),
                                        ("scale_end", 1500, 600)])
def test_local_band_mfma(dtype, ws, causal, mode, nq, nk):
    run_case(dtype, "local", 1, mode, (2,), 64, 64, (nq,), (nk,), ws, 0, causal, seed=ws)


# the persistent band forward (fa_fwd_f16_band.hip: fp16 1d local, ls = 0, d <= 64 = v_d, nq % 8 == 0):
# workgroups that walk several items across slice boundaries (more items than CUs), ragged last
# blocks, nq != nk under the scale maps, causal windows, the smallest and widest windows it takes
@pytest.mark.parametrize("batch,nq,nk,ws,causal,mode,d", [
    ((5, 13), 1024, 1024, 96, False, "none_front", 64),
    ((3, 40), 2048, 2048, 256, False, "none_front", 64),
    ((7, 41), 1000, 1000, 1, False, "none_front", 64),
    ((2, 150), 776, 1552, 130, True, "scale_front", 48),
    ((300,), 1552, 520, 40, False, "scale_end", 64),
    ((2, 131), 1024, 1024, 700, True, "none_front", 64),
    # the wider item instances (positions per item T = 17 and 21 of 9 / 13 / 17 / 21)
    ((2, 9), 2048, 2048, 500, False, "none_front", 64),
    ((3, 5), 2048, 2048, 600, False, "none_front", 64),
    # small windows with nq not a multiple of the 256-query block: the first item's wave-pair
    # ranges start at key tiles below 0 (zero-filled loads, dummy stagger entries, class-0 tiles)
    ((3, 7), 1000, 1000, 40, False, "none_front", 64),
    ((3, 7), 1000, 1000, 40, True, "none_front", 64),
    ((4, 5), 264, 264, 8, False, "none_front", 64),
    ((4, 5), 264, 264, 8, True, "none_front", 64),
    ((2, 3), 1000, 1000, 40, True, "scale_front", 64),
])
def test_band_forward_persistent(batch, nq, nk, ws, causal, mode, d):
    b = int(np.prod(batch))
    run_case(np.float16, "local", 1, mode, batch, d, 64, (nq,), (nk,), ws, 0, causal, seed=ws + b,
             slices=sorted({0, 1, b // 3, b // 2 + 1, b - 2, b - 1}))


@pytest.mark.parametrize("causal,ws", [(False, 100), (True, 77)])
def test_band_edge_mask_large_scores(causal, ws):
    """The band kernel's arithmetic edge mask (fa_fwd_f16_band.hip: min(s, ±(..)·2^100), rows never
    seeded below -2^98) with scores near -3.7e5 in log2 units, past the round-3 constants (2^20 /
    -2^18), where a row whose allowed scores all sat below the floor came back as O = 0.  Q and K are
    constant, so every allowed score is the same and O is the mean of V over each row's window for
    any rounding; m overflows fp16 there (as the reference's would), so only O is compared."""
    fa = _fa()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7 + ws)
    b, d, n = 3, 64, 1024
    Q = np.full((b, d, n), 180.0, np.float16)
    K = np.full((b, d, n), -180.0, np.float16)
    V = rng.uniform(-2, 2, (b, d, n)).astype(np.float16)
    o, l, m = fa.local_1d(*(torch.from_numpy(x).to(dev) for x in (Q, K, V)), ws, 0, causal, "none_front",
                          returning_l_m=True)
    torch.cuda.synchronize()
    prob = O.Problem("local", 1, "none_front", ws, 0, causal)
    O64, _, _, ha = O.forward_f64(Q, K, V, prob)
    assert ha.all()
    _close("O", o.cpu().numpy(), O64, *TOL[np.float16]["fwd"])


@pytest.mark.parametrize("d,vd", [(64, 32), (24, 64), (100, 100), (7, 3)])
def test_odd_channels(d, vd):
    for dt in DTYPES:
        run_case(dt, "causal", 1, "scale_front", (1, 2), d, vd, (150,), (75,), seed=d)


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("d,vd", [(160, 160), (256, 256), (130, 300), (520, 72), (300, 1030)])
@pytest.mark.parametrize("policy,ws,causal", [("full", 1, False), ("causal", 1, False), ("local", 40, True)])
def test_wide_channels(dtype, d, vd, policy, ws, causal):
    """Channel counts past 128: the MFMA kernels up to 256 channels (fp16 for aligned tensors, fp32 and
    fp64 always), the resident / channel-chunked generic kernels past that (the reference has no fixed
    channel cap either: its key tile is sized from shared memory, flash_attention.cu:1977-2067)."""
    run_case(dtype, policy, 1, "scale_front", (2,), d, vd, (97,), (150,), ws=ws, causal=causal, seed=d + vd)


# fp16 forward for 128 < max(d, v_d) <= 256 on MFMA (fa_fwd_f16_wide.hip, 16-B chunk staging: full and
# interval rules, nk % 8 == 0, aligned K / V): several key tiles, ragged query blocks, d != v_d, every
# sync mode
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (130, 200), (200, 64), (64, 256)])
@pytest.mark.parametrize("policy,mode,qs,ks,ws,causal", [
    ("full", "none_front", (300,), (520,), 1, False),
    # square causal, nk % 8 == 0 with a ragged query block: the wide MFMA kernel itself (heaviest
    # blocks first, diagonal edge tiles on every block); 777 (nk % 8 != 0): its element-wise staging
    ("causal", "none_front", (776,), (776,), 1, False),
    ("causal", "none_front", (777,), (777,), 1, False),
    ("causal", "scale_end", (200,), (520,), 1, False),
    ("local", "scale_front", (240,), (480,), 70, True),
    ("local", "none_front", (700,), (704,), 33, False),
])
def test_wide_channels_mfma_forward(d, vd, policy, mode, qs, ks, ws, causal):
    run_case(np.float16, policy, 1, mode, (2,), d, vd, qs, ks, ws=ws, causal=causal, bwd=False, seed=d + 3 * vd)


# fp32 forward for 128 < max(d, v_d) <= 256 on MFMA (fa_fwd_f32_wide.hip: 32-key tiles, every rule, any
# alignment and length)
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (130, 200), (200, 64), (64, 256)])
@pytest.mark.parametrize("policy,seq,mode,qs,ks,ws,ls,causal", [
    ("full", 1, "none_front", (300,), (517,), 1, 1, False),
    ("causal", 1, "scale_end", (203,), (520,), 1, 1, False),
    ("local", 1, "scale_front", (240,), (481,), 70, 1, True),
    ("local", 2, "none_front", (13, 22), (13, 22), 5, 3, True),
])
def test_wide_channels_mfma_forward_f32(d, vd, policy, seq, mode, qs, ks, ws, ls, causal):
    run_case(np.float32, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal, bwd=False,
             seed=d + 7 * vd)


# fp32 backward for 128 < max(d, v_d) <= 256 on MFMA (fa_bwd_f32_wide.hip: 16x16x4 MFMAs, 16 keys /
# queries a wave; every rule, any alignment and length)
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (130, 200), (200, 64), (64, 256)])
@pytest.mark.parametrize("policy,seq,mode,qs,ks,ws,ls,causal", [
    ("full", 1, "none_front", (131,), (197,), 1, 1, False),
    ("causal", 1, "scale_end", (150,), (75,), 1, 1, False),
    ("local", 1, "scale_front", (120,), (241,), 40, 1, True),
    ("local", 2, "none_front", (9, 14), (9, 14), 4, 2, True),
])
def test_wide_channels_mfma_backward_f32(d, vd, policy, seq, mode, qs, ks, ws, ls, causal):
    run_case(np.float32, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal, seed=d + 11 * vd)


# fp64 forward + backward for 128 < max(d, v_d) <= 256 on MFMA (fa_f64.hip: four waves of 16 queries /
# keys, 16-column tiles, dK / dV in channel quarters and dQ in halves per launch; every rule, any
# alignment and length)
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (130, 200), (200, 64), (64, 256)])
@pytest.mark.parametrize("policy,seq,mode,qs,ks,ws,ls,causal", [
    ("full", 1, "none_front", (131,), (197,), 1, 1, False),
    ("causal", 1, "scale_end", (150,), (75,), 1, 1, False),
    ("local", 1, "scale_front", (120,), (241,), 40, 1, True),
    ("local", 1, "none_front", (150,), (150,), 20, 3, False),
    ("local", 2, "none_front", (9, 14), (9, 14), 4, 2, True),
])
def test_wide_channels_mfma_f64(d, vd, policy, seq, mode, qs, ks, ws, ls, causal):
    run_case(np.float64, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal, seed=d + 13 * vd)


# fp16 backward for 128 < max(d, v_d) <= 256 on MFMA (fa_bwd_f16_fast.hip launch_bwd_wide: the one-wave
# dK / dV and dQ passes at D = 256, two 128-channel output chunks per slice; aligned tensors, lengths
# multiples of 8, every rule incl. 2-D windows)
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (136, 256), (256, 64), (72, 200)])
@pytest.mark.parametrize("policy,seq,mode,qs,ks,ws,ls,causal", [
    ("full", 1, "none_front", (264,), (520,), 1, 1, False),
    ("causal", 1, "none_front", (392,), (392,), 1, 1, False),
    ("causal", 1, "scale_end", (200,), (520,), 1, 1, False),
    ("local", 1, "scale_front", (240,), (480,), 70, 1, True),
    ("local", 2, "none_front", (16, 24), (16, 24), 5, 3, True),
])
def test_wide_channels_mfma_backward(d, vd, policy, seq, mode, qs, ks, ws, ls, causal):
    run_case(np.float16, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal, seed=d + 5 * vd)


# fp16 forward + backward for 128 < max(d, v_d) <= 256 on MFMA in the shapes the 16-B chunk staging
# does not take (round 5; they ran on the SIMT kernels before): lengths not multiples of 8 and
# misaligned tensors (element-wise staging: fa_fwd_f16_wide.hip ALN = false, the four-role backward
# passes' ALN = false instances), and the rules that are not intervals (strided 1d and 2d local
# windows: POL 2, per-element order checks on the edge tiles)
@pytest.mark.parametrize("d,vd", [(256, 256), (160, 160), (200, 64)])
@pytest.mark.parametrize("policy,seq,mode,qs,ks,ws,ls,causal,misalign", [
    ("full", 1, "none_front", (131,), (197,), 1, 0, False, False),
    ("causal", 1, "scale_end", (150,), (75,), 1, 0, False, False),
    ("causal", 1, "none_front", (264,), (264,), 1, 0, False, True),
    ("local", 1, "scale_front", (203,), (405,), 30, 0, True, False),
    ("local", 1, "none_front", (150,), (150,), 20, 3, False, False),
    ("local", 1, "none_front", (256,), (256,), 40, 2, True, False),
    ("local", 2, "none_front", (9, 14), (9, 14), 4, 2, True, False),
    ("local", 2, "none_front", (16, 24), (16, 24), 5, 0, False, False),
])
def test_wide_channels_mfma_general(d, vd, policy, seq, mode, qs, ks, ws, ls, causal, misalign):
    run_case(np.float16, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal,
             seed=d + 17 * vd + ls, misalign=misalign)


# the same paths at their edges: fewer keys than one 16-B chunk, one query, fully masked rows (causal
# scale_end with nq > nk), 129 channels, and a 2d window grid larger than a key tile
@pytest.mark.parametrize("d,vd,policy,seq,mode,qs,ks,ws,ls,causal", [
    (256, 256, "full", 1, "none_front", (37,), (5,), 1, 0, False),
    (129, 129, "causal", 1, "none_front", (1,), (77,), 1, 0, False),
    (200, 160, "causal", 1, "scale_end", (300,), (100,), 1, 0, False),
    (256, 256, "local", 2, "scale_front", (21, 26), (42, 52), 6, 1, True),
    (160, 256, "local", 1, "none_front", (519,), (519,), 64, 5, True),
])
def test_wide_channels_mfma_general_edges(d, vd, policy, seq, mode, qs, ks, ws, ls, causal):
    run_case(np.float16, policy, seq, mode, (2,), d, vd, qs, ks, ws=ws, ls=ls, causal=causal, seed=d + vd + ws)


# --------------------------------------------------------------- edge cases
@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
@pytest.mark.parametrize("nq,nk", [(1, 1), (1, 77), (77, 1), (2, 3), (64, 64), (65, 63)])
def test_tiny_sequences(dtype, nq, nk):
    run_case(dtype, "full", 1, "none_front", (2,), 8, 8, (nq,), (nk,))
    run_case(dtype, "causal", 1, "scale_end", (2,), 8, 8, (nq,), (nk,))


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda t: np.dtype(t).name)
def test_fully_masked_rows(dtype):
    # causal scale_end with Nq > Nk leaves the first query rows with no key (orders of Q start below K's)
    run_case(dtype, "causal", 1, "scale_end", (2,), 16, 16, (64,), (16,))
    run_case(dtype, "local", 2, "scale_end", (1,), 16, 16, (4, 6), (6, 4), ws=1, ls=2, causal=True)


def test_empty_batch_and_sequences():
    fa = _fa()
    dev = torch.device("cuda:0")
    for shp_q, shp_k in (((0, 2, 8, 16), (0, 2, 8, 16)), ((1, 2, 8, 0), (1, 2, 8, 16))):
        q = torch.zeros(shp_q, dtype=torch.float16, device=dev)
        k = torch.zeros(shp_k, dtype=torch.float16, device=dev)
        o, l, m = fa.full_1d(q, k, k, returning_l_m=True)
        assert o.shape == shp_q and l.shape == shp_q[:2] + shp_q[3:]
    # no keys at all: every row attends nothing
    q = torch.ones((1, 1, 8, 5), dtype=torch.float32, device=dev)
    k = torch.ones((1, 1, 8, 0), dtype=torch.float32, device=dev)
    o, l, m = fa.full_1d(q, k, k, returning_l_m=True)
    assert (o == 0).all() and (l == 0).all()
    assert m.cpu().numpy().tobytes() == b"\xfa" * (5 * 4)


def test_dtype_dispatch_and_l_dtype():
    fa = _fa()
    dev = torch.device("cuda:0")
    for dt, ldt in ((torch.float16, torch.float32), (torch.float32, torch.float32), (torch.float64, torch.float64)):
        x = torch.randn(1, 2, 8, 32, device=dev, dtype=dt)
        o, l, m = fa.full_1d(x, x, x, returning_l_m=True)
        assert o.dtype == dt and l.dtype == ldt and m.dtype == dt
    with pytest.raises(TypeError):
        x = torch.randn(1, 2, 8, 32, device=dev, dtype=torch.bfloat16)
        fa.full_1d(x, x, x)


def test_batch_dims_are_flattened_and_independent():
    """Any batch rank (batch_shape may include heads) — slices are independent and
    the result is bitwise identical whether computed together or shard by shard."""
    fa = _fa()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.rand((2, 3, 2, 64, 200), device=dev, generator=g).half() * 4 - 2
    k = torch.rand((2, 3, 2, 64, 150), device=dev, generator=g).half() * 4 - 2
    v = torch.rand((2, 3, 2, 64, 150), device=dev, generator=g).half() * 4 - 2
    o = fa.causal_1d(q, k, v, "scale_front")
    for i in range(2):
        oi = fa.causal_1d(q[i], k[i], v[i], "scale_front")
        assert torch.equal(o[i], oi)


# --------------------------------------------- BASELINE configs (sampled)
def test_config2_full_size_sampled():
    """Config 2 at full size (b=128, N=4096, d=64, fp16): 3 slices checked against the oracle."""
    run_case(np.float16, "full", 1, "none_front", (8, 16), 64, 64, (4096,), (4096,), bwd=False, slices=[0, 77, 127],
             seed=1234)


def test_config3_causal_d128_sampled():
    """Config 3 shape at reduced batch (b=2): causal fp16 d=128 N=8192, forward + backward."""
    run_case(np.float16, "causal", 1, "none_front", (1, 2), 128, 128, (8192,), (8192,), seed=3, slices=[1])


def test_config4_local_window256_sampled():
    """Config 4 shape at reduced batch: local ws=256 fp16 d=64 N=16384."""
    run_case(np.float16, "local", 1, "none_front", (1, 2), 64, 64, (16384,), (16384,), ws=256, ls=0, causal=False,
             seed=4, slices=[0])


def test_config5_full2d_f32_sampled():
    """Config 5 shape at reduced batch: full_2d fp32 (64,64) vs (128,128), scale_front."""
    run_case(np.float32, "full", 2, "scale_front", (1, 2), 64, 64, (64, 64), (128, 128), seed=5, slices=[1])


# ------------------------------ fp16 kernel structures forced onto other shapes (selected by env)
# FA_FWD_VARIANT / FA_BWD_VARIANT (diagnostic library only) force a structure onto shapes the
# dispatcher sends elsewhere, so each shipped kernel is parity-checked on every rule it accepts
# (DESIGN.md §3.0, §3.2): 2200 the ping-pong forward (full policy; other rules fall through to the
# 8-wave kernel), 1814 the 8-wave forward, 2000 the paired-block study kept in csrc/diag/.
@pytest.fixture
def diag_lib(monkeypatch):
    """Routes the test through the diagnostic library (libfa_hip_diag.so), where the variant
    selectors exist; the product library has none and would silently run its default.  The diag
    library must have been built from the current sources (its build info carries their hash)."""
    from tf_flash_attention_amd import _lib
    if not __import__("os").path.exists(_lib.DIAG_LIB_PATH):
        pytest.skip("libfa_hip_diag.so not built (make -C tf_flash_attention_amd diag)")
    with _lib.using(_lib.DIAG_LIB_PATH) as h:
        info = _lib.build_info()
        assert "lib=diag" in info and f"src={_lib.source_hash(diag=True)};" in info, info
        yield h


VARIANT_CASES = [
    ("full", 1, "none_front", (264,), (136,), 1, False, 64, 64),
    ("full", 1, "none_front", (300,), (1000,), 1, False, 48, 64),
    ("causal", 1, "none_front", (392,), (392,), 1, False, 64, 64),
    ("causal", 1, "scale_end", (200,), (520,), 1, False, 64, 40),
    ("local", 1, "none_front", (700,), (700,), 33, False, 64, 64),
    ("local", 1, "scale_front", (240,), (480,), 70, True, 64, 64),
    ("causal", 2, "scale_front", (8, 24), (16, 16), 1, False, 64, 64),
]


@pytest.mark.parametrize("variant", ["2000", "2200", "1814"])
@pytest.mark.parametrize("policy,seq_dims,mode,qs,ks,ws,causal,d,vd", VARIANT_CASES)
def test_f16_forward_structures(monkeypatch, diag_lib, variant, policy, seq_dims, mode, qs, ks, ws, causal, d, vd):
    monkeypatch.setenv("FA_FWD_VARIANT", variant)
    run_case(np.float16, policy, seq_dims, mode, (2, 2), d, vd, qs, ks, ws=ws, ls=0, causal=causal, bwd=False,
             seed=int(variant) + d + ws)


# the one-wave-per-SIMD gap-stream forward (fa_fwd_f16_gap.hip, full policy): tails of every kind (nq
# not a multiple of its 256-query block or of the 64-query wave, nk not a multiple of 64 or shorter
# than one tile), d / v_d below 64, 2d shapes; seeds vary the scores' scale so rebases happen
GAP_CASES = [
    ((264,), (136,), 64, 64), ((300,), (1000,), 48, 64), ((256,), (64,), 64, 64), ((1000,), (4096,), 64, 64),
    ((17,), (72,), 64, 33), ((513,), (520,), 40, 64), ((64,), (8,), 64, 64), ((4096,), (256,), 64, 64),
    ((8, 24), (16, 16), 64, 48), ((77,), (3000,), 56, 60),
]


@pytest.mark.parametrize("qs,ks,d,vd", GAP_CASES)
@pytest.mark.parametrize("mode", ["none_front", "scale_end"])
def test_f16_forward_gap_stream(monkeypatch, diag_lib, qs, ks, d, vd, mode):
    monkeypatch.setenv("FA_FWD_VARIANT", "2600")
    run_case(np.float16, "full", len(qs), mode, (2, 3), d, vd, qs, ks, bwd=False, seed=2600 + d + vd + qs[0])


@pytest.mark.parametrize("variant", ["2301", "146"])
@pytest.mark.parametrize("policy,seq_dims,mode,qs,ks,ws,causal,d,vd", VARIANT_CASES)
def test_f16_forward_structures_d128(monkeypatch, diag_lib, variant, policy, seq_dims, mode, qs, ks, ws, causal, d, vd):
    """d in (64, 128]: the ping-pong kernel forced for every interval rule it takes (2301: 1d local
    windows too, with the heavy / light block pairs of the interval-rule instance) and the 4-wave kernel
    (146)."""
    monkeypatch.setenv("FA_FWD_VARIANT", variant)
    run_case(np.float16, policy, seq_dims, mode, (2, 2), d + 64, vd + 32, qs, ks, ws=ws, ls=0, causal=causal,
             bwd=False, seed=int(variant) + d + ws)


# the one-wave D = 128 gap-stream forward (csrc/diag/fa_fwd_f16_gap128.hip, FA_FWD_VARIANT=2700): full,
# causal (the heavy / light pairs), 1d local and 2d interval rules, lengths off the 256-query block and the
# 64-key tile, d != v_d, channels below 128
GAP128_CASES = [
    ("full", 1, "none_front", (264,), (136,), 1, False, 128, 128),
    ("full", 1, "none_front", (300,), (1000,), 1, False, 96, 128),
    ("full", 1, "none_front", (1000,), (4096,), 1, False, 128, 128),
    ("full", 1, "scale_end", (77,), (3000,), 1, False, 120, 100),
    ("full", 1, "none_front", (64,), (8,), 1, False, 128, 128),
    ("causal", 1, "none_front", (600,), (600,), 1, False, 128, 128),
    ("causal", 1, "none_front", (2048,), (2048,), 1, False, 128, 128),
    ("causal", 1, "scale_end", (328,), (776,), 1, False, 96, 128),
    ("local", 1, "none_front", (1000,), (1000,), 70, False, 128, 128),
    ("local", 1, "scale_front", (520,), (264,), 40, True, 128, 80),
    ("causal", 2, "scale_front", (8, 24), (16, 16), 1, False, 128, 128),
]


@pytest.mark.parametrize("policy,seq_dims,mode,qs,ks,ws,causal,d,vd", GAP128_CASES)
def test_f16_forward_gap_stream_d128(monkeypatch, diag_lib, policy, seq_dims, mode, qs, ks, ws, causal, d, vd):
    monkeypatch.setenv("FA_FWD_VARIANT", "2700")
    run_case(np.float16, policy, seq_dims, mode, (2, 2), d, vd, qs, ks, ws=ws, ls=0, causal=causal, bwd=False,
             seed=2700 + d + vd + qs[0] + ws)


# the 64-keys-a-wave dK/dV pass (csrc/diag/fa_bwd_f16_k64.hip, FA_BWD_VARIANT=1700): full, causal and
# 1d local windows at d in (64, 128], lengths off the 256-key block and the 32-query tile, nq != nk
K64_CASES = [
    ("full", "none_front", (264,), (520,), 1, False, 128, 128),
    ("causal", "none_front", (600,), (600,), 1, False, 128, 128),
    ("causal", "scale_end", (328,), (776,), 1, False, 96, 128),
    ("local", "none_front", (1000,), (1000,), 70, False, 128, 128),
    ("local", "scale_front", (520,), (264,), 40, True, 128, 80),
    ("full", "none_front", (64,), (8,), 1, False, 128, 128),
]


@pytest.mark.parametrize("policy,mode,qs,ks,ws,causal,d,vd", K64_CASES)
def test_f16_backward_k64(monkeypatch, diag_lib, policy, mode, qs, ks, ws, causal, d, vd):
    monkeypatch.setenv("FA_BWD_VARIANT", "1700")
    calls = diag_lib.fa_diag_call_count
    calls.restype = __import__("ctypes").c_longlong
    before = calls(1)
    run_case(np.float16, policy, 1, mode, (2, 2), d, vd, qs, ks, ws=ws, ls=0, causal=causal, seed=1700 + d + ws)
    assert calls(1) == before + 1


# backward structures kept in the diagnostic library: 1599 = the one-wave dQ pass (the structure the
# unaligned d > 64 shapes ship with) on aligned shapes, 1068 = the d <= 64 dQ pass with run-ahead
# operand reads, 82 = the d <= 64 passes in eight-wave blocks
@pytest.mark.parametrize("variant,d", [("1599", 128), ("1068", 64), ("82", 64)])
@pytest.mark.parametrize("policy,ws,causal", [("full", 1, False), ("causal", 1, False), ("local", 40, True)])
def test_f16_backward_read_placement(monkeypatch, diag_lib, variant, d, policy, ws, causal):
    monkeypatch.setenv("FA_BWD_VARIANT", variant)
    # autograd runs the backward on its own device thread: the diagnostic library must still be
    # the one that launches it (its call counter moves; the product library has none)
    calls = diag_lib.fa_diag_call_count
    calls.restype = __import__("ctypes").c_longlong
    before = calls(1)
    run_case(np.float16, policy, 1, "none_front", (2,), d, d, (328,), (264,), ws=ws, ls=0, causal=causal,
             seed=int(variant) + d)
    assert calls(1) == before + 1
