"""GPU parity at the BASELINE configs' full sizes (BASELINE.json configs 2-5).

The inputs are generated on the device (seeded U(-2,2), tests/test_base.py:170-173's
distribution, rounded to the config's dtype there): a full-size batch would need many GiB of
host memory.  The op runs over the whole batch through the reference-API mirror; then only
sampled slices are copied back and checked against the float64 oracle with the tolerances of
tests/test_gpu_parity.py (first, middle and last slices, plus the slices where the XCD ranges
and persistent workgroups of the band kernel change hands).

Every slice (round 4): the same float64 math as the oracle, evaluated on the GPU over the whole
batch (_batch_ref_f64: the oracle's own rule evaluator supplies each row block's column band and
mask, torch does the float64 products), is checked against the numpy oracle on the sampled slices
to 1e-9 and then stands in for it on all of them, with the same tolerances.

Size-independent properties over the whole batch as well:
  * batch reversal: the op on the batch in reverse slice order is bitwise the reverse of the
    op on the batch.  A slice's result then does not depend on which workgroup, XCD or
    persistent item walked it, so one wrong walk step anywhere in the batch shows up;
  * O is a convex combination of V rows: |O| <= max|V| everywhere, every value finite;
  * l >= 1 wherever a row attends anything (its largest term is exp(0) at the stored m).
"""

import numpy as np
import pytest
import torch

from oracle import fa_oracle as O
from tests.test_gpu_parity import TOL, _close

pytestmark = pytest.mark.gpu

TORCH = {np.float16: torch.float16, np.float32: torch.float32}


def _fa():
    from tf_flash_attention_amd import flash_attention as fa
    return fa


def _uniform(shape, dtype, gen, dev):
    return (torch.rand(shape, generator=gen, device=dev, dtype=torch.float32) * 4 - 2).to(TORCH[dtype])


def _call(fa, policy, seq_dims, q, k, v, mode, ws):
    if policy == "full":
        f = fa.full_1d if seq_dims == 1 else fa.full_2d
        return f(q, k, v, sync_mode=mode, returning_l_m=True)
    if policy == "causal":
        return fa.causal_1d(q, k, v, mode, returning_l_m=True)
    return fa.local_1d(q, k, v, ws, 0, False, mode, returning_l_m=True)


def _check_lm(dtype, lg, mg, L64, M64, ha):
    rtol, atol = TOL[dtype]["fwd"]
    m_f = mg[:, ha].astype(np.float64)
    ulp = np.abs(np.spacing(np.abs(M64[:, ha]).astype(dtype))).astype(np.float64)
    m_tol = 2 * ulp + (1e-3 * np.maximum(np.abs(M64[:, ha]), 1.0) if dtype == np.float16
                       else 1e-6 * np.abs(M64[:, ha]) + 1e-6)
    assert (np.abs(m_f - M64[:, ha]) <= m_tol).all(), f"m: max err {np.abs(m_f - M64[:, ha]).max():.3e}"
    l_ref = L64[:, ha] * np.exp(M64[:, ha] - m_f)
    _close("l", lg[:, ha].astype(np.float64), l_ref, max(rtol, 1e-6 if dtype == np.float16 else rtol), atol)


def _batch_ref_f64(q, k, v, do, prob, q_seq, k_seq, bchunk):
    """O, l, m (and dQ, dK, dV when do is given) of every slice in float64 on the GPU: the numpy
    oracle's formulas (oracle/fa_oracle.py forward_f64 / backward_f64, row chunks with the rule's
    column band and mask from its own evaluator), batched over slices.  q, k, v, do: [b, c, n]."""
    b, d, nq = q.shape
    vd, nk = v.shape[1], k.shape[2]
    dev = q.device
    scale = 1.0 / np.sqrt(d)
    Of = torch.zeros((b, vd, nq), dtype=torch.float64, device=dev)
    Mf = torch.zeros((b, nq), dtype=torch.float64, device=dev)
    Lf = torch.zeros((b, nq), dtype=torch.float64, device=dev)
    grads = None
    if do is not None:
        grads = tuple(torch.zeros((b, c, n), dtype=torch.float64, device=dev) for c, n in ((d, nq), (d, nk), (vd, nk)))
    ha_all = np.zeros(nq, dtype=bool)
    for r0, r1, c0, c1, mk in O._row_chunks(O._evaluator(prob, q_seq, k_seq), nq):
        if c1 == c0:
            continue
        ha = mk.any(axis=1)
        ha_all[r0:r1] = ha
        mk_t = torch.from_numpy(mk).to(dev)
        ha_t = torch.from_numpy(ha).to(dev)
        for b0 in range(0, b, bchunk):
            b1 = min(b, b0 + bchunk)
            qi = q[b0:b1, :, r0:r1].double()
            ki = k[b0:b1, :, c0:c1].double()
            vi = v[b0:b1, :, c0:c1].double()
            s = torch.where(mk_t, torch.matmul(qi.transpose(1, 2), ki) * scale, -torch.inf)
            mrow = torch.where(ha_t, s.amax(dim=2), 0.0)
            p = torch.exp(s - mrow[:, :, None])
            lsum = p.sum(dim=2)
            p = p / torch.where(ha_t, lsum, 1.0)[:, :, None]
            o = torch.matmul(vi, p.transpose(1, 2))
            Of[b0:b1, :, r0:r1] = o
            Mf[b0:b1, r0:r1] = mrow
            Lf[b0:b1, r0:r1] = lsum
            if grads is not None:
                doi = do[b0:b1, :, r0:r1].double()
                dQ, dK, dV = grads
                dV[b0:b1, :, c0:c1] += torch.matmul(doi, p)
                dp = torch.matmul(doi.transpose(1, 2), vi)
                D = (doi * o).sum(dim=1)
                ds = p * (dp - D[:, :, None]) * scale
                dQ[b0:b1, :, r0:r1] = torch.matmul(ki, ds.transpose(1, 2))
                dK[b0:b1, :, c0:c1] += torch.matmul(qi, ds)
            del s, p
    return Of, Lf, Mf, ha_all, grads


def _close_gpu(name, got, ref, rtol, atol_rel):
    """tests/test_gpu_parity._close on device tensors, with the atol scale taken per slice:
    max(max|ref|, 1) over each slice (leading dim) on its own, so a slice with smaller values
    is not judged against the batch maximum."""
    got = got.double()
    scale = ref.abs().reshape(ref.shape[0], -1).amax(dim=1).clamp(min=1.0)
    scale = scale.reshape((-1,) + (1,) * (ref.dim() - 1))
    err = (got - ref).abs()
    bad = err > atol_rel * scale + rtol * ref.abs()
    assert bool(torch.isfinite(got).all()), f"{name}: non-finite output"
    nbad = int(bad.sum())
    assert nbad == 0, f"{name}: {nbad} / {bad.numel()} elements off (whole batch); max abs err {float(err.max()):.3e}"


def _check_lm_gpu(dtype, lg, mg, L64, M64, ha):
    rtol, atol = TOL[dtype]["fwd"]
    h = torch.from_numpy(ha).to(lg.device)
    m_f = mg.double()[:, h]
    Mr = M64[:, h]
    _, ex = torch.frexp(Mr.abs())  # ulp of |m| in T: 2^(e - 1 - mantissa bits)
    ulp = torch.ldexp(torch.ones_like(Mr), ex - 1 - (10 if dtype == np.float16 else 23))
    m_tol = 2 * ulp + (1e-3 * torch.clamp(Mr.abs(), min=1.0) if dtype == np.float16 else 1e-6 * Mr.abs() + 1e-6)
    err = (m_f - Mr).abs()
    assert bool((err <= m_tol).all()), f"m: max err {float(err.max()):.3e} (whole batch)"
    _close_gpu("l", lg.double()[:, h], L64[:, h] * torch.exp(Mr - m_f), max(rtol, 1e-6 if dtype == np.float16 else rtol),
               atol)


def _properties(o, l, v, name):
    vmax = float(v.abs().max())
    assert bool(torch.isfinite(o).all()), f"{name}: non-finite O"
    assert float(o.abs().max()) <= vmax * (1 + 2e-3), f"{name}: |O| above max|V|"
    # (l is relative to the stored, rounded m: its largest term is exp(max - m_T) >= exp(-|rounding|))
    assert float(l.min()) >= 0.99, f"{name}: l below 1 for a row that attends keys"


def run_full_size(dtype, policy, seq_dims, mode, batch, d, qs, ks, ws=1, bwd=False, slices=(), seed=0,
                  reverse=True, bchunk=16):
    fa = _fa()
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(seed)
    b = int(np.prod(batch))
    q = _uniform(tuple(batch) + (d,) + tuple(qs), dtype, gen, dev)
    k = _uniform(tuple(batch) + (d,) + tuple(ks), dtype, gen, dev)
    v = _uniform(tuple(batch) + (d,) + tuple(ks), dtype, gen, dev)
    do = _uniform(tuple(batch) + (d,) + tuple(qs), dtype, gen, dev) if bwd else None
    for t in (q, k, v):
        t.requires_grad_(bwd)
    o, l, m = _call(fa, policy, seq_dims, q, k, v, mode, ws)
    if bwd:
        o.backward(do)
    torch.cuda.synchronize()
    nq, nk = int(np.prod(qs)), int(np.prod(ks))
    flat = lambda x, c: x.detach().reshape(b, c, -1) if c else x.detach().reshape(b, -1)  # noqa: E731
    sl = sorted(set(int(s) % b for s in slices))
    # ---- oracle on the sampled slices
    Qh, Kh, Vh = (flat(t, d)[sl].cpu().numpy() for t in (q, k, v))
    prob = O.Problem(policy, seq_dims, mode, ws, 0, False)
    shp = lambda x, c, s: x.reshape((len(sl), c) + tuple(s))  # noqa: E731
    O64, L64, M64, ha = O.forward_f64(shp(Qh, d, qs), shp(Kh, d, ks), shp(Vh, d, ks), prob)
    rtol, atol = TOL[dtype]["fwd"]
    _close("O", flat(o, d)[sl].cpu().numpy(), O64.reshape(len(sl), d, nq), rtol, atol)
    _check_lm(dtype, flat(l, 0)[sl].cpu().numpy(), flat(m, 0)[sl].cpu().numpy(),
              L64.reshape(len(sl), nq), M64.reshape(len(sl), nq), ha)
    if bwd:
        dOh = flat(do, d)[sl].cpu().numpy()
        dQ, dK, dV = O.backward_f64(shp(Qh, d, qs), shp(Kh, d, ks), shp(Vh, d, ks), shp(dOh, d, qs), prob)
        rtol, atol = TOL[dtype]["bwd"]
        _close("dQ", flat(q.grad, d)[sl].cpu().numpy(), dQ.reshape(len(sl), d, nq), rtol, atol)
        _close("dK", flat(k.grad, d)[sl].cpu().numpy(), dK.reshape(len(sl), d, nk), rtol, atol)
        _close("dV", flat(v.grad, d)[sl].cpu().numpy(), dV.reshape(len(sl), d, nk), rtol, atol)
    # ---- every slice: the oracle's float64 math on the GPU, pinned to the numpy oracle on the
    #      sampled slices, then checked against the op over the whole batch
    Rf = _batch_ref_f64(flat(q, d), flat(k, d), flat(v, d), flat(do, d) if bwd else None, prob, tuple(qs), tuple(ks),
                        bchunk)
    RO, RL, RM, rha, rgrads = Rf
    assert (rha == ha).all()
    sl_t = torch.tensor(sl, device=dev)
    pin = [("O", RO, O64.reshape(len(sl), d, nq)), ("l", RL, L64.reshape(len(sl), nq)),
           ("m", RM, M64.reshape(len(sl), nq))]
    if bwd:
        pin += [("dQ", rgrads[0], dQ.reshape(len(sl), d, nq)), ("dK", rgrads[1], dK.reshape(len(sl), d, nk)),
                ("dV", rgrads[2], dV.reshape(len(sl), d, nk))]
    for name, r, o64 in pin:
        got, want = r.index_select(0, sl_t).cpu().numpy(), np.asarray(o64, dtype=np.float64)
        fin = np.isfinite(want)
        assert (np.isfinite(got) == fin).all(), f"batch reference {name}: finiteness differs from the oracle"
        assert np.abs(got[fin] - want[fin]).max() <= 1e-9 * max(np.abs(want[fin]).max(), 1.0), \
            f"batch reference {name} disagrees with the numpy oracle"
    rtol, atol = TOL[dtype]["fwd"]
    _close_gpu("O", flat(o, d), RO, rtol, atol)
    _check_lm_gpu(dtype, flat(l, 0), flat(m, 0), RL, RM, ha)
    if bwd:
        rtol, atol = TOL[dtype]["bwd"]
        for name, g, r in (("dQ", q.grad, rgrads[0]), ("dK", k.grad, rgrads[1]), ("dV", v.grad, rgrads[2])):
            _close_gpu(name, flat(g, d), r, rtol, atol)
    del Rf, RO, RL, RM, rgrads
    torch.cuda.empty_cache()
    # ---- size-independent properties over the whole batch
    if ha.all():
        _properties(o.detach(), l, v.detach(), "batch")
    if reverse:
        rq, rk, rv = (flat(t, d).flip(0).contiguous().reshape(t.shape) for t in (q, k, v))
        if bwd:
            for t in (rq, rk, rv):
                t.requires_grad_(True)
        ro, rl, rm = _call(fa, policy, seq_dims, rq, rk, rv, mode, ws)
        assert torch.equal(flat(ro, d).flip(0), flat(o, d)), "O depends on the slice's position in the batch"
        assert torch.equal(flat(rl, 0).flip(0), flat(l, 0)), "l depends on the slice's position in the batch"
        assert torch.equal(flat(rm, 0).flip(0), flat(m, 0)), "m depends on the slice's position in the batch"
        if bwd:
            ro.backward(flat(do, d).flip(0).contiguous().reshape(do.shape))
            for name, g, rg in (("dQ", q.grad, rq.grad), ("dK", k.grad, rk.grad), ("dV", v.grad, rv.grad)):
                assert torch.equal(flat(rg, d).flip(0), flat(g, d)), f"{name} depends on the slice's position"
    torch.cuda.synchronize()


def test_config2_full_size():
    """Config 2: full_1d fp16 B=8 H=16 d=64 N=4096, forward (the headline kernel)."""
    run_full_size(np.float16, "full", 1, "none_front", (8, 16), 64, (4096,), (4096,), slices=(0, 31, 64, 127),
                  seed=2, bchunk=64)


def test_config3_full_size():
    """Config 3: causal_1d fp16 B=8 H=16 d=128 N=8192, forward + backward."""
    run_full_size(np.float16, "causal", 1, "none_front", (8, 16), 128, (8192,), (8192,), bwd=True,
                  slices=(0, 63, 127), seed=3, bchunk=32)


def test_config4_full_size():
    """Config 4: local_1d fp16 window 256, B=64 H=16 d=64 N=16384, forward on ONE GPU (b=1024:
    65,536 persistent items).  The band kernel deals one eighth of the items to each XCD and
    every J-th of those to a workgroup: slices 127/128, 511/512 and 895/896 straddle XCD ranges."""
    run_full_size(np.float16, "local", 1, "none_front", (64, 16), 64, (16384,), (16384,), ws=256,
                  slices=(0, 1, 127, 128, 511, 512, 895, 896, 1023), seed=4, bchunk=128)


def test_config4_per_gpu_shard():
    """Config 4's per-GPU shard on the 8-GPU run: b = 1024 / 8 = 128 slices (shard.shard_range)."""
    from tf_flash_attention_amd import shard
    s0, s1 = shard.shard_range(1024, 8, 3)
    assert s1 - s0 == 128
    run_full_size(np.float16, "local", 1, "none_front", (s1 - s0,), 64, (16384,), (16384,), ws=256,
                  slices=(0, 15, 16, 63, 64, 127), seed=40 + s0, bchunk=128)


def test_config5_full_size():
    """Config 5: full_2d fp32 B=4 H=8 d=64 (64,64) vs (128,128), scale_front; forward and backward."""
    run_full_size(np.float32, "full", 2, "scale_front", (4, 8), 64, (64, 64), (128, 128), bwd=True,
                  slices=(0, 13, 31), seed=5)


def test_band_table_limit_long_local_sequence():
    """nq just above 2^20 (4097 query blocks of 256): past the band kernel's per-slice LDS table of
    first key tiles (kMaxTab = 4096), so the dispatcher must route it elsewhere; checked on the
    rows around block 4096 and at both ends against the oracle's row-range forward."""
    fa = _fa()
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(77)
    n, d, ws = (1 << 20) + 256, 64, 64
    q, k, v = (_uniform((1, d, n), np.float16, gen, dev) for _ in range(3))
    o, l, m = fa.local_1d(q, k, v, ws, 0, False, "none_front", returning_l_m=True)
    torch.cuda.synchronize()
    qh, kh, vh = (t[0].cpu().numpy() for t in (q, k, v))
    prob = O.Problem("local", 1, "none_front", ws, 0, False)
    rtol, atol = TOL[np.float16]["fwd"]
    for r0 in (0, 4095 * 256 - 64, 4096 * 256 - 64, 4096 * 256, n - 64):
        r1 = r0 + 64
        # (none_front, nq == nk: row i attends keys within ws - 1 of i; the oracle still evaluates
        # the rule on a wider range)
        o64, l64, m64, ha = O.forward_rows_f64(qh, kh, vh, prob, [n], [n], r0, r1, max(0, r0 - 2 * ws),
                                               min(n, r1 + 2 * ws))
        _close(f"O[{r0}:{r1}]", o[0, :, r0:r1].cpu().numpy(), o64, rtol, atol)
        _check_lm(np.float16, l[0, r0:r1].cpu().numpy()[None], m[0, r0:r1].cpu().numpy()[None], l64[None], m64[None],
                  ha)


def test_product_library_is_built_from_these_sources():
    """On the GPU box: the product library this process loads carries the hash of the sources
    beside it, and is the product build (not the diagnostic one)."""
    from tf_flash_attention_amd import _lib
    info = _lib.build_info()
    assert f"src={_lib.source_hash()};" in info, (info, _lib.source_hash())
    assert "lib=product" in info, info
