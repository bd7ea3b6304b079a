"""Tolerances of the GPU parity tests (one definition, used by tests/test_gpu_parity.run_case and by the
CPU checks of the gate itself, tests/test_gate_mutations.py and tests/test_oracle.py).

Per element: |got - ref| <= ATOL*S + RTOL*|ref| (+ the gradient rounding term), S = max(max|ref|, 1).
  fp16: forward rtol 1e-3 / atol 1e-3*S (BASELINE.json north_star rtol=1e-3); backward rtol 1e-3 /
        atol 2e-3*S
  fp32: rtol 1e-5 / atol 1e-5*S (north_star rtol=1e-5)
  fp64: rtol 1e-10 / atol 1e-10*S
Gradients add KAPPA x the oracle's per-element rounding-error scale e (oracle.backward_rounding_scale_f64:
the root-sum-square of each term's rounding bound, for the tensor type's and the accumulation's unit
roundoff, U_ROUND).  The term is what a correct computation needs where a gradient is a sum of large
cancelling terms (dK / dQ of a row set with one or two keys, dP ~ D) or where an fp16 score's rounding
is large beside the result (d = 1): profiles/r05_fuzz20000.txt."""
import numpy as np

TOL = {
    np.float16: dict(fwd=(1e-3, 1e-3), bwd=(1e-3, 2e-3)),
    np.float32: dict(fwd=(1e-5, 1e-5), bwd=(1e-5, 1e-5)),
    np.float64: dict(fwd=(1e-10, 1e-10), bwd=(1e-10, 1e-10)),
}
U_ROUND = {np.float16: (2.0 ** -11, 2.0 ** -24), np.float32: (2.0 ** -24, 2.0 ** -24),
           np.float64: (2.0 ** -53, 2.0 ** -53)}
KAPPA = 3.0


def plain_bound(ref, rtol, atol_rel):
    ref = np.asarray(ref, dtype=np.float64)
    scale = max(float(np.max(np.abs(ref))) if ref.size else 0.0, 1.0)
    return atol_rel * scale + rtol * np.abs(ref)


# fp16: where the rounding scale stays below the plain bound (no cancellation: the element's terms do
# not cancel to well below their own size) the rounding term is capped at CAP x the plain bound; only
# cancelling elements (e > plain) get the full KAPPA x e.  Uncapped, the term let defects of ~1.5x the
# plain bound through in fp16 (tests/test_gate_mutations.py); correct fp16 kernels reach 1.31x at most
# over the GPU suite (profiles/r06_gate_stats.txt).  fp32 / fp64 keep the full term: every injected
# defect sits orders of magnitude above their tolerances, while correct fp32 dQ of one- or two-key rows
# reach 3x the plain bound at e ~ 0.7x of it (the r05 cancelling seeds).
CAP = {np.float16: 0.4}


def grad_extra(ref, e, dtype):
    """The rounding term added to the plain gradient bound of each element."""
    e = np.asarray(e, dtype=np.float64)
    full = KAPPA * e
    if dtype not in CAP:
        return full
    rtol, atol = TOL[dtype]["bwd"]
    plain = plain_bound(ref, rtol, atol)
    return np.where(e > plain, full, np.minimum(full, CAP[dtype] * plain))


def grad_bound(ref, e, dtype):
    rtol, atol = TOL[dtype]["bwd"]
    return plain_bound(ref, rtol, atol) + grad_extra(ref, e, dtype)


# Whole-gradient scale check: |slope(got, ref)| <= SLOPE_TOL for every gradient that stands clear of its
# own rounding noise (rms(ref) > SLOPE_SNR * rms(e)).  The per-element bound above cannot see a defect
# that scales a whole gradient by ~2^-8 in fp16 (that is 1.3x its plain bound at the largest element,
# the same ratio the worst correct fp16 case of the suite reaches); the slope averages the rounding
# noise out and sees it at full size.  Measured over the GPU suite (1351 cases, profiles/r06_gate_stats.txt):
# max |slope| of the non-degenerate gradients 1.63e-3 (fp16, a 2-element d = 1 case), 1.9e-6 (fp32),
# 1.4e-15 (fp64); fp16 at d = 1 has its own tolerance (slope_tol).
# fp32 2^-15: a correct d = 256 case of five queries and five keys in a window (fuzz seed 28600) reached 7.7e-6
# in dK (> 2^-17), two cancelling large elements over rounding-level ones; every injected fp32 defect is
# still >= 1e-3 (tests/test_gate_mutations.py)
SLOPE_TOL = {np.float16: 2.0 ** -9, np.float32: 2.0 ** -15, np.float64: 2.0 ** -45}
SLOPE_SNR = 100.0


def slope_applies(ref, e) -> bool:
    ref = np.asarray(ref, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    return bool(ref.size and np.sqrt(np.mean(ref * ref)) > SLOPE_SNR * np.sqrt(np.mean(e * e)))


def elements_ok(got, ref, e, dtype) -> bool:
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return bool(np.isfinite(got).all() and (np.abs(got - ref) <= grad_bound(ref, e, dtype)).all())


def slope_tol(dtype, d=None) -> float:
    """SLOPE_TOL, except fp16 at d = 1: each score is then one product, so the kernels' rounding of the
    pre-scaled Q (one fp16 rounding per query row) is not averaged over channels and the row's
    scores, and its gradients, move coherently; a correct d = 1 case of the 20000-case fuzz reached a slope of
    2.05e-3 (> 2^-9).  3e-3 still rejects dS x (1 + 2^-8) (slope 3.9e-3, tests/test_gate_mutations.py)."""
    return 3e-3 if (dtype == np.float16 and d == 1) else SLOPE_TOL[dtype]


def row_coherent_slope(ref, e, ch) -> float:
    """The slope a correct kernel's rounding can reach when it is coherent within each row of the gradient
    (a query row of dQ, a key row of dK / dV: the `ch` channels of one position of a [batch, ch, positions]
    gradient) and independent between rows: sqrt(sum_rows (sum_c e*|ref|)^2) / sum ref^2.  The fp16
    kernels' per-row roundings (the pre-scaled Q, D = rowsum(dO*O), the row's stored m) move a whole row
    together, so a gradient carried by one or two rows does not average them out; a correct causal case of
    the fuzz with one query row carrying dQ (seed 41712: d = 200, two queries, two keys) reached a dQ slope of
    2.30e-3 against this bound's 3.65e-3.  With many rows the bound falls as 1/sqrt(rows) below SLOPE_TOL."""
    ref = np.asarray(ref, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    rr = float(np.sum(ref * ref))
    if ch is None or rr == 0.0:
        return 0.0
    per_row = np.sum((np.abs(ref) * e).reshape(ref.shape[0], ch, -1), axis=1)
    return float(np.sqrt(np.sum(per_row * per_row)) / rr)


def coherent_slope(ref, e) -> float:
    """The slope of a rounding error of size e coherent over the whole gradient: <e, |ref|> / <ref, ref>."""
    ref = np.asarray(ref, dtype=np.float64)
    rr = float(np.sum(ref * ref))
    return float(np.sum(np.abs(ref) * np.asarray(e, dtype=np.float64)) / rr) if rr > 0.0 else 0.0


def slope_tol_eff(ref, e, dtype, d=None, ch=None) -> float:
    """The slope tolerance of one gradient.  fp16 at d = 1: each score is one product of a query and a key,
    so the rounding of the pre-scaled query moves every score of its row by the same relative amount, and
    that row's error reaches every key's dK / dV as well as its own dQ: the rounding is coherent over the
    whole gradient, not per row (a correct full-window causal case, seed 72261: 577 queries, 418 keys, dK
    slope -3.43e-3 against this bound's 8.36e-3).  Everywhere else: slope_tol, or the row-coherent bound
    where a gradient rests on few rows."""
    tol = max(slope_tol(dtype, d), row_coherent_slope(ref, e, ch))
    if dtype == np.float16 and d == 1:
        tol = max(tol, coherent_slope(ref, e))
    return tol


def slope_ok(got, ref, e, dtype, d=None, ch=None) -> bool:
    return (not slope_applies(ref, e)) or abs(scale_slope(got, ref)) <= slope_tol_eff(ref, e, dtype, d, ch)


def grad_ok(got, ref, e, dtype, d=None, ch=None) -> bool:
    return elements_ok(got, ref, e, dtype) and slope_ok(got, ref, e, dtype, d, ch)


def scale_slope(got, ref):
    """beta = <got, ref> / <ref, ref> - 1: the least-squares relative scale of got against ref (0 when
    got is ref plus errors uncorrelated with it; a defect that scales a whole gradient, e.g. dS by
    1 + 2^-8, shows up here at its full size)."""
    got = np.asarray(got, dtype=np.float64).ravel()
    ref = np.asarray(ref, dtype=np.float64).ravel()
    rr = float(ref @ ref)
    return float(got @ ref) / rr - 1.0 if rr > 0 else 0.0


def grad_stats(got, ref, e, dtype) -> dict:
    """Per-gradient statistics of the gate (tests/test_gpu_parity.py writes them when FA_GATE_STATS
    names a file): how far the errors sit from the plain rtol/atol bound and from the full bound, the
    fraction of elements that pass only because of the rounding term, and the scale slope."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    rtol, atol = TOL[dtype]["bwd"]
    err = np.abs(got - ref)
    plain = plain_bound(ref, rtol, atol)
    full = plain + grad_extra(ref, e, dtype)
    return dict(n=int(err.size), max_err_over_plain=float((err / plain).max()) if err.size else 0.0,
                max_err_over_full=float((err / full).max()) if err.size else 0.0,
                frac_over_plain=float((err > plain).mean()) if err.size else 0.0,
                slope=scale_slope(got, ref), ref_rms=float(np.sqrt(np.mean(ref * ref))) if err.size else 0.0)


def max_abs_dot(Q, K, mask, chunk=512):
    """Per slice and query row, max over the row's allowed keys of sum_c |q_c| |k_c| (Q [b, d, nq], K [b, d, nk],
    mask [nq, nk]; 0 for a row with no allowed key): the scale of the rounding a score, and so the row max,
    can carry when Q is rounded before the product (tests/test_gpu_parity.py's fp16 m bound)."""
    b, _, nq = Q.shape
    out = np.zeros((b, nq))
    for i in range(b):
        aq = np.abs(Q[i].astype(np.float64)).T
        ak = np.abs(K[i].astype(np.float64))
        for r0 in range(0, nq, chunk):
            p = aq[r0:r0 + chunk] @ ak
            out[i, r0:r0 + chunk] = np.where(mask[r0:r0 + chunk], p, 0.0).max(axis=1)
    return out
