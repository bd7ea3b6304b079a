"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every
symbol include/fa_api.h declares; its host-side rule code (the same fa_rules.h
the kernels execute) matches the oracle; the Python mirror reproduces the
reference op surface and its error messages.  No device compute here."""

import ctypes
import os
import re

import numpy as np
import pytest

from oracle import fa_oracle as O
from tf_flash_attention_amd import _lib
from tf_flash_attention_amd import flash_attention as fa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POL = {"full": _lib.FULL, "causal": _lib.CAUSAL, "local": _lib.LOCAL}
SYNC = {"none_front": _lib.NONE_FRONT, "scale_front": _lib.SCALE_FRONT, "scale_end": _lib.SCALE_END}


def test_library_exports_every_declared_symbol():
    header = open(os.path.join(ROOT, "include", "fa_api.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\**\s*(fa_\w+)\s*\(", header, flags=re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS), declared ^ set(_lib.EXPORTED_SYMBOLS)
    L = _lib.lib()
    for sym in declared:
        assert hasattr(L, sym), sym
    assert b"gfx950" in L.fa_build_info()


def test_sync_mode_lookup():
    L = _lib.lib()
    for name, v in SYNC.items():
        assert L.fa_sync_mode_from_string(name.encode()) == v
    assert L.fa_sync_mode_from_string(b"bogus") == -1
    with pytest.raises(fa.InvalidArgumentError, match="Unsupported sync_mode: bogus"):
        fa._sync_mode_id("bogus")


def _prob(policy, qs, ks, mode="none_front", ws=1, ls=0, causal=False, dtype=_lib.F32, b=1, d=8, vd=8):
    return _lib.make_problem(dtype, POL[policy], len(qs), SYNC[mode], b, qs, ks, d, vd, ws, ls, causal)


def _lib_mask(p, nq, nk):
    buf = (ctypes.c_uint8 * (nq * nk))()
    assert _lib.lib().fa_rule_mask(p, ctypes.cast(buf, ctypes.c_void_p)) == 0
    return np.frombuffer(buf, dtype=np.uint8).reshape(nq, nk).astype(bool)


def _cases(seed, n):
    rng = np.random.default_rng(seed)
    for _ in range(n):
        dims = int(rng.integers(1, 3))
        if dims == 1:
            qs, ks = [int(rng.integers(1, 70))], [int(rng.integers(1, 70))]
        else:
            qs = [int(rng.integers(1, 10)), int(rng.integers(1, 10))]
            ks = [int(rng.integers(1, 10)), int(rng.integers(1, 10))]
        yield (qs, ks, str(rng.choice(O.SYNC_MODES)), str(rng.choice(O.POLICIES)), int(rng.integers(1, 7)),
               int(rng.integers(0, 3)), bool(rng.integers(0, 2)))


def test_library_rule_mask_matches_oracle():
    for qs, ks, mode, pol, ws, ls, causal in _cases(11, 300):
        p = _prob(pol, qs, ks, mode, ws, ls, causal)
        got = _lib_mask(p, int(np.prod(qs)), int(np.prod(ks)))
        ref = O.rule_mask(qs, ks, mode, pol, ws, ls, causal)
        assert (got == ref).all(), (qs, ks, mode, pol, ws, ls, causal)
        assert _lib.lib().fa_allowed_pairs(p) == int(ref.sum())


def test_block_ranges_are_conservative_and_tile_class_exact():
    """Every allowed pair lies inside the K range of its Q block and the Q range of
    its K block; tile class 2 => all allowed, 0 => none (the kernels skip on it)."""
    L = _lib.lib()
    out = (ctypes.c_int32 * 5)()
    rng = np.random.default_rng(5)
    for qs, ks, mode, pol, ws, ls, causal in _cases(13, 160):
        p = _prob(pol, qs, ks, mode, ws, ls, causal)
        nq, nk = int(np.prod(qs)), int(np.prod(ks))
        ref = O.rule_mask(qs, ks, mode, pol, ws, ls, causal)
        for _ in range(6):
            bq = int(rng.integers(1, 9))
            bk = int(rng.integers(1, 9))
            q0 = int(rng.integers(0, nq)); q1 = min(nq - 1, q0 + bq - 1)
            k0 = int(rng.integers(0, nk)); k1 = min(nk - 1, k0 + bk - 1)
            assert L.fa_rule_probe(p, q0, q1, k0, k1, out) == 0
            kb, ke, qb, qe, cls = list(out)
            rows = ref[q0:q1 + 1]
            ks_allowed = np.nonzero(rows.any(axis=0))[0]
            if ks_allowed.size:
                assert kb <= ks_allowed.min() and ks_allowed.max() < ke, (qs, ks, mode, pol, ws, ls, causal, q0, q1)
            cols = ref[:, k0:k1 + 1]
            qs_allowed = np.nonzero(cols.any(axis=1))[0]
            if qs_allowed.size:
                assert qb <= qs_allowed.min() and qs_allowed.max() < qe, (qs, ks, mode, pol, ws, ls, causal, k0, k1)
            tile = ref[q0:q1 + 1, k0:k1 + 1]
            if cls == 2:
                assert tile.all()
            if cls == 0:
                assert not tile.any()


def test_validate_rejects_bad_problems():
    L = _lib.lib()
    assert L.fa_validate(_prob("full", [16], [16])) == 0
    bad = [
        _prob("local", [16], [16], ws=0),
        _prob("local", [16], [16], ls=31),
        _prob("local", [16], [16], ws=2, ls=30),
        _prob("full", [16], [16], d=0),
    ]
    for p in bad:
        assert L.fa_validate(p) == _lib.FA_ERR_INVALID_ARGUMENT
        assert _lib.last_error()
    p = _prob("full", [16], [16])
    p.sync_mode = 7
    assert L.fa_validate(p) == _lib.FA_ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("ls", [0, 1])
def test_window_near_int32_max_does_not_overflow(causal, ls):
    """window_size up to INT32_MAX (fa_validate accepts ws << ls <= INT32_MAX): the rule's reach and
    interval arithmetic must saturate, not wrap (64x64 local gave 128 pairs, not 4096)."""
    from oracle import fa_oracle as O
    ws = (2 ** 31 - 1) >> ls
    L = _lib.lib()
    for seq_dims, qs, ks in ((1, [64], [64]), (1, [40], [72]), (2, [8, 8], [8, 8])):
        p = _prob("local", qs, ks, ws=ws, ls=ls, causal=causal)
        assert L.fa_validate(p) == 0
        mask = O.problem_mask(O.Problem("local", seq_dims, "none_front", ws, ls, causal), qs, ks)
        assert L.fa_allowed_pairs(p) == int(mask.sum())
        np.testing.assert_array_equal(_lib_mask(p, int(np.prod(qs)), int(np.prod(ks))), mask)
        nq, nk = int(np.prod(qs)), int(np.prod(ks))
        out = (ctypes.c_int32 * 5)()
        for q0, q1, k0, k1 in ((0, nq - 1, 0, nk - 1), (3, 9, 10, 20), (nq - 5, nq - 1, 0, 4)):
            assert L.fa_rule_probe(p, q0, q1, k0, k1, out) == 0
            kb, ke, qb, qe = out[0], out[1], out[2], out[3]
            need_k = np.nonzero(mask[q0:q1 + 1].any(axis=0))[0]
            need_q = np.nonzero(mask[:, k0:k1 + 1].any(axis=1))[0]
            if need_k.size:
                assert kb <= need_k.min() and ke > need_k.max()
            if need_q.size:
                assert qb <= need_q.min() and qe > need_q.max()


def test_library_was_built_from_these_sources():
    """fa_build_info() carries the hash of the sources the library was compiled from (Makefile
    SRC_HASH): a stale or foreign libfa_hip.so fails here, on CPU and on the GPU box alike."""
    info = _lib.build_info()
    assert f"src={_lib.source_hash()};" in info, (info, _lib.source_hash())
    assert "lib=product" in info


def test_product_library_reads_no_environment():
    """A/B variants, ablations (outputs WRONG) and stamp builds live only in libfa_hip_diag.so
    (-DFA_DIAG); the product library carries no variant selector and imports no getenv."""
    path = _lib.LIB_PATH
    data = open(path, "rb").read()
    for key in (b"FA_FWD_VARIANT", b"FA_BWD_VARIANT", b"FA_FWD_ABL"):
        assert key not in data
    import subprocess
    nm = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True)
    if nm.returncode == 0:
        assert "getenv" not in nm.stdout


def test_backward_rejects_mismatched_dtypes():
    """flash_attention_backward.cc:51-154 types: q,k,v,o,m: T; l: float (Float16 ops) or T."""
    import torch
    t = lambda *s, dt=torch.float16: torch.zeros(s, dtype=dt)  # noqa: E731
    Q, K, V, Oo, l, m, dO = (t(1, 8, 16), t(1, 8, 12), t(1, 8, 12), t(1, 8, 16), t(1, 16, dt=torch.float32),
                             t(1, 16), t(1, 8, 16))
    with pytest.raises(fa.InvalidArgumentError):  # all well-typed: only the device check fails on CPU
        fa.attention_backward("full", 1, Q, K, V, Oo, l, m, dO, "none_front")
    cases = {"K": dict(K=t(1, 8, 12, dt=torch.float32)), "V": dict(V=t(1, 8, 12, dt=torch.float32)),
             "O": dict(O=t(1, 8, 16, dt=torch.float32)), "m": dict(m=t(1, 16, dt=torch.float32)),
             "l": dict(l=t(1, 16))}
    for name, over in cases.items():
        args = dict(Q=Q, K=K, V=V, O=Oo, l=l, m=m, dO=dO)
        args.update(over)
        with pytest.raises(TypeError, match=name):
            fa.attention_backward("full", 1, args["Q"], args["K"], args["V"], args["O"], args["l"], args["m"],
                                  args["dO"], "none_front")
    Q32 = [x.float() for x in (Q, K, V, Oo)]
    with pytest.raises(TypeError, match="l must be"):  # fp32 op: l is T, not float16
        fa.attention_backward("full", 1, *Q32, t(1, 16), t(1, 16, dt=torch.float32), dO.float(), "none_front")


def test_backward_workspace_size():
    p = _prob("causal", [100], [60], b=3, d=16, vd=8, dtype=_lib.F16)
    n = _lib.lib().fa_backward_workspace_bytes(p)
    assert n >= 4 * 3 * 16 * 100 + 2 * 4 * 3 * 100
    p.dtype = _lib.F64
    assert _lib.lib().fa_backward_workspace_bytes(p) >= 8 * 3 * 16 * 100


def test_estimate_flops_is_algorithmic():
    # config 2 FLOPs = 4*64*128*4096^2
    flops = fa.estimate_forward_flops("full", 1, (8, 16, 64, 4096), (8, 16, 64, 4096), (8, 16, 64, 4096))
    assert flops == pytest.approx(549.755813888e9)
    f3 = fa.estimate_forward_flops("causal", 1, (8, 16, 128, 8192), (8, 16, 128, 8192), (8, 16, 128, 8192),
                                   "none_front")
    assert f3 == pytest.approx(512 * 128 * 8192 * 8193 / 2)
    f4 = fa._fa_kernel.estimate_local_attention_forward1d_flops((64, 16, 64, 16384), (64, 16, 64, 16384),
                                                                 (64, 16, 64, 16384), sync_mode="none_front",
                                                                 window_size=256, log2_stride_size=0,
                                                                 is_causal=False)
    assert f4 == pytest.approx(256 * 1024 * (16384 * 511 - 256 * 255))


def test_shape_error_messages_match_reference():
    """Messages of VerifyAndExtractShapes (flash_attention_forward.cc:100-133)."""
    V = fa.verify_and_extract_shapes
    with pytest.raises(fa.InvalidArgumentError, match="The number of dimensions of Q, K, and V should be equal"):
        V(1, (1, 2, 8, 16), (2, 8, 16), (1, 2, 8, 16))
    with pytest.raises(fa.InvalidArgumentError, match="should be >= 4"):
        V(2, (2, 8, 16), (2, 8, 16), (2, 8, 16))
    with pytest.raises(fa.InvalidArgumentError, match="The channel dimension of Q and K should be equal"):
        V(1, (1, 2, 8, 16), (1, 2, 4, 16), (1, 2, 8, 16))
    with pytest.raises(fa.InvalidArgumentError) as e:
        V(1, (1, 2, 8, 16), (1, 3, 8, 16), (1, 2, 8, 16))
    assert str(e.value) == ("The batch shape of all inputs should be equal, but Q_batch_shape = [1,2], "
                            "K_batch_shape = [1,3], V_batch_shape = [1,2] were received")
    with pytest.raises(fa.InvalidArgumentError) as e:
        V(1, (1, 2, 8, 16), (1, 2, 8, 16), (1, 2, 8, 15))
    assert str(e.value) == ("The sequence shape of K and V are expected to be equal, but K_seq_shape = [16], "
                            "V_seq_shape = [15] are detected")
    Qb, Qs, Qch, Kb, Ks, Kch, Vb, Vs, Vch = V(2, (3, 8, 4, 5), (3, 8, 6, 7), (3, 2, 6, 7))
    assert (Qb, Qs, Qch, Ks, Vch) == ((3,), (4, 5), 8, (6, 7), 2)


def test_backward_shape_errors():
    import torch
    t = lambda *s: torch.empty(s)  # noqa: E731
    Q, K, V, Oo, l, m, dO = t(1, 2, 8, 16), t(1, 2, 8, 12), t(1, 2, 4, 12), t(1, 2, 4, 16), t(1, 2, 16), t(1, 2, 16), \
        t(1, 2, 4, 16)
    fa.verify_backward_shapes(1, Q, K, V, Oo, l, m, dO)
    with pytest.raises(fa.InvalidArgumentError, match="The channel dimension of V and O should be equal"):
        fa.verify_backward_shapes(1, Q, K, V, t(1, 2, 5, 16), l, m, dO)
    with pytest.raises(fa.InvalidArgumentError, match="number of dimensions of l and m"):
        fa.verify_backward_shapes(1, Q, K, V, Oo, t(2, 16), m, dO)
    with pytest.raises(fa.InvalidArgumentError, match="The sequence shape of Q, O, l, m, and dO should be equal"):
        fa.verify_backward_shapes(1, Q, K, V, Oo, l, m, t(1, 2, 4, 15))


def test_op_surface_mirrors_reference_registrations():
    """12 forward + 12 backward ops (REGISTER_OP, flash_attention_forward.cc:144-253,
    flash_attention_backward.cc:51-154) + 6 flops estimators, TF snake_case names."""
    names = set(vars(fa._fa_kernel))
    for pol in ("full", "causal", "local"):
        for sd in (1, 2):
            for suf in ("", "_float16"):
                assert f"{pol}_attention_forward{sd}d{suf}" in names
                assert f"{pol}_attention_backward{sd}d{suf}" in names
            assert f"estimate_{pol}_attention_forward{sd}d_flops" in names
    assert len(names) == 30
    assert fa.gradient_op_for("CausalAttentionForward1dFloat16") is fa._fa_kernel.causal_attention_backward1d_float16
    assert fa.gradient_op_for("LocalAttentionForward2d") is fa._fa_kernel.local_attention_backward2d
    with pytest.raises(ValueError):
        fa.gradient_op_for("Bogus")


def _snake(name):
    return re.sub(r"(?<=[a-z0-9])(?=[A-Z])", "_", name).lower()


def test_tf_op_library_registers_the_same_ops():
    """tf_op/fa_tf_ops.cc (the TensorFlow-ROCm op library; not buildable here) registers exactly
    the 30 op names the Python mirror exposes — expanded from its registration macros."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "tf_flash_attention_amd", "tf_op",
                            "fa_tf_ops.cc")).read()
    dims = [int(x) for x in re.findall(r"^FA_REGISTER_OPS\((\d)\)", src, re.M)]
    body = src[src.index("#define FA_REGISTER_OPS(sd)"):].split("\n\n")[0]
    ops, kernels = set(), set()
    for sd in dims:
        for kind, fam in re.findall(r"FA_REGISTER_(FORWARD|BACKWARD|FLOPS)_OP\(\"(\w+)\"", body):
            if kind == "FLOPS":
                ops.add(f"Estimate{fam}{sd}dFlops")
            else:
                ops.update({f"{fam}{sd}dFloat16", f"{fam}{sd}d"})
    for fam, sd in re.findall(r"^FA_REGISTER_KERNELS\(\"(\w+)\", FA_\w+, (\d)\)", src, re.M):
        for d in ("Forward", "Backward"):
            kernels.update({f"{fam}{d}{sd}dFloat16", f"{fam}{d}{sd}d"})
        kernels.add(f"Estimate{fam}Forward{sd}dFlops")
    assert len(ops) == 30 and ops == kernels
    assert {_snake(o) for o in ops} == set(vars(fa._fa_kernel))


def test_cpu_tensors_fail_loudly():
    """No CPU fallback: host tensors are rejected, never computed by a slow path."""
    import torch
    x = torch.zeros(1, 2, 8, 16)
    with pytest.raises(fa.InvalidArgumentError, match="no CPU kernel"):
        fa.full_1d(x, x, x)


def test_using_override_rejects_overlap_across_threads():
    """_lib.using() routes the whole process; a second thread may not open a block while
    another thread's block is open (nesting within one thread is fine)."""
    import threading
    path = _lib.LIB_PATH
    errors = []
    inside = threading.Event()
    release = threading.Event()

    def holder():
        with _lib.using(path):
            with _lib.using(path):  # nested, same thread
                inside.set()
                release.wait(10)

    t = threading.Thread(target=holder)
    t.start()
    assert inside.wait(10)
    try:
        with _lib.using(path):
            pass
    except RuntimeError as e:
        errors.append(str(e))
    finally:
        release.set()
        t.join(10)
    assert errors and "another thread" in errors[0]
    with _lib.using(path):  # free again once the holder's blocks have closed
        pass
