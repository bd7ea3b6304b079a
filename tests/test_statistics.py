"""The 'flops' statistic of the forward ops (the reference's ops.RegisterStatistics hooks,
flash_attention.py:475-562): name dispatch, attrs, and the error for other ops.  CPU only: the
estimate is a host function of the C ABI (fa_estimate_forward_flops)."""
import pytest

from tf_flash_attention_amd import flash_attention as fa

SHAPE1 = ((2, 4, 32, 300), (2, 4, 32, 500), (2, 4, 16, 500))
SHAPE2 = ((2, 8, 12, 10), (2, 8, 24, 20), (2, 8, 24, 20))


@pytest.mark.parametrize("op", fa._STAT_OPS)
def test_statistic_matches_estimate(op):
    sd = 2 if "2d" in op else 1
    q, k, v = SHAPE2 if sd == 2 else SHAPE1
    policy = op.split("Attention")[0].lower()
    attrs = {"sync_mode": "scale_front", "window_size": 5, "log2_stride_size": 1, "is_causal": True}
    got = fa.forward_flops_statistics(op, q, k, v, attrs)
    kw = {"sync_mode": "scale_front"}
    if policy == "local":
        kw.update(window_size=5, log2_stride_size=1, is_causal=True)
    assert got == fa.estimate_forward_flops(policy, sd, q, k, v, **kw)
    assert got > 0


def test_statistic_local_attrs_matter():
    q, k, v = SHAPE1
    base = {"sync_mode": "none_front", "log2_stride_size": 0, "is_causal": False}
    narrow = fa.forward_flops_statistics("LocalAttentionForward1d", q, k, v, dict(base, window_size=4))
    wide = fa.forward_flops_statistics("LocalAttentionForward1dFloat16", q, k, v, dict(base, window_size=64))
    assert 0 < narrow < wide


@pytest.mark.parametrize("op", ["FullAttentionBackward1d", "FullAttentionForward3d", "Foo", "CausalAttentionForward1dFloat32"])
def test_statistic_rejects_other_ops(op):
    with pytest.raises(ValueError, match="Unsupported op"):
        fa.forward_flops_statistics(op, *SHAPE1, {"sync_mode": "none_front"})


def test_register_without_tensorflow():
    try:
        import tensorflow  # noqa: F401
    except ImportError:
        assert fa.register_tf_statistics() is False
        return
    assert fa.register_tf_statistics() is True
