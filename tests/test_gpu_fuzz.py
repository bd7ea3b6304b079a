"""Seeded random sweep over the op's whole parameter space against the float64 oracle (the same check
as test_gpu_parity.run_case): dtype, policy, 1d / 2d, sync mode, channel counts 1..256 (d != v_d),
ragged and tiny lengths, window sizes and strides, look-ahead, misaligned tensors.  Each case is drawn
from its own seed, so a failure names a reproducible case.  FA_FUZZ_N sets the number of cases (400 by
default; the round-5 runs are recorded in DESIGN.md §4); FA_FUZZ_LARGE=1 draws the reference tests'
lengths (1d up to 4096, 2d up to 64 x 64) at d <= 128."""
import os

import numpy as np
import pytest

from tests.test_gpu_parity import run_case

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("FA_FUZZ_N", "400"))
START = int(os.environ.get("FA_FUZZ_START", "0"))  # (long sweeps run in slices: cases START .. N_CASES-1)
LARGE = os.environ.get("FA_FUZZ_LARGE", "") == "1"  # lengths up to 4096 (1d) / 64 x 64 (2d), d <= 128
CHANNELS = [1, 3, 8, 16, 24, 32, 48, 64, 65, 96, 100, 128, 129, 160, 200, 256]


def draw(i):
    rng = np.random.default_rng(1_000_003 * (i + 1))
    dtype = [np.float16, np.float32, np.float64][rng.integers(3)]
    policy = ["full", "causal", "local"][rng.integers(3)]
    seq = 1 if rng.random() < 0.7 else 2
    mode = ["none_front", "scale_front", "scale_end"][rng.integers(3)]
    chans = CHANNELS[:12] if LARGE else CHANNELS
    d = int(chans[rng.integers(len(chans))])
    vd = d if rng.random() < 0.6 else int(chans[rng.integers(len(chans))])
    if seq == 1:
        lim = 4097 if LARGE else (700 if max(d, vd) <= 128 else 400)
        qs = (int(rng.integers(1, lim)),)
        ks = (int(rng.integers(1, lim)),) if rng.random() < 0.6 else qs
    else:
        lim = 65 if LARGE else 25
        qs = (int(rng.integers(1, lim)), int(rng.integers(1, lim)))
        ks = (int(rng.integers(1, lim)), int(rng.integers(1, lim))) if rng.random() < 0.6 else qs
    ws = int(rng.integers(1, (300 if LARGE else 80) if seq == 1 else 10))
    ls = int(rng.integers(0, 4)) if rng.random() < 0.5 else 0
    causal = bool(rng.random() < 0.5)
    misalign = bool(rng.random() < 0.15)
    batch = (int(rng.integers(1, 3)),)
    return dict(dtype=dtype, policy=policy, seq_dims=seq, mode=mode, batch=batch, d=d, vd=vd, qs=qs, ks=ks, ws=ws,
                ls=ls, causal=causal, misalign=misalign, seed=i)


def _id(i):
    c = draw(i)
    return (f"{i}-{np.dtype(c['dtype']).name}-{c['policy']}{c['seq_dims']}d-{c['mode']}-d{c['d']}v{c['vd']}-"
            f"q{'x'.join(map(str, c['qs']))}k{'x'.join(map(str, c['ks']))}"
            + (f"-w{c['ws']}s{c['ls']}{'c' if c['causal'] else ''}" if c["policy"] == "local" else "")
            + ("-mis" if c["misalign"] else ""))


@pytest.mark.parametrize("i", range(START, N_CASES), ids=_id)
def test_fuzz_case(i):
    c = draw(i)
    run_case(c["dtype"], c["policy"], c["seq_dims"], c["mode"], c["batch"], c["d"], c["vd"], c["qs"], c["ks"],
             ws=c["ws"], ls=c["ls"], causal=c["causal"], seed=c["seed"], misalign=c["misalign"])


# seeds past the default range whose gradients are sums of large cancelling terms (one or two keys,
# d = 1 scores): the cases that shaped the rounding scale of test_gpu_parity (profiles/r05_fuzz20000.txt,
# r05_fuzz60000.txt), kept in the default suite
CANCELLING = [4430, 5575, 5806, 11060, 12759, 14319, 16424, 17566, 19100, 19286, 19452, 32191, 50464, 53126]


@pytest.mark.parametrize("i", CANCELLING, ids=_id)
def test_fuzz_cancelling_case(i):
    test_fuzz_case(i)


# seeds past the default range whose correct gradients reached the scale-slope tolerance of tests/gate.py:
# 28600 (fp32, d = 256, five queries and keys), 41712 (fp16, dQ resting on one query row), 72261 (fp16,
# d = 1, rounding coherent over the whole dK); profiles/r06_fuzz20000.txt, r06_fuzz100000.txt, DESIGN.md §4
COHERENT = [28600, 41712, 72261]


@pytest.mark.parametrize("i", COHERENT, ids=_id)
def test_fuzz_coherent_case(i):
    test_fuzz_case(i)
