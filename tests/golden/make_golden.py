"""Generates tests/golden/config1_full1d_f32.npz from the oracle (seeded numpy PCG64).

Config 1 of BASELINE.json: full_1d fp32 B=2 H=4 d=32 N=128, inputs ~U(-2,2)
(tests/test_base.py:170-173 draws U(-2,2) with seed 1234; TF's RNG stream is not
reproducible without TF, so numpy PCG64 seed 1234 is used instead).

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import fa_oracle as O  # noqa: E402


def main():
    rng = np.random.default_rng(1234)
    shape = (2, 4, 32, 128)
    Q = rng.uniform(-2, 2, shape).astype(np.float32)
    K = rng.uniform(-2, 2, shape).astype(np.float32)
    V = rng.uniform(-2, 2, shape).astype(np.float32)
    dO = rng.uniform(-2, 2, shape).astype(np.float32)
    prob = O.Problem("full", 1, "none_front")
    Oo, lo, mo = O.forward(Q, K, V, prob)
    dQ, dK, dV = O.backward_f64(Q, K, V, dO, prob)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config1_full1d_f32.npz")
    np.savez_compressed(out, Q=Q, K=K, V=V, dO=dO, O=Oo, l=lo, m=mo,
                        dQ=dQ.astype(np.float32), dK=dK.astype(np.float32), dV=dV.astype(np.float32))
    print("wrote", out)


if __name__ == "__main__":
    main()
