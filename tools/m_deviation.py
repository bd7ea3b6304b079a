"""Measure how far the fp16 kernels' m output lies from the float64 oracle's row max, in fp16
ulps, over a set of shapes (the number DESIGN.md §4 quotes for the fp16 m deviation).

  python tools/m_deviation.py [--lib path/to/libfa_hip*.so]   (GPU; FA_FWD_VARIANT applies with the diag library)

Prints one JSON line per case and a summary line: max |m - m64| (absolute), max in ulps of
fp16(m64), and the fraction of rows within 0 / 1 / 2 ulps.  Test infrastructure: reads the oracle.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [
    # policy, seq_dims, d, n, ws, causal
    ("full", 1, 64, 4096, 1, False),
    ("full", 1, 64, 1000, 1, False),
    ("causal", 1, 64, 2048, 1, False),
    ("local", 1, 64, 2048, 256, False),
    ("full", 1, 128, 2048, 1, False),
    ("causal", 1, 128, 2048, 1, False),
    ("full", 1, 48, 1024, 1, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--slices", type=int, default=4)
    args = ap.parse_args()
    if args.lib:
        os.environ["FA_HIP_LIB"] = args.lib
    import torch
    from oracle import fa_oracle as O
    from tf_flash_attention_amd import flash_attention as fa

    dev = torch.device("cuda:0")
    worst_abs, worst_ulp, tot, within = 0.0, 0.0, 0, np.zeros(3)
    for policy, sd, d, n, ws, causal in CASES:
        rng = np.random.default_rng(7)
        b = 8
        Q = rng.uniform(-2, 2, (b, d, n)).astype(np.float16)
        K = rng.uniform(-2, 2, (b, d, n)).astype(np.float16)
        V = rng.uniform(-2, 2, (b, d, n)).astype(np.float16)
        tq, tk, tv = (torch.from_numpy(x).to(dev) for x in (Q, K, V))
        o, l, m = fa.attention_forward(policy, sd, tq, tk, tv, "none_front", ws, 0, causal)
        torch.cuda.synchronize()
        sl = list(range(args.slices))
        prob = O.Problem(policy, sd, "none_front", ws, 0, causal)
        _, _, M64, ha = O.forward_f64(Q, K, V, prob, slices=sl)
        M64 = M64.reshape(len(sl), n)[:, ha]
        mg = m.cpu().numpy().reshape(b, n)[sl][:, ha].astype(np.float64)
        ulp = np.abs(np.spacing(np.abs(M64).astype(np.float16))).astype(np.float64)
        err = np.abs(mg - M64)
        # rounding the exact max to fp16 already costs up to half an ulp: count against fp16(m64)
        eu = np.abs(mg - M64.astype(np.float16).astype(np.float64)) / ulp
        rec = {"policy": policy, "d": d, "n": n, "ws": ws, "max_abs": float(err.max()),
               "max_ulp": float(eu.max()), "frac_exact": float((eu == 0).mean()),
               "frac_le1": float((eu <= 1).mean()), "max_rel": float((err / np.maximum(np.abs(M64), 1e-30)).max())}
        print(json.dumps(rec), flush=True)
        worst_abs, worst_ulp = max(worst_abs, rec["max_abs"]), max(worst_ulp, rec["max_ulp"])
        tot += eu.size
        within += [(eu == 0).sum(), (eu <= 1).sum(), (eu <= 2).sum()]
    print(json.dumps({"summary": True, "variant": os.environ.get("FA_FWD_VARIANT", "default"),
                      "max_abs": worst_abs, "max_ulp": worst_ulp,
                      "frac_exact": within[0] / tot, "frac_le1ulp": within[1] / tot, "frac_le2ulp": within[2] / tot}))


if __name__ == "__main__":
    main()
