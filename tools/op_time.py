"""Times forward and backward separately for a bench config (event-timed, median of N).
Usage: python tools/op_time.py [c2|c3|c4|c5] [--b B]  (B overrides the flattened batch)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="c3")
    ap.add_argument("--b", type=int, default=None)
    args = ap.parse_args()
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, _, _ = bench.CONFIGS[args.config]
    b = args.b or int(np.prod(batch))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda shp: (torch.rand(shp, generator=g, device=dev) * 4 - 2).to(dt)  # noqa: E731
    q, k, v, do = mk((b, d) + qs), mk((b, d) + ks), mk((b, d) + ks), mk((b, d) + qs)
    ff = fa.estimate_forward_flops(policy, seq_dims, q.shape, k.shape, v.shape, sync, ws, ls, causal)
    pairs = ff / (4.0 * d)
    bf = 10.0 * d * pairs
    o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    tf = timeit(lambda: fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal))
    tb = timeit(lambda: fa.attention_backward(policy, seq_dims, q, k, v, o, l, m, do, sync, ws, ls, causal))
    print(json.dumps({"config": args.config, "b": b, "fwd_ms": round(tf, 4), "fwd_tflops": round(ff / tf / 1e9, 1),
                      "bwd_ms": round(tb, 4), "bwd_tflops": round(bf / tb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
