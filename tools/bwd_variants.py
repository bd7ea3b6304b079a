"""A/B timing of backward variants (FA_BWD_VARIANT) in one process, interleaved rounds, with a
max-abs check of dQ/dK/dV against the first variant.  Usage: python tools/bwd_variants.py [config] v1 v2 ..."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# variant / ablation / stamp builds live only in the diagnostic library (make -C tf_flash_attention_amd diag)
os.environ.setdefault("FA_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "tf_flash_attention_amd", "libfa_hip_diag.so"))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    cfgname = args.pop(0) if args and args[0] in bench.CONFIGS else "c3"
    variants = args or ["-1"]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, _, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    mk = lambda shp: (torch.rand(shp, generator=g, device=dev) * 4 - 2).to(dt)  # noqa: E731
    q, k, v, do = mk((b, d) + qs), mk((b, d) + ks), mk((b, d) + ks), mk((b, d) + qs)
    o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    ff = fa.estimate_forward_flops(policy, seq_dims, q.shape, k.shape, v.shape, sync, ws, ls, causal)
    bf = 10.0 * d * ff / (4.0 * d)
    ref, res = None, {x: [] for x in variants}
    for rnd in range(3):
        for x in variants:
            os.environ["FA_BWD_VARIANT"] = x
            run = lambda: fa.attention_backward(policy, seq_dims, q, k, v, o, l, m, do, sync, ws, ls, causal)  # noqa: E731
            for _ in range(2):
                grads = run()
            torch.cuda.synchronize()
            if rnd == 0:
                if ref is None:
                    ref = [t.float() for t in grads]
                err = max((t.float() - r).abs().max().item() for t, r in zip(grads, ref))
                print(f"variant {x}: max|grad - grad_first| = {err:.3e}", flush=True)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a_, b_ in evs:
                a_.record()
                run()
                b_.record()
            torch.cuda.synchronize()
            res[x].append(float(np.median([a_.elapsed_time(b_) for a_, b_ in evs])))
    for x in variants:
        ms = min(res[x])
        print(json.dumps({"config": cfgname, "variant": x, "ms": [round(t, 3) for t in res[x]],
                          "bwd_tflops": round(bf / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
