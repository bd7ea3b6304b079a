"""Timing-only ablations of the streamlined fp16 forward (FA_FWD_VARIANT=1899, FA_FWD_ABL=<bits>):
each removes one part of the key loop (outputs are wrong) so its share of the time shows.
Usage: python tools/fwd_ablate.py [config] bits...   (0 = the full kernel)"""
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
    cfgname = args.pop(0) if args and args[0].startswith("c") else "c2"
    bits = args or ["0"]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    flops = fa.estimate_forward_flops(policy, seq_dims, q.shape, k.shape, v.shape, sync, ws, ls, causal)
    os.environ["FA_FWD_VARIANT"] = "1899"
    res = {x: [] for x in bits}
    for _ in range(3):
        for x in bits:
            os.environ["FA_FWD_ABL"] = x
            for _ in range(3):
                fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for a_, b_ in evs:
                a_.record()
                fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
                b_.record()
            torch.cuda.synchronize()
            res[x].append(float(np.median([a_.elapsed_time(b_) for a_, b_ in evs])))
    for x in bits:
        ms = min(res[x])
        print(json.dumps({"config": cfgname, "ablate": x, "ms": round(ms, 4), "tflops_equiv": round(flops / ms / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
