"""A/B timing of forward structure variants in ONE process (interleaved rounds),
selected through FA_FWD_VARIANT.  Usage: [FV_POLICY=full|causal] [FV_D=d] [FV_BATCH=b,h] python tools/fwd_variants.py [config] v1 v2 ..."""
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
    cfgname = args.pop(0) if args and args[0] in bench.CONFIGS else "c2"
    variants = args or ["-1"]
    cfg = bench.CONFIGS[cfgname]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = cfg
    policy = os.environ.get("FV_POLICY", policy)  # e.g. FV_POLICY=full: config 3's shape without the mask
    d = int(os.environ.get("FV_D", d))  # e.g. FV_D=128: config 4's band at d = 128
    if "FV_BATCH" in os.environ:  # e.g. FV_BATCH=8,16
        batch = tuple(int(x) for x in os.environ["FV_BATCH"].split(","))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    flops = fa.estimate_forward_flops(policy, seq_dims, q.shape, k.shape, v.shape, sync, ws, ls, causal)
    ref = None
    res = {vv: [] for vv in variants}
    # clock ramp: ~1.5 s of back-to-back launches before the first timed round
    os.environ["FA_FWD_VARIANT"] = variants[0]
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    while True:
        for _ in range(20):
            fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        torch.cuda.synchronize()
        if t0.elapsed_time(t1) > 1500:
            break
    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for vv in variants:
            os.environ["FA_FWD_VARIANT"] = vv
            for _ in range(3):
                o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
            torch.cuda.synchronize()
            if rnd == 0:
                if ref is None:
                    ref = o.float()
                err = (o.float() - ref).abs().max().item()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for a_, b_ in evs:
                a_.record()
                fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
                b_.record()
            torch.cuda.synchronize()
            ms = float(np.median([a_.elapsed_time(b_) for a_, b_ in evs]))
            res[vv].append(ms)
            if rnd == 0:
                print(f"variant {vv}: max|o - o_first| = {err:.3e}", flush=True)
    for vv in variants:
        ms = min(res[vv])
        print(json.dumps({"config": cfgname, "variant": vv, "ms": [round(x, 4) for x in res[vv]],
                          "tflops": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
