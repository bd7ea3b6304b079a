"""A/B timing of two builds of the product library in ONE process (interleaved rounds), through
_lib.using(): the forward and the backward of a bench config, with a bitwise check of every output
against the first library.  Usage: python tools/lib_ab.py [config] libA.so libB.so ..."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_flash_attention_amd import _lib  # noqa: E402
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    cfgname = args.pop(0) if args and args[0] in bench.CONFIGS else "c3"
    libs = [os.path.abspath(x) for x in args]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, _, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    mk = lambda shp: (torch.rand(shp, generator=g, device=dev) * 4 - 2).to(dt)  # noqa: E731
    q, k, v, do = mk((b, d) + qs), mk((b, d) + ks), mk((b, d) + ks), mk((b, d) + qs)
    fwd = lambda: fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)  # noqa: E731
    ref = None
    res = {x: {"fwd": [], "bwd": []} for x in libs}
    for rnd in range(5):
        for x in libs:
            with _lib.using(x):
                o, l, m = fwd()
                bwd = lambda: fa.attention_backward(policy, seq_dims, q, k, v, o, l, m, do, sync, ws, ls, causal)  # noqa: E731
                outs = [o, l, m] + list(bwd())
                torch.cuda.synchronize()
                if rnd == 0:
                    if ref is None:
                        ref = [t.clone() for t in outs]
                    same = all(torch.equal(t, r) for t, r in zip(outs, ref))
                    print(f"{os.path.basename(x)}: outputs bitwise equal to the first library: {same}", flush=True)
                for name, fn in (("fwd", fwd), ("bwd", bwd)):
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
                    for a_, b_ in evs:
                        a_.record()
                        fn()
                        b_.record()
                    torch.cuda.synchronize()
                    res[x][name].append(float(np.median([a_.elapsed_time(b_) for a_, b_ in evs])))
    for x in libs:
        print(json.dumps({"config": cfgname, "lib": os.path.basename(x),
                          "fwd_ms": [round(t, 3) for t in res[x]["fwd"]],
                          "bwd_ms": [round(t, 3) for t in res[x]["bwd"]]}), flush=True)


if __name__ == "__main__":
    main()
