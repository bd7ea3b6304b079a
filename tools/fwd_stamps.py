"""Phase breakdown of the streamlined fp16 forward's key loop from a diagnostic build
(FA_FWD_VARIANT=1899, FA_FWD_ABL=4096): per-wave s_memtime sums written over l.
Usage: python tools/fwd_stamps.py [config] [abl]"""
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
    abl = args[0] if args else "4096"
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    os.environ["FA_FWD_VARIANT"] = "1899"
    os.environ["FA_FWD_ABL"] = abl
    for _ in range(5):
        o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    nq = int(np.prod(qs))
    lw = l.reshape(b, nq // 32, 32)[:, :, :7].float().cpu().numpy().reshape(-1, 7)
    tot = lw.sum(axis=1, keepdims=True)
    share = (lw / tot).mean(axis=0)
    names = ["barrier", "loads+mask", "qk+max", "rebase+exp+pv", "loop overhead", "frag reads", "lds stores"]
    print(json.dumps({"config": cfgname, "abl": abl, "mean_cycles_per_wave": float(tot.mean()),
                      "share": {n: round(float(x), 4) for n, x in zip(names, share)}}), flush=True)


if __name__ == "__main__":
    main()
