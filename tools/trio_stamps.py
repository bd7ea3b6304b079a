"""Phase breakdown of the three-group rotation forward from its stamp build (FA_FWD_VARIANT=2503):
per-wave s_memtime sums (MFMA phase, softA, softB, barrier waits) written over l, per group.
Usage: python tools/trio_stamps.py [config] [variant]"""
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
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c2"
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    os.environ["FA_FWD_VARIANT"] = sys.argv[2] if len(sys.argv) > 2 else "2503"
    for _ in range(5):
        o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    nq = int(np.prod(qs))
    nfull = nq // 384
    # [b, full blocks, wave, lane r < 4] (the ragged last block is left out)
    lw = l.reshape(b, nq)[:, :nfull * 384].reshape(b, nfull, 12, 32)[:, :, :, :4].float().cpu().numpy()
    rounds = int(np.prod(ks)) // 64 + 1
    rounds += rounds % 2
    names = ["MFMA phase", "softA", "softB", "barrier waits"]
    for grp in (0, 1, 2):
        x = lw[:, :, 4 * grp:4 * grp + 4, :].reshape(-1, 4).mean(axis=0) / rounds
        print(json.dumps({"config": cfgname, "group": grp, "cycles_per_round": round(float(x.sum()), 1),
                          "parts": {n: round(float(v), 1) for n, v in zip(names, x)}}), flush=True)


if __name__ == "__main__":
    main()
