"""Phase shares of the d = 128 ping-pong forward from its stamp build (FA_FWD_VARIANT=2361; 2304 / 2359 add stamps inside the MFMA phase):
per-wave s_memtime sums over the key loop, written over l.  Usage: python tools/pp128_stamps.py [config] [variant]"""
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
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c3"
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    os.environ["FA_FWD_VARIANT"] = sys.argv[2] if len(sys.argv) > 2 else "2361"
    for _ in range(5):
        o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    nq = int(np.prod(qs))
    lw = l.reshape(b, nq // 256, 8, 32)[:, :, :, :10].float().cpu().numpy()  # [b, blocks, wave, part]
    names = ["barrier before MFMA", "MFMA phase (rest)", "barrier before VALU", "softmax phase", None,
             "stores+loads", "QK half 0", "reads + PV half 0", "reads + QK half 1", "PV half 1"]
    if os.environ["FA_FWD_VARIANT"] in ("2345", "2346", "2347"):  # the staging-wait stamp builds
        names[5:8] = ["to staging", "staging loads' wait", "stores + loads issue"]
    if os.environ["FA_FWD_VARIANT"] == "2347":
        names[7:9] = ["loads issue", "stores (to completion)"]
    for grp in (0, 1):
        x = lw[:, :, 4 * grp:4 * grp + 4, :].reshape(-1, 10)
        per = x.sum(axis=0) / x[:, 4].sum()
        per[4] = 0.0
        print(json.dumps({"config": cfgname, "group": grp, "cycles_per_step": round(float(per.sum()), 1),
                          "parts": {n: round(float(v), 1) for n, v in zip(names, per) if n and v > 0}}), flush=True)


if __name__ == "__main__":
    main()
