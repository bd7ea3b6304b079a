"""Phase timeline of the persistent band forward from the stamp build (tools/stamp/build.sh):
s_memtime of waves 0 (group 0) and 4 (group 1) of workgroup 0 at the four phase edges of every
position of its first four items (written over the last slice's Q; outputs WRONG).
Usage: python tools/stamp/band_stamps.py [T]   (T: positions an item, 10 for c4)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["FA_HIP_LIB"] = os.path.join(ROOT, "tools", "stamp", "build", "libfa_hip_stamp.so")
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def main():
    cfg = bench.CONFIGS["c4"]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = cfg
    dev = torch.device("cuda:0")
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, device=dev) * 4 - 2).to(dt)
    for _ in range(200):  # clock ramp (the stamps land in q's last slice: refreshed below)
        fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    q[-1].uniform_(-2, 2)
    fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    t = q[-1].reshape(-1).view(torch.int64)[: 4 * T * 4 * 2].cpu().numpy().reshape(4 * T, 4, 2).astype(np.int64)
    for g in range(2):
        ts = t[:, :, g]
        mf = ts[:, 1] - ts[:, 0]
        bar1 = ts[:, 2] - ts[:, 1]
        va = ts[:, 3] - ts[:, 2]
        bar0 = ts[1:, 0] - ts[:-1, 3]
        print(f"group {g}: per position  mfma {np.median(mf):.0f}  wait->valu {np.median(bar1):.0f}  valu {np.median(va):.0f}"
              f"  wait->mfma {np.median(bar0):.0f}  total {np.median(np.diff(ts[:, 0])):.0f} cycles")
        for p in range(2 * T, 4 * T):
            print(f"  pos {p:2d} it {p % T:2d}: mfma {mf[p]:6d} wait {bar1[p]:6d} valu {va[p]:6d} "
                  f"{'wait ' + str(bar0[p]) if p < len(bar0) else ''}")


if __name__ == "__main__":
    main()
