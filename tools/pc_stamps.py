"""Phase breakdown of the producer / consumer dK/dV pass (FA_BWD_VARIANT=1404 / 1406, diagnostic
library): per-wave s_memtime sums per step part, read back from the dQ workspace.
Usage: python tools/pc_stamps.py [variant]   (c3 shape)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FA_HIP_LIB", os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip_diag.so"))
os.environ["FA_BWD_VARIANT"] = sys.argv[1] if len(sys.argv) > 1 else "1404"
from tf_flash_attention_amd import _lib, flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def main():
    policy, sd, dt, batch, d, qs, ks, sync, ws, ls, causal, _, _ = bench.CONFIGS["c3"]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    b = int(np.prod(batch))
    mk = lambda shp: (torch.rand(shp, generator=g, device=dev) * 4 - 2).to(dt)  # noqa: E731
    q, k, v, do = mk((b, d) + qs), mk((b, d) + ks), mk((b, d) + ks), mk((b, d) + qs)
    o, l, m = fa.attention_forward(policy, sd, q, k, v, sync, ws, ls, causal)
    prob = _lib.make_problem(_lib.F16, fa._POLICIES[policy], sd, fa._sync_mode_id(sync), b, qs, ks, d, d, ws, ls, causal)
    L = _lib.lib()
    nbytes = L.fa_backward_workspace_bytes(prob)
    wsb = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(3):
        st = L.fa_backward(fa._stream_handle(dev), prob, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                           l.data_ptr(), m.data_ptr(), do.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                           wsb.data_ptr(), nbytes)
        assert st == 0
    torch.cuda.synchronize()
    nwg = b * ((qs[0] + 127) // 128)
    x = wsb[: nwg * 8 * 4 * 8].view(torch.int64).cpu().numpy().reshape(nwg, 8, 4)[:, :, :3].astype(np.float64)
    # steps per workgroup: ntiles + 1 rounded up to 4 (causal: tiles from the block's diagonal on)
    k0 = (np.arange(nwg) % (ks[0] // 128)) * 128
    steps = ((qs[0] - k0) // 32 + 1 + 3) // 4 * 4
    per = x / steps[:, None, None]
    names = ["stage+barrier", "MFMA part", "softmax/hand-over part"]
    for grp, role in ((0, "producer"), (1, "consumer")):
        y = per[:, 4 * grp:4 * grp + 4, :].reshape(-1, 3).mean(axis=0)
        print(json.dumps({"role": role, "cycles_per_step": round(float(y.sum()), 1),
                          "parts": {n_: round(float(v_), 1) for n_, v_ in zip(names, y)}}), flush=True)


if __name__ == "__main__":
    main()
