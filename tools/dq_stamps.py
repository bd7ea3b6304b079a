"""Phase breakdown of the producer / consumer dQ pass (FA_BWD_VARIANT=1604, diagnostic library):
per-wave s_memtime sums per step part, read back from the dQ workspace (c3 shape).
Producer parts: barrier, half-0 S/dP MFMAs, half-0 softmax + hand-over, half-1 MFMAs, half-1 softmax.
Consumer parts: barrier, staging (stores + loads), hand-over reads, dQ MFMAs (+ K reads).
Usage: python tools/dq_stamps.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FA_HIP_LIB", os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip_diag.so"))
os.environ["FA_BWD_VARIANT"] = "1604"
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
    nqb = qs[0] // 128
    nwg = b * nqb
    x = wsb[: nwg * 8 * 8 * 8].view(torch.int64).cpu().numpy().reshape(nwg, 8, 8)[:, :, :5].astype(np.float64)
    # the dQ pass launches heaviest query blocks first: block id -> q0 = (nqb - 1 - bid % nqb) * 128;
    # steps = ntiles + 1 rounded up to 4, ntiles = (q0 + 128) / 64 under the causal rule
    q0 = (nqb - 1 - np.arange(nwg) % nqb) * 128
    steps = (((q0 + 128) // 64) + 1 + 3) // 4 * 4
    per = x / steps[:, None, None]
    names = {0: ["barrier", "S/dP half 0", "softmax half 0", "S/dP half 1", "softmax half 1"],
             1: ["barrier", "staging", "hand-over reads", "dQ MFMAs", "-"]}
    for grp, role in ((0, "producer"), (1, "consumer")):
        y = per[:, 4 * grp:4 * grp + 4, :].reshape(-1, 5).mean(axis=0)
        print(json.dumps({"role": role, "cycles_per_step": round(float(y.sum()), 1),
                          "parts": {n_: round(float(v_), 1) for n_, v_ in zip(names[grp], y)}}), flush=True)


if __name__ == "__main__":
    main()
