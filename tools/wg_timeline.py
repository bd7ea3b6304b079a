"""Workgroup timeline of the ping-pong forward (FA_FWD_VARIANT=2204 build): per-workgroup entry /
prologue / loop / exit times and the gap between consecutive workgroups on one CU.
Usage: python tools/wg_timeline.py [nk]   (c2 shape: b=128, d=64, nq=4096)"""
import collections
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


def main():
    nk = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    os.environ["FA_FWD_VARIANT"] = sys.argv[2] if len(sys.argv) > 2 else "2204"  # 2274-2276: ablations
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    b, d, nq = 128, 64, 4096
    q = (torch.rand((b, d, nq), generator=g, device=dev) * 4 - 2).half()
    k = (torch.rand((b, d, nk), generator=g, device=dev) * 4 - 2).half()
    v = (torch.rand((b, d, nk), generator=g, device=dev) * 4 - 2).half()
    for _ in range(30):  # long enough for the clock to settle
        o, l, m = fa.full_1d(q, k, v, returning_l_m=True)
    torch.cuda.synchronize()
    raw = l.detach().contiguous().view(torch.int32).cpu().numpy().reshape(b, nq).astype(np.uint32)
    nqb = nq // 256
    rec = raw.reshape(b, nqb, 256)[:, :, :10].reshape(-1, 10).astype(np.uint64)
    t0 = rec[:, 0] + (rec[:, 1] << np.uint64(32))
    pro, loop, end = rec[:, 2].astype(np.int64), rec[:, 3].astype(np.int64), rec[:, 4].astype(np.int64)
    cpro, cloop, cend = rec[:, 5].astype(np.int64), rec[:, 6].astype(np.int64), rec[:, 7].astype(np.int64)
    hw, xcc = rec[:, 8].astype(np.int64), rec[:, 9].astype(np.int64)
    cu = (xcc & 0xF) * 256 + ((hw >> 8) & 0xFF)
    t0 = (t0 - t0.min()).astype(np.int64)
    gaps = []
    per_cu = collections.defaultdict(list)
    for i in range(len(t0)):
        per_cu[int(cu[i])].append((int(t0[i]), int(t0[i] + end[i])))
    for lst in per_cu.values():
        lst.sort()
        for (s0, e0), (s1, e1) in zip(lst, lst[1:]):
            gaps.append(s1 - e0)
    tick_ns = 10.0  # s_memrealtime: 100 MHz
    out = {
        "nk": nk, "variant": os.environ["FA_FWD_VARIANT"], "workgroups": int(len(t0)), "cus_seen": len(per_cu),
        "wg_per_cu_mean": float(np.mean([len(x) for x in per_cu.values()])),
        "span_us": float((t0 + end).max() * tick_ns / 1e3),
        "wg_us_mean": float(end.mean() * tick_ns / 1e3),
        "prologue_us_mean": float(pro.mean() * tick_ns / 1e3),
        "loop_us_mean": float((loop - pro).mean() * tick_ns / 1e3),
        "epilogue_us_mean": float((end - loop).mean() * tick_ns / 1e3),
        "cycles_prologue": float(cpro.mean()), "cycles_loop": float((cloop - cpro).mean()),
        "cycles_epilogue": float((cend - cloop).mean()),
        "clock_ghz": float((cend.mean()) / (end.mean() * tick_ns)),
        "gap_us_mean": float(np.mean(gaps) * tick_ns / 1e3) if gaps else None,
        "gap_us_p90": float(np.percentile(gaps, 90) * tick_ns / 1e3) if gaps else None,
        "first_start_spread_us": float(np.sort(t0)[min(255, len(t0) - 1)] * tick_ns / 1e3),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
