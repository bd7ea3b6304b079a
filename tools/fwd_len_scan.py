"""Forward time vs key length at fixed queries (full policy, fp16, d=64, b=128, nq=4096): separates
per-workgroup fixed cost (prologue / epilogue / launch) from per-key-tile cost.
Usage: python tools/fwd_len_scan.py [variant]"""
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
    if len(sys.argv) > 1:
        os.environ["FA_FWD_VARIANT"] = sys.argv[1]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    b, d, nq = 128, 64, 4096
    q = (torch.rand((b, d, nq), generator=g, device=dev) * 4 - 2).half()
    res = []
    for nk in (1024, 2048, 4096, 8192):
        k = (torch.rand((b, d, nk), generator=g, device=dev) * 4 - 2).half()
        v = (torch.rand((b, d, nk), generator=g, device=dev) * 4 - 2).half()
        for _ in range(20):
            fa.full_1d(q, k, v)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a_, b_ in evs:
            a_.record()
            fa.full_1d(q, k, v)
            b_.record()
        torch.cuda.synchronize()
        ms = float(np.median([a_.elapsed_time(b_) for a_, b_ in evs]))
        res.append((nk, ms))
        print(json.dumps({"nk": nk, "ms": round(ms, 4), "tflops": round(4 * d * b * nq * nk / ms / 1e9, 1)}), flush=True)
    x = np.array([r[0] for r in res], dtype=float)
    y = np.array([r[1] for r in res])
    slope, icpt = np.polyfit(x, y, 1)
    print(json.dumps({"fixed_ms": round(float(icpt), 4), "ms_per_1k_keys": round(float(slope * 1024), 4),
                      "fixed_share_at_4096": round(float(icpt / (icpt + slope * 4096)), 3)}), flush=True)


if __name__ == "__main__":
    main()
