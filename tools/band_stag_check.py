"""Bitwise A/B of the persistent band forward (the default: staggered groups, split epilogue)
against a diagnostic variant (default: 2400, the unstaggered structure) over a set of 1d
local-window shapes the band kernel takes (diagnostic library).  A variant that keeps every wave's
tile sequence must give the same O, l, m bits.
Usage: python tools/band_stag_check.py [variant]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FA_HIP_LIB", os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip_diag.so"))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402

# (b, d, nq, nk, sync, ws, look_ahead)
SHAPES = [
    (4, 64, 4096, 4096, "none_front", 256, False),
    (3, 64, 2056, 2056, "none_front", 256, True),
    (2, 48, 1024, 1024, "none_front", 33, False),
    (2, 64, 1536, 3072, "scale_front", 70, False),
    (2, 64, 3072, 1536, "scale_end", 100, True),
    (5, 64, 800, 800, "scale_end", 511, False),
    (2, 64, 4096, 4096, "none_front", 600, False),
    (2, 64, 264, 264, "none_front", 16, False),
    (2, 64, 3000, 3000, "none_front", 300, False),
    (1, 64, 200, 200, "none_front", 50, True),
    (3, 40, 1024, 2048, "scale_front", 128, True),
    (64, 64, 16384, 16384, "none_front", 256, False),
]


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "2400"
    dev = torch.device("cuda:0")
    worst = 0.0
    for (b, d, nq, nk, sync, ws, la) in SHAPES:
        g = torch.Generator(device=dev).manual_seed(nq + ws)
        q = (torch.rand((b, d, nq), generator=g, device=dev) * 4 - 2).half()
        k = (torch.rand((b, d, nk), generator=g, device=dev) * 4 - 2).half()
        v = (torch.rand((b, 64, nk), generator=g, device=dev) * 4 - 2).half()
        res = []
        for x in ("-1", variant):
            os.environ["FA_FWD_VARIANT"] = x
            res.append(fa.attention_forward("local", 1, q, k, v, sync, ws, 0, la))
        torch.cuda.synchronize()
        diffs = [float((a.float() - c.float()).abs().max()) for a, c in zip(res[0], res[1])]
        same = all(torch.equal(a, c) for a, c in zip(res[0], res[1]))
        worst = max(worst, max(diffs))
        print(json.dumps({"shape": [b, d, nq, nk, sync, ws, la], "bitwise": same, "max_diff_olm": diffs}), flush=True)
    print(json.dumps({"variant": variant, "worst": worst}))


if __name__ == "__main__":
    main()
