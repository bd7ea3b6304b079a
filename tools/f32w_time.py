"""fp32 backward time at 256 channels (fa_bwd_f32_wide.hip): b = 32, d = 256, N = 4096, full.
Usage: python tools/f32w_time.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
from wide_time import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, d, n = 32, 256, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v, do = ((torch.rand((b, d, n), generator=g, device=dev) * 4 - 2) for _ in range(4))
    o, l, m = fa.attention_forward("full", 1, q, k, v, "none_front", 1, 0, False)
    t = timed(lambda: fa.attention_backward("full", 1, q, k, v, o, l, m, do, "none_front"))
    flops = 2.5 * 2.0 * (d + d) * n * n * b
    print(json.dumps({"shape": f"full_1d fp32 b={b} d={d} n={n}", "pass": "backward", "ms": round(t, 4),
                      "tflops": round(flops / t / 1e9, 1), "fp32_mfma_peak_frac": round(flops / t / 1e9 / 157.3, 3)}))


if __name__ == "__main__":
    main()
