"""Run fp16 forward + backward over shapes outside the interval-rule / aligned envelope (strided and
2d local windows, lengths not divisible by 8, misaligned pointers, d <= 32), so a rocprofv3 kernel
trace shows which kernels serve them:

  rocprofv3 --kernel-trace --stats -d gpurun_out/disp -o run -- python3 tools/dispatch_trace.py

The two-pass backward (bwd_dkdv_kernel / bwd_dq_kernel) should be the only backward kernels in the
trace: no bwd_f16_kernel (single-pass, atomics) and no bwd_generic_kernel.

With the argument f64 it runs fp64 forward + backward at 128 < D <= 256 over every rule class instead
(the trace should show fwd_f64_kernel / bwd_dkdv_f64_kernel / bwd_dq_f64_kernel and no *_generic_*).
With f16w: fp16 at 128 < D <= 256 in the shapes past the 16-B chunk staging and the interval rules
(odd lengths, a misaligned pointer, strided 1d and 2d local windows): fwd_f16_wide_kernel and the
four-role bwd_dkdv_w4_kernel / bwd_dq_w4_kernel only, no *_generic_*.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402

SHAPES = [
    # policy, seq_dims, d, qs, ks, ws, ls, causal, misalign
    ("local", 1, 64, (520,), (520,), 20, 2, False, False),
    ("local", 2, 128, (24, 20), (24, 20), 5, 0, False, False),
    ("local", 2, 64, (16, 24), (20, 12), 3, 1, True, False),
    ("full", 1, 64, (263,), (517,), 1, 0, False, False),
    ("causal", 1, 128, (333,), (199,), 1, 0, False, False),
    ("full", 1, 64, (256,), (192,), 1, 0, False, True),
    ("causal", 1, 16, (200,), (200,), 1, 0, False, False),
]


SHAPES_F64 = [
    ("full", 1, 256, (131,), (197,), 1, 0, False, False),
    ("causal", 1, 256, (150,), (150,), 1, 0, False, False),
    ("local", 1, 200, (120,), (241,), 40, 0, True, False),
    ("local", 2, 256, (9, 14), (9, 14), 4, 2, True, False),
]


SHAPES_F16W = [
    ("full", 1, 256, (131,), (197,), 1, 0, False, False),
    ("causal", 1, 160, (150,), (75,), 1, 0, False, False),
    ("causal", 1, 256, (264,), (264,), 1, 0, False, True),
    ("local", 1, 256, (150,), (150,), 20, 3, False, False),
    ("local", 2, 200, (9, 14), (9, 14), 4, 2, True, False),
    ("local", 2, 256, (16, 24), (16, 24), 5, 0, False, False),
]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    dt = torch.float64 if mode == "f64" else torch.float16
    shapes = {"f64": SHAPES_F64, "f16w": SHAPES_F16W}.get(mode, SHAPES)
    for policy, sd, d, qs, ks, ws, ls, causal, mis in shapes:
        def mk(shape):
            n = 1
            for x in shape:
                n *= x
            buf = (torch.rand(n + 1, generator=g, device=dev, dtype=torch.float64) * 4 - 2).to(dt)
            t = (buf[1:] if mis else buf[:n]).view(shape)
            return t.requires_grad_(True)
        q, k, v = mk((2, d) + qs), mk((2, d) + ks), mk((2, d) + ks)
        o, l, m = fa.attention_forward(policy, sd, q, k, v, "none_front", ws, ls, causal)
        fa.attention_backward(policy, sd, q, k, v, o, l, m, torch.ones_like(o), "none_front", ws, ls, causal)
    torch.cuda.synchronize()
    print("dispatch trace shapes done")


if __name__ == "__main__":
    main()
