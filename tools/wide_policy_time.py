"""Forward TF/s (algorithmic, allowed pairs) of the full and causal policies at equal shapes, one process:
d = 256 (§3.0d wide kernel) at N = 4096 / 8192 and d = 128 (§3.0b ping-pong) at N = 8192, b = 128;
with the argument `bwd`, the d = 128 backward (§3.2) at N = 8192 instead."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402


def run_bwd(b, d, n, policy, reps=5):
    """backward (dQ, dK, dV) rate: 2.5x the forward's algorithmic FLOPs"""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2)
    q, k, v, do = ((torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half() for _ in range(4))
    fl = 2.5 * fa.estimate_forward_flops(policy, 1, q.shape, k.shape, v.shape, "none_front", 1, 0, False)
    o, l, m = fa.attention_forward(policy, 1, q, k, v, "none_front")
    for _ in range(2):
        fa.attention_backward(policy, 1, q, k, v, o, l, m, do, "none_front")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fa.attention_backward(policy, 1, q, k, v, o, l, m, do, "none_front")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"bwd b={b} d={d} n={n} {policy:6s} {ms:8.3f} ms {fl / ms / 1e9:8.1f} TF/s", flush=True)


def run(b, d, n, policy, causal=False, reps=10):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    q, k, v = ((torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half() for _ in range(3))
    fl = fa.estimate_forward_flops(policy, 1, q.shape, k.shape, v.shape, "none_front", 1, 0, causal)
    for _ in range(3):
        fa.attention_forward(policy, 1, q, k, v, "none_front", 1, 0, causal)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fa.attention_forward(policy, 1, q, k, v, "none_front", 1, 0, causal)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"b={b} d={d} n={n} {policy:6s} {ms:8.3f} ms {fl / ms / 1e9:8.1f} TF/s", flush=True)


if len(sys.argv) == 1:
    for n in (4096, 8192):
        for pol in ("full", "causal"):
            run(128, 256, n, pol)
    for pol in ("full", "causal"):
        run(128, 128, 8192, pol)
if len(sys.argv) > 1 and sys.argv[1] == "bwd":
    for pol in ("full", "causal"):
        run_bwd(128, 128, 8192, pol)
