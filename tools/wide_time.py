"""Forward and backward time at 256 channels, plus the fp32 forward there (config 2's shape at d = 256): the MFMA kernels
(fa_fwd_f16_wide.hip; fa_bwd_f16_fast.hip launch_bwd_wide) against the SIMT kernels the same calls took
before round 4 (reached here through a K pointer one element off 16-B alignment, which the MFMA kernels
do not take).  Usage: python tools/wide_time.py [b] [n]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2]


def main():
    dev = torch.device("cuda:0")
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    d = 256
    g = torch.Generator(device=dev).manual_seed(0)
    q = (torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half()
    k = (torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half()
    v = (torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half()
    kb = torch.empty(k.numel() + 1, dtype=k.dtype, device=dev)
    kb[1:].copy_(k.reshape(-1))
    km = kb[1:].view(k.shape)
    flops = 2.0 * (d + d) * n * n * b
    t_mfma = timed(lambda: fa.attention_forward("full", 1, q, k, v, "none_front", 1, 0, False))
    o1, _, _ = fa.attention_forward("full", 1, q, k, v, "none_front", 1, 0, False)
    t_simt = timed(lambda: fa.attention_forward("full", 1, q, km, v, "none_front", 1, 0, False), n=3)
    o2, _, _ = fa.attention_forward("full", 1, q, km, v, "none_front", 1, 0, False)
    print(json.dumps({"shape": f"full_1d fp16 b={b} d={d} n={n}", "pass": "forward", "mfma_ms": round(t_mfma, 4),
                      "mfma_tflops": round(flops / t_mfma / 1e9, 1), "simt_ms": round(t_simt, 4),
                      "simt_tflops": round(flops / t_simt / 1e9, 1),
                      "max_abs_diff": float((o1.float() - o2.float()).abs().max())}), flush=True)
    # backward: dK / dV pass (4 matmuls) + dQ pass (3 matmuls: Sᵀ, dPᵀ recomputed, dQ) = 2.5x the forward
    o1, l1, m1 = fa.attention_forward("full", 1, q, k, v, "none_front", 1, 0, False)
    do = (torch.rand((b, d, n), generator=g, device=dev) * 4 - 2).half()
    bflops = 2.5 * flops
    t_bm = timed(lambda: fa.attention_backward("full", 1, q, k, v, o1, l1, m1, do, "none_front"))
    g1 = fa.attention_backward("full", 1, q, k, v, o1, l1, m1, do, "none_front")
    t_bs = timed(lambda: fa.attention_backward("full", 1, q, km, v, o1, l1, m1, do, "none_front"), n=3)
    g2 = fa.attention_backward("full", 1, q, km, v, o1, l1, m1, do, "none_front")
    diff = max(float((x.float() - y.float()).abs().max() / y.float().abs().max()) for x, y in zip(g1, g2))
    print(json.dumps({"shape": f"full_1d fp16 b={b} d={d} n={n}", "pass": "backward", "mfma_ms": round(t_bm, 4),
                      "mfma_tflops": round(bflops / t_bm / 1e9, 1), "simt_ms": round(t_bs, 4),
                      "simt_tflops": round(bflops / t_bs / 1e9, 1), "max_rel_diff": diff}), flush=True)
    # fp32 forward on the MFMA kernel (fa_fwd_f32_wide.hip), a quarter of the batch
    b32 = max(b // 4, 1)
    q32, k32, v32 = (x[:b32].float() for x in (q, k, v))
    t32 = timed(lambda: fa.attention_forward("full", 1, q32, k32, v32, "none_front", 1, 0, False))
    f32 = flops * b32 / b
    print(json.dumps({"shape": f"full_1d fp32 b={b32} d={d} n={n}", "pass": "forward", "mfma_ms": round(t32, 4),
                      "mfma_tflops": round(f32 / t32 / 1e9, 1), "fp32_mfma_peak_frac": round(f32 / t32 / 1e9 / 157.3, 3)}),
          flush=True)
    # fp32 backward (fa_bwd_f32_wide.hip)
    o32, l32, m32 = fa.attention_forward("full", 1, q32, k32, v32, "none_front", 1, 0, False)
    do32 = do[:b32].float()
    tb32 = timed(lambda: fa.attention_backward("full", 1, q32, k32, v32, o32, l32, m32, do32, "none_front"))
    print(json.dumps({"shape": f"full_1d fp32 b={b32} d={d} n={n}", "pass": "backward", "mfma_ms": round(tb32, 4),
                      "mfma_tflops": round(2.5 * f32 / tb32 / 1e9, 1),
                      "fp32_mfma_peak_frac": round(2.5 * f32 / tb32 / 1e9 / 157.3, 3)}), flush=True)


if __name__ == "__main__":
    main()
