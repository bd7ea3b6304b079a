"""Structured-input check of a forward variant of the diagnostic library against a torch float32 reference:
Q = 0 (uniform softmax) with V = 1, V[c][k] = c and V[c][k] = k / nk, then random inputs; prints the
error per channel quarter and per 32-query block, so a layout fault shows where it is.
Usage: python tools/debug_variant.py VARIANT [policy] [d] [nq] [nk]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FA_HIP_LIB", os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip_diag.so"))
os.environ["FA_FWD_VARIANT"] = sys.argv[1]
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402


def ref(q, k, v, causal):
    s = torch.einsum("bcq,bck->bqk", q.float(), k.float()) / q.shape[1] ** 0.5
    if causal:
        nq, nk = s.shape[1], s.shape[2]
        s = s.masked_fill(torch.arange(nk, device=s.device)[None, :] > torch.arange(nq, device=s.device)[:, None], -1e30)
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bqk,bck->bcq", p, v.float())


def main():
    policy = sys.argv[2] if len(sys.argv) > 2 else "full"
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    nq = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    nk = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    b = 2
    causal = policy == "causal"
    cases = {
        "Q=0,V=1": (torch.zeros(b, d, nq), torch.rand(b, d, nk) * 4 - 2, torch.ones(b, d, nk)),
        "Q=0,V=c": (torch.zeros(b, d, nq), torch.rand(b, d, nk) * 4 - 2,
                    (torch.arange(d).float() / d)[None, :, None].expand(b, d, nk).contiguous()),
        "Q=0,V=k": (torch.zeros(b, d, nq), torch.rand(b, d, nk) * 4 - 2,
                    (torch.arange(nk).float() / nk)[None, None, :].expand(b, d, nk).contiguous()),
        "random": (torch.rand(b, d, nq) * 4 - 2, torch.rand(b, d, nk) * 4 - 2, torch.rand(b, d, nk) * 4 - 2),
    }
    for name, (q, k, v) in cases.items():
        q, k, v = (x.half().to(dev) for x in (q, k, v))
        o, l, m = fa.attention_forward(policy, 1, q, k, v, "none_front", 1, 0, False)
        torch.cuda.synchronize()
        r = ref(q, k, v, causal)
        e = (o.float() - r).abs()
        print(f"{name}: max err {e.max().item():.3e}  (max|ref| {r.abs().max().item():.3f})")
        if e.max().item() > 1e-2:
            eq = e[0].reshape(d // 32, 32, nq // 32, 32).amax(dim=(1, 3))  # [channel quarter][query block]
            torch.set_printoptions(precision=2, linewidth=200)
            print("  error by channel quarter (rows) x 32-query block (cols):")
            print(eq.cpu())
            print("  o[0, 0, :8]", o[0, 0, :8].float().cpu(), " ref", r[0, 0, :8].cpu())
            print("  o[0, :8, 0]", o[0, :8, 0].float().cpu(), " ref", r[0, :8, 0].cpu())
            print("  l[0, :8]", l[0, :8].cpu(), " m[0, :8]", m[0, :8].float().cpu())


if __name__ == "__main__":
    main()
