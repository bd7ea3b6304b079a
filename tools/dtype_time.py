import json, os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from tf_flash_attention_amd import flash_attention as fa
dev = torch.device("cuda:0")
def t(fn, n=5):
    for _ in range(2): fn()
    torch.cuda.synchronize()
    e=[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a,b in e: a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a,b in e]))
for dt, d, nq, b, pol in [(torch.float64, 64, 4096, 32, "full"), (torch.float64, 64, 4096, 32, "causal"), (torch.float64, 32, 4096, 64, "full"), (torch.float64, 128, 4096, 16, "full")]:
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda: (torch.rand((b, d, nq), generator=g, device=dev) * 4 - 2).to(dt)
    q, k, v, do = mk(), mk(), mk(), mk()
    ff = fa.estimate_forward_flops(pol, 1, q.shape, k.shape, v.shape, "none_front", 1, 0, False)
    o, l, m = fa.attention_forward(pol, 1, q, k, v, "none_front", 1, 0, False)
    tf_ = t(lambda: fa.attention_forward(pol, 1, q, k, v, "none_front", 1, 0, False))
    tb = t(lambda: fa.attention_backward(pol, 1, q, k, v, o, l, m, do, "none_front", 1, 0, False))
    print(json.dumps({"dtype": str(dt), "d": d, "policy": pol, "fwd_ms": round(tf_, 3), "fwd_tf": round(ff/tf_/1e9, 1), "bwd_ms": round(tb, 3), "bwd_tf": round(2.5*ff/tb/1e9, 1)}), flush=True)
