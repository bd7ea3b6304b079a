"""Forward error of diagnostic-library variants against the float64 oracle on sampled slices of a
bench config (the same seeded U(-2,2) inputs for every variant).  Prints, per variant, the max
|O - O64| / max(max|O64|, 1) (the parity tests' scaled error), the max |m - m64| and the max
relative l error.  Usage: python tools/variant_parity.py [config] v1 v2 ..."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FA_HIP_LIB", os.path.join(ROOT, "tf_flash_attention_amd", "libfa_hip_diag.so"))
from oracle import fa_oracle as O  # noqa: E402
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    cfgname = args.pop(0) if args and args[0] in bench.CONFIGS else "c2"
    variants = args or ["-1"]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = bench.CONFIGS[cfgname]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(4321)
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, generator=g, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, generator=g, device=dev) * 4 - 2).to(dt)
    sl = sorted({0, b // 2, b - 1})
    prob = O.Problem(policy, seq_dims, sync, ws, ls, causal)
    host = [t[sl].cpu().numpy() for t in (q, k, v)]
    O64, L64, M64, ha = O.forward_f64(*host, prob)
    O64 = O64.reshape(len(sl), d, -1)
    L64 = L64.reshape(len(sl), -1)
    M64 = M64.reshape(len(sl), -1)
    for vv in variants:
        os.environ["FA_FWD_VARIANT"] = vv
        o, l, m = fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
        torch.cuda.synchronize()
        og = o[sl].reshape(len(sl), d, -1).double().cpu().numpy()
        lg = l[sl].reshape(len(sl), -1).double().cpu().numpy()
        mg = m[sl].reshape(len(sl), -1).double().cpu().numpy()
        e_o = float(np.max(np.abs(og - O64)) / max(np.max(np.abs(O64)), 1.0))
        e_m = float(np.max(np.abs(mg - M64)[:, ha]))
        l_ref = L64 * np.exp(M64 - mg)
        e_l = float(np.max((np.abs(lg - l_ref) / np.maximum(l_ref, 1e-30))[:, ha]))
        print(json.dumps({"config": cfgname, "variant": vv, "slices": sl, "o_err_scaled": e_o, "m_abs_err": e_m,
                          "l_rel_err": e_l}), flush=True)


if __name__ == "__main__":
    main()
