"""Step and gap timeline of the one-wave D = 128 gap-stream forward (csrc/fa_fwd_f16_gap128.hip, variant 2700)
from the stamp build (tools/stamp/gap128_stamp.sh; outputs WRONG), at config 3's shape under the full policy
(every block the same 128 steps): per step of every wave of workgroups 0 and gridDim/2 the barrier wait,
segment A, block B's check (+ block A's mask), segment B and block A's check; and, for wave 0 of workgroup 0
at one step, the cycles of each pair of gaps (32 MFMAs a segment: 64 x 33.76 = 2160 cycles a step for the
MFMAs alone, MI355X_MICROARCH.md).
Usage: python tools/stamp/gap_stamps.py [gaps]   (gaps: the build with the per-gap stamps)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GAPS = len(sys.argv) > 1 and sys.argv[1] == "gaps"
os.environ["FA_HIP_LIB"] = os.path.join(ROOT, "tools", "stamp", "build_gap128",
                                        "libfa_hip_diag_gaps.so" if GAPS else "libfa_hip_diag.so")
os.environ["FA_FWD_VARIANT"] = "2700"
from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
import bench  # noqa: E402

NW, NSTEP, GAP_STEP = 4, 64, 20


def main():
    cfg = bench.CONFIGS["c3"]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = cfg
    policy = "full"
    dev = torch.device("cuda:0")
    b = int(np.prod(batch))
    q = (torch.rand((b, d) + qs, device=dev) * 4 - 2).to(dt)
    k = (torch.rand((b, d) + ks, device=dev) * 4 - 2).to(dt)
    v = (torch.rand((b, d) + ks, device=dev) * 4 - 2).to(dt)
    for _ in range(300):  # clock ramp (the stamps land in q's last slice: refreshed below)
        fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    q[-1].uniform_(-2, 2)
    fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)
    torch.cuda.synchronize()
    raw = q[-1].reshape(-1).view(torch.int64)[: 2 * NW * NSTEP * 6 + 32].cpu().numpy().astype(np.int64)
    t = raw[: 2 * NW * NSTEP * 6].reshape(2, NW, NSTEP, 6)
    names = ["barrier", "seg A", "check B", "seg B", "check A"]
    out = {"per_step_median_cycles": {}, "gap_step": GAP_STEP}
    for sel in range(2):
        for w in range(NW):
            ts = t[sel, w]
            parts = np.diff(ts, axis=1)  # (NSTEP, 5)
            step = np.diff(ts[:, 0])
            med = {n: float(np.median(parts[2:-2, i])) for i, n in enumerate(names)}
            med["step"] = float(np.median(step[2:-2]))
            out["per_step_median_cycles"][f"wg{sel}_w{w}"] = med
            print(f"wg {'0' if sel == 0 else 'mid'} wave {w}: " + "  ".join(f"{n} {v:.0f}" for n, v in med.items()))
    print(json.dumps(out))
    if not GAPS:
        return
    g = raw[2 * NW * NSTEP * 6:]
    s0 = t[0, 0, GAP_STEP]
    # gap pair j's cycles: from the previous stamp (pair 0 of A from the step's 'after barrier' stamp, pair 0
    # of B from 'after check B / mask A')
    prev = np.concatenate([[s0[1]], g[:15], [s0[3]], g[16:31]]) & 0xFFFFFFFF
    gc = ((g - prev) & 0xFFFFFFFF).tolist()  # (the gap stamps keep the counter's low 32 bits)
    out["gap_cycles"] = gc
    print(f"step {GAP_STEP}, wave 0 of workgroup 0, cycles per pair of gaps (segment A then B):")
    print("  A:", gc[:16], "sum", sum(gc[:16]))
    print("  B:", gc[16:], "sum", sum(gc[16:]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
