"""GPU tests that start fresh processes: the batch×head-sharded HIP path from two ranks, and the
native C-ABI harness (tools/fa_native_bench, the internal_test.cu equivalent).

Sharding: every (batch, head) slice is independent in forward and backward (the reference's
grid.y = b, flash_attention.cu:2172-2176), so each rank's slab of the outputs must be BITWISE
equal to the same slab of a single-process run — the kernels on these rules write every output
exactly once (no atomics), so the sum order cannot differ either."""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    # c4's shape family (local 1d band, d = 64) and c3's (causal, d = 128), scaled down
    "local64": dict(policy="local", seq_dims=1, sync="none_front", ws=48, ls=0, causal=False, batch=(3, 4), d=64,
                    nq=1024, nk=1024, dtype=np.float16),
    "causal128": dict(policy="causal", seq_dims=1, sync="none_front", ws=1, ls=0, causal=False, batch=(2, 3), d=128,
                      nq=640, nk=512, dtype=np.float16),
    "full2d_f32": dict(policy="full", seq_dims=2, sync="scale_front", ws=1, ls=0, causal=False, batch=(5,), d=64,
                       nq=(16, 16), nk=(32, 32), dtype=np.float32),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_two_process_shards_match_single_process(tmp_path, case):
    from tf_flash_attention_amd import flash_attention as fa
    c = CASES[case]
    rng = np.random.default_rng(11)
    qs = c["nq"] if isinstance(c["nq"], tuple) else (c["nq"],)
    ks = c["nk"] if isinstance(c["nk"], tuple) else (c["nk"],)
    Q = rng.uniform(-2, 2, c["batch"] + (c["d"],) + qs).astype(c["dtype"])
    K = rng.uniform(-2, 2, c["batch"] + (c["d"],) + ks).astype(c["dtype"])
    V = rng.uniform(-2, 2, c["batch"] + (c["d"],) + ks).astype(c["dtype"])
    dO = rng.uniform(-2, 2, Q.shape).astype(c["dtype"])
    np.savez(tmp_path / f"{case}_inputs.npz", Q=Q, K=K, V=V, dO=dO, policy=c["policy"], seq_dims=c["seq_dims"],
             sync=c["sync"], ws=c["ws"], ls=c["ls"], causal=c["causal"])
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(x).to(dev) for n, x in dict(Q=Q, K=K, V=V, dO=dO).items()}
    args = (c["sync"], c["ws"], c["ls"], c["causal"])
    O, l, m = fa.attention_forward(c["policy"], c["seq_dims"], t["Q"], t["K"], t["V"], *args)
    dQ, dK, dV = fa.attention_backward(c["policy"], c["seq_dims"], t["Q"], t["K"], t["V"], O, l, m, t["dO"], *args)
    b = int(np.prod(c["batch"]))
    full = {k: v.cpu().numpy().reshape((b,) + tuple(v.shape[len(c["batch"]):]))
            for k, v in dict(O=O, l=l, m=m, dQ=dQ, dK=dK, dV=dV).items()}

    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_shard_worker.py"),
                                       str(tmp_path), case], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out[-2000:]
    covered = []
    for r in range(world):
        f = np.load(tmp_path / f"{case}_rank{r}.npz")
        s0, s1 = int(f["start"]), int(f["stop"])
        covered += list(range(s0, s1))
        for k in ("O", "l", "m", "dQ", "dK", "dV"):
            got = f[k]
            np.testing.assert_array_equal(got.view(np.uint8), full[k][s0:s1].view(np.uint8), err_msg=f"{case} {k} r{r}")
    assert covered == list(range(b))


@pytest.mark.gpu
def test_native_harness_check():
    """tools/fa_native_bench check: the C ABI driven from C++ with no Python or framework, every
    policy × dtype against a double-precision CPU loop (internal_test.cu:249-317 equivalent)."""
    exe = os.path.join(ROOT, "tools", "fa_native_bench")
    if not os.path.exists(exe):
        pytest.fail("tools/fa_native_bench is not built (make -C tf_flash_attention_amd native)")
    r = subprocess.run([exe, "check"], capture_output=True, text=True, timeout=120)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert len(lines) >= 18
    assert all(x["ok"] for x in lines), [x for x in lines if not x["ok"]]
