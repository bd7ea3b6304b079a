"""Worker for tests/test_gpu_multiproc.py: one rank of a batch×head-sharded run of the HIP path.

Started as a fresh process (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* in the environment, as
bench.py's own spawner and torch.distributed.run set them).  It joins a gloo group (control
plane only), takes its contiguous slab of the flattened batch with shard.local_shard (a view:
pointer offset, no copy), runs the op's forward and backward on GPU local_rank % device_count,
and writes its slab of O, l, m, dQ, dK, dV to <outdir>/rank<r>.npz.  No data-path collective."""

import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tf_flash_attention_amd import flash_attention as fa  # noqa: E402
from tf_flash_attention_amd import shard  # noqa: E402


def main(indir: str, case: str):
    world, rank, local = shard.dist_env()
    dist.init_process_group("gloo")
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    f = np.load(os.path.join(indir, f"{case}_inputs.npz"))
    policy, seq_dims, sync, ws, ls, causal = (str(f["policy"]), int(f["seq_dims"]), str(f["sync"]), int(f["ws"]),
                                              int(f["ls"]), bool(f["causal"]))
    t = {n: shard.local_shard(torch.from_numpy(f[n]).to(dev), seq_dims, world, rank) for n in ("Q", "K", "V", "dO")}
    O, l, m = fa.attention_forward(policy, seq_dims, t["Q"], t["K"], t["V"], sync, ws, ls, causal)
    dQ, dK, dV = fa.attention_backward(policy, seq_dims, t["Q"], t["K"], t["V"], O, l, m, t["dO"], sync, ws, ls,
                                       causal)
    torch.cuda.synchronize()
    start, stop = shard.shard_range(int(np.prod(f["Q"].shape[:f["Q"].ndim - seq_dims - 1])), world, rank)
    np.savez(os.path.join(indir, f"{case}_rank{rank}.npz"), start=start, stop=stop,
             **{k: v.cpu().numpy() for k, v in dict(O=O, l=l, m=m, dQ=dQ, dK=dK, dV=dV).items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
