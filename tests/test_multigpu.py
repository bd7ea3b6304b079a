"""Multi-GPU path on CPU: world_size-2 gloo processes.

The batch×head shards must tile the flattened batch exactly once and be
independent (each rank's oracle result on its slab equals the corresponding
slab of the single-process result), and the bench's barrier + max-over-ranks
timing reduction must work.  No data-path collective exists to test: there is
none by design (shard.py)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tf_flash_attention_amd import shard


def test_shard_ranges_tile_the_batch():
    for b in (1, 7, 8, 128, 1024, 1000):
        for world in (1, 2, 3, 4, 8):
            spans = [shard.shard_range(b, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == b
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            sizes = [s1 - s0 for s0, s1 in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(8, 2, 2)


def test_local_shard_is_a_view_of_the_batch_slab():
    x = torch.arange(2 * 3 * 4 * 5, dtype=torch.float32).reshape(2, 3, 4, 5)  # batch (2,3), C=4, N=5
    parts = [shard.local_shard(x, 1, 4, r) for r in range(4)]
    assert torch.equal(torch.cat(parts), x.reshape(6, 4, 5))
    assert parts[1].data_ptr() == x.reshape(6, 4, 5)[2].data_ptr()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import fa_oracle as O
        rng = np.random.default_rng(7)
        Q = rng.uniform(-2, 2, (2, 3, 8, 40)).astype(np.float32)   # b = 6 slices
        K = rng.uniform(-2, 2, (2, 3, 8, 24)).astype(np.float32)
        V = rng.uniform(-2, 2, (2, 3, 8, 24)).astype(np.float32)
        prob = O.Problem("causal", 1, "scale_end")
        ws, r, _ = shard.dist_env()
        qs, ks, vs = (shard.local_shard(torch.from_numpy(t), 1, ws, r).numpy() for t in (Q, K, V))
        o_local, _, _, _ = O.forward_f64(qs, ks, vs, prob)
        start, stop = shard.shard_range(6, ws, r)
        # control-plane only: barrier + max of per-rank "timings"
        dist.barrier()
        tmax = shard.max_over_ranks([1.0 + rank, 10.0 - rank])
        out[rank] = (start, stop, o_local, tmax)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_are_independent():
    from oracle import fa_oracle as O
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    rng = np.random.default_rng(7)
    Q = rng.uniform(-2, 2, (2, 3, 8, 40)).astype(np.float32)
    K = rng.uniform(-2, 2, (2, 3, 8, 24)).astype(np.float32)
    V = rng.uniform(-2, 2, (2, 3, 8, 24)).astype(np.float32)
    full, _, _, _ = O.forward_f64(Q.reshape(6, 8, 40), K.reshape(6, 8, 24), V.reshape(6, 8, 24),
                                  O.Problem("causal", 1, "scale_end"))
    covered = []
    for rank in range(world):
        start, stop, o_local, tmax = out[rank]
        np.testing.assert_array_equal(o_local, full[start:stop])
        covered += list(range(start, stop))
        assert tmax == [2.0, 10.0]
    assert covered == list(range(6))


def test_bench_batch_shard_split():
    """bench.py's default (--shard) splits every config's batch×head slices across the ranks, so
    a 1→8 scaling run measures the op's shard efficiency; --weak keeps the whole batch per rank."""
    import bench
    for name, cfg in bench.CONFIGS.items():
        b_total = int(np.prod(cfg[3]))
        for world in (1, 2, 4, 8):
            per = [bench.rank_batch(cfg, world, r) for r in range(world)]
            assert sum(b for b, _ in per) == b_total, name
            assert all(mode == "strong" for _, mode in per)
            assert max(b for b, _ in per) - min(b for b, _ in per) <= 1
            assert bench.rank_batch(cfg, world, 0, weak=True) == (b_total, "weak")
    assert bench.rank_batch(bench.CONFIGS["c2"], 2, 1) == (64, "strong")
    assert bench.rank_batch(bench.CONFIGS["c4"], 8, 7) == (128, "strong")
