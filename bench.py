#!/usr/bin/env python3
"""Benchmark of the fused flash-attention hot path on MI355X.

Default (the driver's contract): BASELINE.json config 2 — full_1d fp16,
B=8 H=16 d=64 Nq=Nk=4096, forward — metric "fwd TFLOP/s per GPU + MFMA util %".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--shard|--weak]
                  [--no-cpu-baseline]

For N>1: one process per GPU, each rank runs its own shard of batch×head
slices (no data-path collective; a gloo barrier / max-reduce over CPU tensors
only brackets the timed region).  Under torch.distributed.run the ranks come
from the environment; without it (WORLD_SIZE unset) `--gpus N` starts N fresh
child processes itself, before anything touches the GPU, and exits with the
worst child's status.
Default (--shard): the config's batch×head slices are split across the ranks
(strong scaling: c2 b=128 is 64 slices a rank at N=2, 16 at N=8), so a 1→8
curve measures the op's batch-shard efficiency (BASELINE north_star: "near-linear
batch-shard scaling").  --weak: every rank runs the whole config batch (the
round-1..3 behaviour for c2/c3/c5).

A step = one pass of the op over the rank's batch with inputs resident in HBM
(c3: forward + backward).  Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tf_flash_attention_amd import flash_attention as fa  # noqa: E402  (the HIP library loads lazily)
from tf_flash_attention_amd import shard  # noqa: E402

MFMA_PEAK = {"fp16": 2516.6, "fp32": 157.3, "fp64": 78.6}   # dense TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (policy, seq_dims, dtype, batch, d, q_seq, k_seq, sync, ws, ls, causal, backward, -)
    "c2": ("full", 1, torch.float16, (8, 16), 64, (4096,), (4096,), "none_front", 1, 0, False, False, "weak"),
    "c3": ("causal", 1, torch.float16, (8, 16), 128, (8192,), (8192,), "none_front", 1, 0, False, True, "weak"),
    "c4": ("local", 1, torch.float16, (64, 16), 64, (16384,), (16384,), "none_front", 256, 0, False, False, "strong"),
    "c5": ("full", 2, torch.float32, (4, 8), 64, (64, 64), (128, 128), "scale_front", 1, 0, False, False, "weak"),
    # not a BASELINE config: config 2's shape at d = 32, inside the reference's own test channel range
    # (tests/test_1d.py:57-66 draws C in [8, 32]); profiled to price the d <= 32 forward
    "d32": ("full", 1, torch.float16, (8, 16), 32, (4096,), (4096,), "none_front", 1, 0, False, False, "weak"),
    # not a BASELINE config: config 2's shape at d = 256, past the d <= 128 kernels (fa_fwd_f16_wide.hip)
    "w256": ("full", 1, torch.float16, (8, 16), 256, (4096,), (4096,), "none_front", 1, 0, False, False, "weak"),
    "w256b": ("causal", 1, torch.float16, (8, 16), 256, (8192,), (8192,), "none_front", 1, 0, False, True, "weak"),
}
WORKLOAD = {
    "c2": "full_1d fp16 B=8 H=16 d=64 Nq=Nk=4096 forward (BASELINE config 2)",
    "c3": "causal_1d fp16 B=8 H=16 d=128 N=8192 forward+backward (BASELINE config 3)",
    "c4": "local_1d fp16 window=256 B=64 H=16 d=64 N=16384 forward (BASELINE config 4)",
    "c5": "full_2d fp32 B=4 H=8 d=64 (64,64)x(128,128) scale_front forward (BASELINE config 5)",
    "d32": "full_1d fp16 B=8 H=16 d=32 Nq=Nk=4096 forward (config 2 at the reference tests' d=32; diagnostic)",
    "w256": "full_1d fp16 B=8 H=16 d=256 Nq=Nk=4096 forward (config 2 at d=256, past 128 channels; diagnostic)",
    "w256b": "causal_1d fp16 B=8 H=16 d=256 N=8192 forward+backward (config 3 at d=256; diagnostic)",
}
DTYPE_NAME = {torch.float16: "fp16", torch.float32: "fp32", torch.float64: "fp64"}


def rank_batch(cfg, world: int, rank: int, weak: bool = False):
    """(slices this rank runs, "strong"|"weak"): by default the config's flattened batch split into
    contiguous slabs (shard.shard_range); with ``weak`` every rank runs all of it."""
    b_total = int(np.prod(cfg[3]))
    if weak:
        return b_total, "weak"
    s0, s1 = shard.shard_range(b_total, world, rank)
    return s1 - s0, "strong"


def _call_forward(cfg, q, k, v):
    policy, seq_dims, _, _, _, _, _, sync, ws, ls, causal, _, _ = cfg
    return fa.attention_forward(policy, seq_dims, q, k, v, sync, ws, ls, causal)


def _call_backward(cfg, q, k, v, o, l, m, do):
    policy, seq_dims, _, _, _, _, _, sync, ws, ls, causal, _, _ = cfg
    return fa.attention_backward(policy, seq_dims, q, k, v, o, l, m, do, sync, ws, ls, causal)


def usable_cpus() -> tuple:
    """(cpus this process may run on, why): the affinity mask, capped by a cgroup CPU quota when
    one is set (a GPU box grants each GPU a share of a larger host; os.cpu_count() is the host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = "affinity mask"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            if q < n:
                n, why = q, f"cgroup cpu.max quota ({quota}/{period})"
    except (OSError, ValueError):
        pass
    return n, why


def cpu_baseline(cfg, budget_s: float):
    """The reference's naive (TF) CPU attention, restated in numpy fp32
    (oracle.naive_attention_slice_f32, tests/test_1d.py:69-76; for a forward+backward config also
    oracle.naive_attention_backward_slice_f32, the autodiff of that graph), timed on a bounded
    sample of (b,h) slices of the same workload on every CPU this process may use; fp16 inputs
    upcast to fp32."""
    from oracle import fa_oracle as O
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = cfg
    ncpu, why = usable_cpus()
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        limiter = threadpool_limits(limits=ncpu)
    except Exception:  # pragma: no cover
        threadpool_info, limiter = None, None
    rng = np.random.default_rng(0)
    nq, nk = int(np.prod(qs)), int(np.prod(ks))
    prob = O.Problem(policy, seq_dims, sync, ws, ls, causal)
    mask = None
    if policy != "full":
        mask = O.problem_mask(prob, list(qs), list(ks))
    pairs = nq * nk if mask is None else int(mask.sum())
    flops_slice = 2.0 * (d + d) * pairs + (2.0 * (3 * d + 2 * d) * pairs if bwd else 0.0)
    q = rng.uniform(-2, 2, (d, nq)).astype(np.float32)
    k = rng.uniform(-2, 2, (d, nk)).astype(np.float32)
    v = rng.uniform(-2, 2, (d, nk)).astype(np.float32)
    do = rng.uniform(-2, 2, (d, nq)).astype(np.float32) if bwd else None
    O.naive_attention_slice_f32(q[:, :64], k[:, :64], v[:, :64])  # warm BLAS threads
    cores = ncpu
    if threadpool_info is not None:
        used = [p.get("num_threads", 1) for p in threadpool_info() if p.get("user_api") == "blas"]
        cores = max(used or [ncpu])
    n, t0 = 0, time.perf_counter()
    while True:
        O.naive_attention_slice_f32(q, k, v, mask)
        if bwd:
            O.naive_attention_backward_slice_f32(q, k, v, do, mask)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= int(np.prod(batch)):
            break
    if limiter is not None:
        limiter.restore_original_limits()
    tflops = flops_slice * n / el / 1e12
    what = "forward + backward" if bwd else "forward"
    return {"value": tflops, "unit": "TFLOP/s", "cores": int(cores), "kind": "port",
            "host_cpus": os.cpu_count(), "usable_cpus": ncpu, "usable_cpus_from": why, "cpu_model": _cpu_model(),
            "sample": f"{n} of {int(np.prod(batch))} (b,h) slices of the workload, {what}, numpy fp32 naive attention "
                      f"(einsum->softmax->einsum, tests/test_1d.py:69-76; backward = its autodiff) on "
                      f"{cores} BLAS threads, {el:.1f}s; fp16 inputs upcast"}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def spawn_ranks(n: int, argv) -> int:
    """Start `n` fresh bench processes (RANK/WORLD_SIZE/LOCAL_RANK set, gloo rendezvous on
    127.0.0.1) and wait for them.  Called only from a parent that has not touched the GPU:
    the children initialise HIP themselves (rank r on GPU r % device_count).  Returns the
    worst exit status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    # poll: the first rank that fails ends the others (they would otherwise wait in the gloo
    # rendezvous or barrier for its 30-minute timeout), and its status is returned
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.05)


def algorithmic_bytes(cfg, b):
    """(read, write) HBM bytes one step must move.  Forward: Q,K,V in;
    O, l, m out.  Backward adds Q,K,V,O,dO,l,m in; dQ,dK,dV out."""
    policy, seq_dims, dt, batch, d, qs, ks, *_ = cfg
    bwd = cfg[11]
    nq, nk = int(np.prod(qs)), int(np.prod(ks))
    t = torch.tensor([], dtype=dt).element_size()
    lt = 4 if t == 2 else t
    rd, wr = b * (nq * d + 2 * nk * d) * t, b * (nq * d * t + nq * (lt + t))
    if bwd:
        rd += b * ((3 * nq * d + 2 * nk * d) * t + nq * (lt + t))
        wr += b * (nq * d + 2 * nk * d) * t
    return rd, wr


def load_traffic(workload_key: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/traffic_<key>.json),
    written by tools/pmc_traffic.py; None if absent."""
    path = os.path.join(ROOT, "profiles", f"traffic_{workload_key}.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get("hbm_bytes_per_launch"), t.get("algorithmic_read_bytes", 0) + t.get("algorithmic_write_bytes", 0)
    except Exception:
        return None, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=40)
    # the chip's clock ramps for the first ~0.5 s of back-to-back launches on a fresh box (c2 at
    # --warmup 5 ran 0.64 ms/step against 0.57 after the ramp): untimed warm-up continues past the
    # W steps until this much wall time has gone by; the line reports both
    ap.add_argument("--warmup-s", type=float, default=1.0)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--shard", dest="weak", action="store_false", default=False,
                    help="split the config's batch across ranks (strong scaling; the default)")
    ap.add_argument("--weak", dest="weak", action="store_true",
                    help="every rank runs the whole config batch (weak scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = shard.dist_env()
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo's rendezvous prints "[Gloo] Rank r is connected to ..." on the process's stdout, where
        # the driver reads the one JSON line: keep file descriptor 1 on /dev/null while it connects
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            import datetime
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=5))
        finally:
            os.dup2(saved, 1)
            os.close(devnull)
            os.close(saved)
    # one process per GPU; modulo only matters when rehearsing N ranks on fewer GPUs
    ndev = max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)

    cfg = CONFIGS[args.config]
    policy, seq_dims, dt, batch, d, qs, ks, sync, ws, ls, causal, bwd, _ = cfg
    # the config's slices split across ranks (contiguous slabs, no collective), or all of them
    b_rank, scaling = rank_batch(cfg, world, rank, args.weak)
    shape_q = (b_rank, d) + qs
    shape_k = (b_rank, d) + ks
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    # U(-2,2) synthetic inputs generated on device (tests/test_base.py:170-173 distribution)
    q = (torch.rand(shape_q, generator=g, device=dev, dtype=torch.float32) * 4 - 2).to(dt)
    k = (torch.rand(shape_k, generator=g, device=dev, dtype=torch.float32) * 4 - 2).to(dt)
    v = (torch.rand(shape_k, generator=g, device=dev, dtype=torch.float32) * 4 - 2).to(dt)
    do = (torch.rand(shape_q, generator=g, device=dev, dtype=torch.float32) * 4 - 2).to(dt) if bwd else None

    fwd_flops_rank = fa.estimate_forward_flops(policy, seq_dims, shape_q, shape_k, shape_k, sync, ws, ls, causal)
    pairs_rank = fwd_flops_rank / (2.0 * (d + d))
    bwd_flops_rank = 2.0 * (3 * d + 2 * d) * pairs_rank if bwd else 0.0
    step_flops_rank = fwd_flops_rank + bwd_flops_rank

    o = l = m = None

    def step():
        nonlocal o, l, m
        o, l, m = _call_forward(cfg, q, k, v)
        if bwd:
            _call_backward(cfg, q, k, v, o, l, m, do)

    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    extra = 0
    while time.perf_counter() - tw < args.warmup_s:
        for _ in range(8):
            step()
        extra += 8
        torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw

    # HIP events on the launch stream bracket the timed region (one pair: an event pair around every
    # step added ~8 us of gap a step on c2, 1.6 % of its step); their span / K is the average launch
    # duration the roofline divides by, and agrees with the rocprofv3 kernel average (profiles/)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    if dist:
        elapsed, kern_ms = shard.max_over_ranks([elapsed, kern_ms])
        total_flops = shard.sum_over_ranks([step_flops_rank])[0] * args.steps
    else:
        total_flops = step_flops_rank * args.steps
    value = total_flops / elapsed / 1e12
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        dname = DTYPE_NAME[dt]
        peak = MFMA_PEAK[dname]
        achieved = step_flops_rank / (kern_ms * 1e-3) / 1e12  # one rank's launches / event-timed duration
        traffic, traffic_alg = load_traffic(args.config)
        rd, wr = algorithmic_bytes(cfg, b_rank)
        alg_bytes = rd + wr
        if traffic is not None and traffic_alg and traffic_alg != alg_bytes:
            traffic = traffic * alg_bytes / traffic_alg  # profiled at another batch: per-slice scaling
        # the binding roof: time at MFMA peak vs time at HBM peak for the algorithmic work
        hbm_bound = alg_bytes / (HBM_PEAK_GBS * 1e9) > step_flops_rank / (peak * 1e12)
        if hbm_bound:
            roof = {"bound": "hbm", "achieved": round(alg_bytes / (kern_ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s"}
        else:
            roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof.update({"traffic": traffic,
                     "traffic_source": f"profiles/traffic_{args.config}.json (rocprofv3 PMC FETCH_SIZE + WRITE_SIZE "
                                       "of this kernel, committed from a separate profiling run; not measured here)"
                     if traffic is not None else None,
                     "algorithmic_flops_per_launch": step_flops_rank,
                     "algorithmic_bytes_per_launch": alg_bytes, "event_ms_per_launch": round(kern_ms, 4)})
        line = {
            "metric": "fwd TFLOP/s per GPU + MFMA util %, fp16 full_1d d=64 seq=4096" if args.config == "c2"
            else f"TFLOP/s ({args.config})",
            "value": round(value, 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_extra_steps": extra,
            "warmup_s": round(warm_s, 3),
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": dname,
            "data": "synthetic U(-2,2), generated on device",
            "config": {"workload": WORKLOAD[args.config], "b_total": int(np.prod(batch)) * (world if args.weak else 1),
                       "b_per_rank": b_rank, "d": d, "q_seq": list(qs),
                       "k_seq": list(ks), "policy": policy, "sync_mode": sync,
                       "parallelism": f"batch-shard x{world} (no collective)"},
            "per_gpu_tflops": round(value / world, 3),
            "mfma_util_pct": round(100.0 * achieved / peak, 2),
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
