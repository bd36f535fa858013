"""Multi-GPU layout of the transport path: one process per GPU, sharded by session.

Packets are independent given (key, counter), and a session's keys and
counters never leave its owner, so the batch shards with no data-path collective:
session s belongs to rank s mod world (the reference's sessions are likewise disjoint,
EstablishedSession.java:59-71). The only collectives are the benchmark's timing
barrier and the max/sum reductions of its report — on RCCL ("nccl") on the GPU box and
on gloo in the CPU tests.
"""
from __future__ import annotations

import numpy as np


def session_shard(n_sessions: int, rank: int, world: int) -> np.ndarray:
    """Sessions owned by `rank`: s with s mod world == rank."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return np.arange(rank, n_sessions, world, dtype=np.int64)


def shard_packets(total: int, n_sessions: int, rank: int, world: int):
    """Per-rank packet columns for `total` packets spread evenly over `n_sessions`:
    (local key slot, global session id, per-session counter) per packet. Each session
    counts its packets from 0, as SymmetricKeypair issues counters (SymmetricKeypair.java:64)."""
    mine = session_shard(n_sessions, rank, world)
    per = total // n_sessions
    slots = np.repeat(np.arange(len(mine), dtype=np.int64), per)
    sessions = np.repeat(mine, per)
    counters = np.tile(np.arange(per, dtype=np.uint64), len(mine))
    return slots, sessions, counters


def reduce_report(dist, device, timings, payload: float, ok: bool):
    """Max of each timing and sum of the payload / failures over the ranks (world > 1).
    Returns (timings_max, payload_sum, all_ok)."""
    import torch
    t = torch.tensor(list(timings), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    p = torch.tensor([payload, 0.0 if ok else 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(p)
    return t.tolist(), p[0].item(), p[1].item() == 0.0


PER_GPU_KEYS = ("elapsed_s", "payload_bytes", "packets", "seal_ms", "open_ms", "kernel_ms")


def gather_per_rank(dist, device, row: dict):
    """Every rank's own figures (PER_GPU_KEYS) gathered to all ranks, in rank order, so the
    report shows each GPU's rate next to the aggregate (BASELINE configs[3]: per-GPU and
    aggregate GiB/s; a straggler shows as one low entry). GiB/s per rank = its payload over
    its own elapsed time."""
    import torch
    mine = torch.tensor([float(row[k]) for k in PER_GPU_KEYS], dtype=torch.float64, device=device)
    world = dist.get_world_size() if dist is not None else 1
    if world > 1:
        out = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(out, mine)
    else:
        out = [mine]
    rows = []
    for r, t in enumerate(out):
        d = dict(zip(PER_GPU_KEYS, t.tolist()))
        d["packets"] = int(d["packets"])
        d["payload_bytes"] = int(d["payload_bytes"])
        d["rank"] = r
        d["gib_s"] = d["payload_bytes"] / d["elapsed_s"] / float(1 << 30) if d["elapsed_s"] > 0 else 0.0
        rows.append(d)
    return rows
