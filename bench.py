#!/usr/bin/env python3
"""bench.py — device-resident transport AEAD throughput on MI355X.

Metric (BASELINE.json): device-resident AEAD GiB/s, 64K x 1420B seal+open.
One step = seal a batch of synthetic packets (plaintext -> ct||tag) and open the
result (ct||tag -> plaintext), both on the GPU with inputs resident in HBM.
value = payload bytes sealed + opened by all ranks / max-over-ranks time / 2^30.

Workloads (--workload):
  c1 (default)  65536 x 1420 B per GPU, one session key, counters 0..65535
                (BASELINE configs[1]; weak scaling: each rank owns its own sessions)
  c2            65536 packets per GPU, lengths uniform in [64, 9000], 256 session keys
  c3            8,388,608 x 1420 B in total, sharded by session over the ranks (strong)

Multi-GPU: one process per GPU (torchrun); packets are independent, so each rank
works on its own shard — no collective on the data path. The only collectives
are the timing barrier and the max-over-ranks reduction.

The JSON line also carries:
  roofline      the seal kernel (k_stream<SEAL>) against the 8 TB/s HBM peak, with
                algorithmic bytes = n * (2L + 16) per launch and the launch duration
                from HIP events on the launch stream; `traffic` from the committed
                rocprofv3 PMC summary (profiles/pmc_*.json) when present
  cpu_baseline  the CPU restatement (oracle/liboracle.so, bit-exact to the
                reference) timed on this host's cores, rank 0, N = 1 only
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident AEAD GiB/s, 64K x 1420B seal+open, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)


def splitmix_np(seed: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + np.arange(1, words + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def build_workload(name: str, rank: int, world: int):
    """Per-rank packet batch: (lengths, key_slot per packet, counters, nkeys, description)."""
    seed = 0x5EED2026 + 7919 * rank
    if name == "c1":
        n, L = 65536, 1420
        lengths = np.full(n, L, np.int64)
        slots = np.zeros(n, np.int64)
        counters = np.arange(n, dtype=np.uint64)
        return lengths, slots, counters, 1, f"C1: {n} x {L}B per GPU, one session key per GPU", True
    if name == "c2":
        n = 65536
        lengths = (64 + splitmix_np(seed, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
        slots = np.arange(n, dtype=np.int64) % 256
        counters = (np.arange(n, dtype=np.uint64) // 256)
        return lengths, slots, counters, 256, f"C2: {n} packets per GPU, 64..9000B, 256 session keys", False
    if name == "c3":
        total, L, sessions = 8 * 1024 * 1024, 1420, 1024
        # session s -> GPU s mod world; each session's packets carry its own counters
        my_sessions = np.arange(rank, sessions, world)
        per = total // sessions
        n = per * len(my_sessions)
        lengths = np.full(n, L, np.int64)
        slots = np.repeat(np.arange(len(my_sessions)), per)
        counters = np.tile(np.arange(per, dtype=np.uint64), len(my_sessions))
        return lengths, slots, counters, len(my_sessions), f"C3: {total} x {L}B total over {world} GPU(s), sharded by session", True
    raise SystemExit(f"unknown workload {name}")


def cpu_baseline(lengths, slots, counters, keys, budget_s: float = 1.5):
    """Time the CPU restatement (oracle) on a bounded sample of the same workload."""
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    n = min(len(lengths), 16384)
    L = lengths[:n]
    S = ((L + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = desc["out_off"] = off
    desc["counter"], desc["len"], desc["key_slot"] = counters[:n], L, slots[:n]
    inp = splitmix_np(99, int(S.sum()))
    ct = np.zeros_like(inp)
    pt = np.zeros_like(inp)
    payload = 2.0 * float(L.sum())

    def run(th, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.seal_batch(desc, inp, ct, keys, threads=th)
            st = O.open_batch(desc, ct, pt, keys, threads=th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                assert not st.any()
                return reps * payload / dt / GIB, reps

    multi, reps = run(threads, budget_s)
    single, _ = run(1, budget_s / 3)
    return {"value": round(multi, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} packets of the same workload, seal+open, {reps} reps, oracle/liboracle.so "
                      f"(-O3, bit-exact restatement of the reference C path)",
            "single_thread": round(single, 3)}


def pmc_traffic():
    """Per-launch HBM bytes of the seal kernel from the newest committed PMC summary."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return d.get("seal_hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c1", choices=["c1", "c2", "c3"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    wg = importlib.import_module("wireguard-java_amd")
    lengths, slots, counters, nkeys, wdesc, uniform = build_workload(args.workload, rank, world)
    n = len(lengths)
    keys = splitmix_np(0xC0FFEE + rank, 32 * nkeys)
    eng = wg.Engine(local, key_slots=max(nkeys, 1))
    eng.set_keys(0, keys.tobytes())

    # layout: packets at 16-byte aligned strides; pt buffer, ct||tag buffer, decrypted pt buffer
    S = ((lengths + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    desc = wg.pack_desc(off, off, counters, lengths, slots)
    total = int(S.sum())
    d_desc = torch.from_numpy(wg.desc_as_int64(desc)).to(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
    ct = torch.zeros(total, dtype=torch.uint8, device=dev)
    back = torch.zeros(total, dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)
    max_len = int(lengths.max())

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        eng.seal(d_desc, pt, ct, max_len, uniform=uniform)
        if ev is not None:
            ev[1].record()
        eng.open(d_desc, ct, back, status, max_len, uniform=uniform)
        if ev is not None:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    seal_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    open_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))

    # correctness guard on the device: open(seal(x)) == x, every tag verified
    ok_status = int(status.abs().sum().item()) == 0
    mask = torch.zeros(total, dtype=torch.bool, device=dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lengths).to(dev)
    idx = torch.arange(total, device=dev)
    pkt = torch.searchsorted(d_off, idx, right=True) - 1
    mask = (idx - d_off[pkt]) < d_len[pkt]
    ok_data = bool(torch.equal(back[mask], pt[mask]))

    payload = 2.0 * float(lengths.sum())  # sealed + opened bytes per step on this rank
    if world > 1:
        t = torch.tensor([elapsed, seal_ms, open_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, seal_ms, open_ms = t.tolist()
        p = torch.tensor([payload], dtype=torch.float64, device=dev)
        dist.all_reduce(p)
        payload_all = p.item()
        okt = torch.tensor([0 if (ok_status and ok_data) else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(okt)
        all_ok = okt.item() == 0
    else:
        payload_all = payload
        all_ok = ok_status and ok_data

    value = payload_all * args.steps / elapsed / GIB
    seal_alg = float((2 * lengths + 16).sum())  # read L + write L+16 per packet
    achieved = seal_alg / (seal_ms * 1e-3) / 1e9
    traffic = pmc_traffic() if args.workload == "c1" else None

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c3" else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (random payload in HBM, splitmix64 keys, sequential counters)",
            "config": {"workload": wdesc, "packets_per_gpu": n, "payload_bytes": int(lengths.mean()),
                       "sessions_per_gpu": nkeys, "parallelism": f"dp{world} sharded by session, no collective"},
            "roofline": {"bound": "hbm", "kernel": "k_stream<SEAL>", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "seal_ms": round(seal_ms, 4), "open_ms": round(open_ms, 4),
                         "alg_bytes_per_launch": int(seal_alg)},
            "verified": all_ok,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(lengths, slots, counters, keys)
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    if not all_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
