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
  c4            host-to-host (BASELINE configs[4]): 65536 x 1420 B from a host tun ring
                to a host UDP ring (16-B headers, 1452-B stride) and back, through
                wg_seal_host / wg_open_host; PCIe-inclusive, reported in DESIGN.md,
                never the headline value. --host-mem pinned (zero-copy or, with
                WG_HOST_PATH=copy, the copy pipeline) or pageable (copy pipeline)

Multi-GPU: one process per GPU; packets are independent, so each rank works on its own
shard — no collective on the data path. The only collectives are the timing barrier and
the max-over-ranks reduction. Under torchrun (WORLD_SIZE set) this process is one rank;
`python bench.py --gpus N` without torchrun starts the N rank processes itself (fresh
child processes, before anything touches the GPU), waits for them and exits with the
first failing rank's status. Rank 0 prints the JSON line.

The JSON line also carries:
  roofline      the transport kernel (k_step: one launch that seals and then opens the batch)
                against the 8 TB/s HBM peak: achieved = sum(4L + 32) per step / GPU time per step
                (SURVEY.md §8d), GPU time from HIP events on the launch stream around
                the timed region; `traffic` = HBM bytes per launch from the committed
                rocprofv3 PMC summary (profiles/pmc_*.json) when present.
                Steps on K > 1 streams (--streams; default 2 for uniform workloads): the batch is
                cut into K runs whose launches overlap, so a launch's duration says nothing about
                the kernel; `roofline` is then the one-stream kernel, the same steps re-timed on
                one stream right after the timed region (`kernel_ms`, one launch per step), and
                `roofline.step` the timed K-stream steps (`value` comes from those)
  cpu_baseline  the CPU restatement (oracle/liboracle.so, bit-exact to the
                reference) timed on this host's cores, rank 0, N = 1 only
  oracle_sample ct||tag of 2048 seeded packets of the timed batch against the oracle (every rank,
                its own shard), gathered right after the timed region from the buffers the timed
                launches wrote (poisoned before it); a mismatch on any rank makes `verified` false
Before the W warmup steps every rank runs untimed steps for --ramp-ms (default 150 ms)
so the GPU clocks have ramped before the timed region (ramp_ms in the JSON line).
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import re
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident AEAD GiB/s, 64K x 1420B seal+open, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue peak: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction (MI355X_MICROARCH.md)
VALU_PEAK_WIPS = 1024 * 2.4e9 / 2
GIB = float(1 << 30)


def splitmix_np(seed: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + np.arange(1, words + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def imix_lengths(seed: int, n: int) -> np.ndarray:
    """Simple IMIX payload lengths: 40, 576 and 1500 B with probabilities 7/12, 4/12 and 1/12."""
    u = splitmix_np(seed, 4 * n).view("<u4") % 12
    return np.where(u < 7, 40, np.where(u < 11, 576, 1500)).astype(np.int64)


def build_workload(name: str, rank: int, world: int, packets: int = 0, keys: int = 0):
    """Per-rank packet batch: (lengths, key_slot per packet, counters, nkeys, description).
    packets / keys (diagnostic runs only, --packets / --keys): another batch size or session count
    for C1 / C2; the description then says so."""
    seed = 0x5EED2026 + 7919 * rank
    if name == "c1":
        n, L, k = packets or 65536, 1420, keys or 1
        lengths = np.full(n, L, np.int64)
        slots = np.arange(n, dtype=np.int64) % k
        counters = np.arange(n, dtype=np.uint64) // k
        tag = "" if (n, k) == (65536, 1) else f" [diagnostic: {n} packets, {k} keys]"
        return lengths, slots, counters, k, f"C1: {n} x {L}B per GPU, one session key per GPU{tag}", True
    if name == "c2":
        n, k = packets or 65536, keys or 256
        lengths = (64 + splitmix_np(seed, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
        slots = np.arange(n, dtype=np.int64) % k
        counters = (np.arange(n, dtype=np.uint64) // k)
        tag = "" if (n, k) == (65536, 256) else f" [diagnostic: {n} packets, {k} keys]"
        return lengths, slots, counters, k, f"C2: {n} packets per GPU, 64..9000B, 256 session keys{tag}", False
    if name == "imix":
        # "also report an IMIX-like mix": simple IMIX, inner packets of 40 / 576 / 1500 B
        # in the ratio 7 : 4 : 1 (seeded draw per packet), C2's 256 sessions
        n, k = packets or 65536, keys or 256
        lengths = imix_lengths(seed, n)
        slots = np.arange(n, dtype=np.int64) % k
        counters = (np.arange(n, dtype=np.uint64) // k)
        tag = "" if (n, k) == (65536, 256) else f" [diagnostic: {n} packets, {k} keys]"
        return lengths, slots, counters, k, f"IMIX: {n} packets per GPU, 40/576/1500B at 7:4:1, 256 session keys{tag}", False
    if name == "c3":
        total, L, sessions = 8 * 1024 * 1024, 1420, 1024
        # session s -> GPU s mod world; each session's packets carry its own counters
        D = importlib.import_module("wireguard-java_amd.dist")
        slots, _, counters = D.shard_packets(total, sessions, rank, world)
        lengths = np.full(len(slots), L, np.int64)
        nkeys = len(D.session_shard(sessions, rank, world))
        return lengths, slots, counters, nkeys, f"C3: {total} x {L}B total over {world} GPU(s), sharded by session", True
    raise SystemExit(f"unknown workload {name}")


def host_cpus(cgroup_root: str = "/sys/fs/cgroup"):
    """CPUs this process can keep busy, and where the number comes from: the affinity mask, capped by
    a cgroup CPU quota (v2 `cpu.max` "quota period", or v1 `cpu/cpu.cfs_quota_us` / `cfs_period_us`).
    The same rule as the library's host_cpus() (wg_pp.hip). A GPU box here allows 16 CPUs of time while
    its affinity covers every CPU of the machine, so os.cpu_count() alone overstates what a timing can use.
    Returns (cpus, source) with source "quota" when the quota is the binding limit, else "affinity"."""
    try:
        n = len(os.sched_getaffinity(0))
        src = "affinity"
    except (AttributeError, OSError):
        n, src = os.cpu_count() or 1, "cpu_count"
    quota = None
    try:
        with open(os.path.join(cgroup_root, "cpu.max")) as f:
            q, period = f.read().split()[:2]
        if q != "max" and int(period) > 0:
            quota = max(1, int(q) // int(period))
    except (OSError, ValueError):
        try:
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_quota_us")) as f:
                q = int(f.read().strip())
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_period_us")) as f:
                period = int(f.read().strip())
            if q > 0 and period > 0:
                quota = max(1, q // period)
        except (OSError, ValueError):
            pass
    if quota is not None and quota < n:
        return quota, "quota"
    return max(1, n), src


def oracle_sample_check(sample, keys):
    """The checker, after the timed region: the ciphertext || tag the timed kernel wrote for a seeded
    sample of packets, compared byte for byte with the CPU restatement sealing the same plaintext
    (`verified` alone is open(seal(x)) == x, which a self-consistent seal bug would pass)."""
    from oracle import oracle as O
    desc, pt, ct = sample
    ref = np.zeros_like(ct)
    O.seal_batch(desc, pt, ref, keys, threads=host_cpus()[0])
    L = desc["len"].astype(np.int64)
    ok = all(np.array_equal(ct[int(o):int(o) + int(l) + 16], ref[int(o):int(o) + int(l) + 16])
             for o, l in zip(desc["in_off"], L))
    return {"packets": int(len(desc)), "bit_exact": bool(ok),
            "what": "ct||tag of a seeded sample of the timed batch vs oracle/liboracle.so sealing its plaintext"}


def cpu_baseline(lengths, slots, counters, keys, budget_s: float = 1.5, cgroup_root: str = "/sys/fs/cgroup"):
    """Time the CPU restatement (oracle) on a bounded sample of the same workload, on as many threads as
    the process may keep busy (host_cpus: affinity capped by the cgroup quota), and on one thread."""
    from oracle import oracle as O
    threads, cores_source = host_cpus(cgroup_root)
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
        reps, ts, to, t0 = 0, 0.0, 0.0, time.perf_counter()
        while True:
            a = time.perf_counter()
            O.seal_batch(desc, inp, ct, keys, threads=th)
            b = time.perf_counter()
            st = O.open_batch(desc, ct, pt, keys, threads=th)
            ts += b - a
            to += time.perf_counter() - b
            reps += 1
            if time.perf_counter() - t0 >= budget:
                assert not st.any()
                half = payload / 2
                return reps * payload / (ts + to) / GIB, reps * half / ts / GIB, reps * half / to / GIB, reps

    multi, m_seal, m_open, reps = run(threads, budget_s)
    single, s_seal, s_open, _ = run(1, budget_s / 3)
    return {"value": round(multi, 3), "unit": "GiB/s", "cores": threads, "cores_source": cores_source,
            "kind": "port",
            "sample": f"{n} packets of the same workload, seal+open, {reps} reps, oracle/liboracle.so "
                      f"(-O3, bit-exact restatement of the reference C path)",
            "seal": round(m_seal, 3), "open": round(m_open, 3),
            "single_thread": round(single, 3), "single_thread_seal": round(s_seal, 3),
            "single_thread_open": round(s_open, 3)}


def _pmc_summary(workload):
    """The newest committed PMC summary for a workload: profiles/pmc_rNN_<workload>.json as
    tools/prof_window.py writes it (timed-window dispatches only, per-kernel entries
    "k_transport<seal>" / "k_transport<open>" / "k_duplex"), else the older flat
    profiles/pmc_rNN*.json (C1 only)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_r[0-9][0-9]_{workload}.json")))
    if files:
        return "window", json.load(open(files[-1]))
    if workload != "c1":
        return None, None
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "pmc_r[0-9][0-9]*.json"))
                   if not re.search(r"_c\d\.json$", f))
    return ("flat", json.load(open(files[-1]))) if files else (None, None)


def _pmc_value(workload, mode, get, flat_get):
    """Per-launch value of a counter-derived figure: the mean of the seal and open launches (serial
    mode, or a step as two launches), the k_duplex launch (duplex mode) or the k_step launch
    (mode "fused": one WG_F_AFTER_SEAL step)."""
    try:
        fmt, d = _pmc_summary(workload)
        if fmt == "window":
            if mode == "duplex":
                return get(d["k_duplex"]) if "k_duplex" in d else None
            if mode == "fused":
                return get(d["k_step"]) if "k_step" in d else None
            v = [get(d[k]) for k in ("k_transport<seal>", "k_transport<open>") if k in d]
            return sum(v) / 2 if len(v) == 2 else None
        if fmt == "flat" and mode != "fused":
            return flat_get(d, mode)
    except (KeyError, TypeError, ValueError, OSError):
        return None
    return None


def pmc_valu_insts(workload="c1", mode="serial"):
    """SQ_INSTS_VALU per transport-kernel launch from the committed PMC summary."""
    def flat(d, mode):
        if mode == "duplex" and "duplex" in d:
            return d["duplex"]["counters_mean"]["SQ_INSTS_VALU"]
        v = [d[k]["counters_mean"]["SQ_INSTS_VALU"] for k in ("seal", "open") if k in d]
        return (sum(v) if mode == "duplex" else sum(v) / len(v)) if len(v) == 2 else None
    return _pmc_value(workload, mode, lambda e: e["counters_mean"]["SQ_INSTS_VALU"], flat)


def pmc_traffic(workload="c1", mode="serial"):
    """Per-launch HBM bytes of the transport kernel from the committed PMC summary (FETCH_SIZE and
    WRITE_SIZE passes with the gfx950 corrections, see tools/prof_window.py)."""
    def flat(d, mode):
        if mode == "duplex" and "duplex_hbm_bytes_per_launch" in d:
            return d["duplex_hbm_bytes_per_launch"]
        v = [d[k] for k in ("seal_hbm_bytes_per_launch", "open_hbm_bytes_per_launch") if k in d]
        return None if len(v) != 2 else sum(v) if mode == "duplex" else sum(v) / 2
    v = _pmc_value(workload, mode, lambda e: e["hbm_bytes_per_launch"], flat)
    return round(v) if v is not None else None


def host_bench(args):
    """configs[4]: tun ring -> seal -> UDP ring -> open -> tun ring, buffers in host memory."""
    import torch
    wg = importlib.import_module("wireguard-java_amd")
    n, L, tun_stride = 65536, 1420, 1440
    wire = 16 + L + 16
    eng = wg.Engine(0, key_slots=1)
    eng.set_keys(0, splitmix_np(0xC0FFEE, 32).tobytes())
    sd = wg.pack_desc(np.arange(n, dtype=np.uint64) * tun_stride, np.arange(n, dtype=np.uint64) * wire + 16,
                      np.arange(n, dtype=np.uint64), L, 0)
    od = sd.copy()
    od["in_off"], od["out_off"] = sd["out_off"], sd["in_off"]
    if args.host_mem == "pinned":
        tun, ring, back = eng.host_alloc(n * tun_stride), eng.host_alloc(n * wire), eng.host_alloc(n * tun_stride)
    else:
        tun, ring, back = (np.empty(n * tun_stride, np.uint8), np.empty(n * wire, np.uint8),
                           np.empty(n * tun_stride, np.uint8))
    tun[:] = splitmix_np(0x5EED2026, n * tun_stride)
    ring[:] = 0
    back[:] = 0

    def step():
        eng.seal_host(sd, tun, ring, L, uniform=True)
        st = eng.open_host(od, ring, back, L, uniform=True)
        return st

    for _ in range(args.warmup):
        step()
    seal_t = open_t = 0.0
    for _ in range(args.steps):
        t0 = time.perf_counter()
        eng.seal_host(sd, tun, ring, L, uniform=True)
        t1 = time.perf_counter()
        st = eng.open_host(od, ring, back, L, uniform=True)
        t2 = time.perf_counter()
        seal_t += t1 - t0
        open_t += t2 - t1
    ok = not st.any() and np.array_equal(back.reshape(n, tun_stride)[:, :L], tun.reshape(n, tun_stride)[:, :L])
    payload = 2.0 * n * L * args.steps
    mode = os.environ.get("WG_HOST_PATH", "auto")
    path = "zero-copy" if args.host_mem == "pinned" and mode != "copy" else "copy pipeline"
    print(json.dumps({
        "metric": "host-to-host AEAD GiB/s (PCIe-inclusive), 64K x 1420B seal+open, 1 MI355X",
        "value": round(payload / (seal_t + open_t) / GIB, 2), "unit": "GiB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round((seal_t + open_t) * 1e3 / args.steps, 3), "higher_is_better": True,
        "seal_ms": round(seal_t * 1e3 / args.steps, 3), "open_ms": round(open_t * 1e3 / args.steps, 3),
        "host_mem": args.host_mem, "path": path, "verified": bool(ok),
        "config": {"workload": "C4: tun ring (1440-B slots) -> UDP ring (16-B header + ct||tag, 1452-B stride) "
                               "-> tun ring, 65536 x 1420B, host buffers"}}), flush=True)
    if args.host_mem == "pinned":
        for a in (tun, ring, back):
            eng.host_free(a)
    eng.close()
    del torch


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start one child process per GPU (rank i on GPU i) with the torchrun environment and
    wait for all of them. Nothing here touches the GPU; the children are new processes."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def launch_check(args):
    """--launch-check: the multi-rank plumbing without a GPU (gloo on CPU): rendezvous,
    barrier-bracketed timing, max-over-ranks and payload sum, rank 0's JSON line."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    elapsed = time.perf_counter() - t0
    D = importlib.import_module("wireguard-java_amd.dist")
    per_gpu = D.gather_per_rank(dist if world > 1 else None, "cpu", {
        "elapsed_s": elapsed, "payload_bytes": 1000.0 * (rank + 1), "packets": 10 * (rank + 1), "seal_ms": 0.0,
        "open_ms": 0.0, "kernel_ms": 0.0})
    if world > 1:
        (elapsed,), payload, ok = D.reduce_report(dist, "cpu", [elapsed], 1000.0 * (rank + 1), True)
        dist.barrier()
        dist.destroy_process_group()
    else:
        payload, ok = 1000.0, True
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "elapsed_max": elapsed,
                          "payload_sum": payload, "ok": ok, "per_gpu": per_gpu}), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    # untimed seal+open steps for at least this long before the warmup steps: the
    # MI355X raises its clocks over the first tens of ms of load (a 20-step run measured
    # 961-1027 GiB/s on C1, 1220 once ramped; profiles/r01_kernel_study.md §5)
    ap.add_argument("--ramp-ms", type=float, default=150.0)
    ap.add_argument("--workload", default="c1", choices=["c1", "c2", "c3", "c4", "imix"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-mem", default="pinned", choices=["pinned", "pageable"])
    # --streams K: each step's batch as K runs of consecutive packets, each sealed and opened on its own
    # HIP stream (the same packets and bytes per step); 0 = auto: 2 for the uniform workloads, whose
    # one-launch steps otherwise leave the machine partly idle while each launch's last waves drain
    # (C1 +7-9% in an alternating A/B, profiles/r04_streams_ab.jsonl), 1 for C2 (its half batches
    # take a different slot plan: -4%)
    ap.add_argument("--streams", type=int, default=0)
    # --stagger 1 (default with two streams): the second stream runs a continuous stream of half-batch launches
    # offset by a quarter batch (its first launch is the first quarter of its half, every later one a half batch
    # window that wraps around its half, its last the remaining quarter), so the two streams' launches are half a
    # launch apart from the first step, as in a long run, and end together; every packet is still sealed and
    # opened exactly once per step. --stagger 0: both streams start and end on the same batch boundaries
    # (measured in round 6 on the driver's 20-step command, six alternations: medians 1,462 vs 1,470 GiB/s, the
    # same GPU time per step; profiles/r06_stagger_ab.jsonl. Off by default: the plain batch-aligned schedule)
    ap.add_argument("--stagger", type=int, default=0, choices=[0, 1])
    # the end of the timed region is detected by polling the last event (as a pipeline stage polls its
    # completion) instead of the blocking synchronize alone, whose wake-up adds to every run's wall time;
    # --spin-sync 0: the blocking synchronize only
    ap.add_argument("--spin-sync", type=int, default=1, choices=[0, 1])
    # duplex: each step is ONE wg_duplex_batch launch that seals this step's batch and opens
    # the previous step's ciphertext (double-buffered); serial: a seal launch, then an open
    # launch of the same batch
    # step: ONE wg_duplex_batch(seal, open | WG_F_AFTER_SEAL) per step: the seal launch, then the open
    # launch of what it sealed (the same two launches as serial; a mixed-length batch is ordered
    # longest-first once for both); serial: wg_seal_batch, then wg_open_batch
    ap.add_argument("--mode", default="step", choices=["step", "serial", "duplex"])
    ap.add_argument("--kernel", default="default", help="transport kernel (wg_ctx_set_kernel): default|wave1|tile")
    # --variant 1: a WG_F_AFTER_SEAL step as two launches (seal, then open) instead of one k_step launch
    ap.add_argument("--variant", type=int, default=0, choices=[0, 1])
    # --graph: the K timed steps are captured once into a HIP graph (torch.cuda.CUDAGraph) and the timed
    # region is one replay of it: the same launches with no host enqueue between them (used for the
    # kernel traces, where the profiler makes each host enqueue slower than a step)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    # multi-rank rehearsal on a one-GPU box (not the metric's configuration): the report's collectives
    # over gloo instead of RCCL, and every rank on cuda:0 with its own wg_ctx (tests/test_gpu_dist.py)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    # diagnostic knobs (not the metric's configuration): batch size and session count of C1 / C2
    ap.add_argument("--packets", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--keys", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if args.launch_check:
        return launch_check(args)
    if args.workload == "c4":
        return host_bench(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torchrun (WORLD_SIZE set) the ranks always form an RCCL group, one rank included, so the
    # rendezvous, barriers and gathers of the multi-GPU line run on the GPU path at any N
    use_dist = "WORLD_SIZE" in os.environ
    if args.same_device:
        local = 0
    if use_dist:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    rdev = dev if args.dist_backend == "nccl" else "cpu"  # where the report's reductions run

    wg = importlib.import_module("wireguard-java_amd")
    lengths, slots, counters, nkeys, wdesc, uniform = build_workload(args.workload, rank, world, args.packets, args.keys)
    n = len(lengths)
    keys = splitmix_np(0xC0FFEE + rank, 32 * nkeys)
    eng = wg.Engine(local, key_slots=max(nkeys, 1))
    eng.set_kernel(args.kernel, variant=args.variant if args.kernel in ("default", "transport") else 0)
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

    # --streams K: the batch is cut into K runs of consecutive packets, each sealed and
    # then opened on its own stream; the runs' kernels overlap, so one run's launch tail
    # is filled by another run's waves (the work and every packet's seal -> open order
    # are unchanged)
    K = args.streams if args.streams > 0 else (2 if uniform and args.mode == "step" else 1)
    cuts = [n * i // K for i in range(K + 1)]
    fused_step_mode = args.mode == "step" and args.kernel in ("default", "transport") and args.variant == 0
    main_stream = torch.cuda.current_stream()
    side = [main_stream] if K == 1 else [torch.cuda.Stream(device=dev) for _ in range(K)]

    cts = [ct, torch.zeros_like(ct)] if args.mode == "duplex" else [ct]
    k_step = [0]

    # prepared launches (engine.prepare_duplex): one foreign call per launch, the argument structs built once,
    # each bound to its stream, so the host enqueues a step in a few microseconds and the first launch of the
    # timed region starts sooner after t0 (not with --graph, whose capture runs on torch's capture stream)
    stagger = K == 2 and args.mode == "step" and args.stagger == 1 and not args.graph and args.kernel in (
        "default", "transport") and args.variant == 0
    st2 = None
    prep_a = prep_b = prep_q1 = prep_w = prep_q2 = None
    if K == 2 and fused_step_mode and not args.graph:
        a, b = cuts[0], cuts[1]
        prep_a = eng.prepare_duplex(d_desc[a:b], pt, ct, max_len, d_desc[a:b], ct, back, status[a:b], max_len,
                                    uniform=uniform, after_seal=True, stream=side[0].cuda_stream)
        if stagger:
            # stream B's half as a ring of descriptors (its half twice) with its own statuses: launch windows of
            # m packets starting at a quarter of the half wrap around it and stay contiguous
            m = n - cuts[1]
            q = m // 2
            desc2 = torch.cat([d_desc[cuts[1]:], d_desc[cuts[1]:cuts[1] + q]])  # B's half, then its first quarter again
            st2 = torch.zeros(m + q, dtype=torch.int32, device=dev)
            st2_used = m + q if args.steps >= 2 else m  # a one-step window runs Q1 and Q2 only
            sb = side[1].cuda_stream
            prep_q1 = eng.prepare_duplex(desc2[:q], pt, ct, max_len, desc2[:q], ct, back, st2[:q], max_len,
                                         uniform=uniform, after_seal=True, stream=sb)
            prep_w = eng.prepare_duplex(desc2[q:q + m], pt, ct, max_len, desc2[q:q + m], ct, back, st2[q:q + m],
                                        max_len, uniform=uniform, after_seal=True, stream=sb)
            prep_q2 = eng.prepare_duplex(desc2[q:m], pt, ct, max_len, desc2[q:m], ct, back, st2[q:m], max_len,
                                         uniform=uniform, after_seal=True, stream=sb)
        else:
            a, b = cuts[1], cuts[2]
            prep_b = eng.prepare_duplex(d_desc[a:b], pt, ct, max_len, d_desc[a:b], ct, back, status[a:b], max_len,
                                        uniform=uniform, after_seal=True, stream=side[1].cuda_stream)
    prep_one = None
    if K == 1 and fused_step_mode and not args.graph:
        prep_one = eng.prepare_duplex(d_desc, pt, ct, max_len, d_desc, ct, back, status, max_len, uniform=uniform,
                                      after_seal=True, stream=main_stream.cuda_stream)
    launch_count = [0]  # transport launches enqueued so far (the profiler tools' window)

    def run_steps(k):
        """k steps on the K streams (between fork() and join())."""
        if k <= 0:
            return
        if prep_one is not None:
            for _ in range(k):
                prep_one()
            launch_count[0] += k
            return
        if prep_a is None:
            for _ in range(k):
                step()
            launch_count[0] += k * (1 if args.mode == "duplex" else K * (1 if fused_step_mode else 2))
            return
        if not stagger:
            for _ in range(k):
                prep_a()
                prep_b()
            launch_count[0] += 2 * k
            return
        prep_a()
        prep_q1()
        for _ in range(k - 1):
            prep_a()
            prep_w()
        prep_q2()
        launch_count[0] += 2 * k + 1

    def step_duplex():
        k = k_step[0]
        k_step[0] += 1
        eng.duplex(d_desc, pt, cts[k & 1], max_len, d_desc, cts[(k + 1) & 1], back, status, max_len, uniform=uniform)

    def step():
        if args.mode == "duplex":
            return step_duplex()
        if K == 1:  # the current stream (a graph's capture stream under --graph)
            if args.mode == "step":
                eng.duplex(d_desc, pt, ct, max_len, d_desc, ct, back, status, max_len, uniform=uniform,
                           after_seal=True)
            else:
                eng.seal(d_desc, pt, ct, max_len, uniform=uniform)
                eng.open(d_desc, ct, back, status, max_len, uniform=uniform)
            return
        if args.mode == "step":
            for i in range(K):
                a, b = cuts[i], cuts[i + 1]
                with torch.cuda.stream(side[i]):
                    eng.duplex(d_desc[a:b], pt, ct, max_len, d_desc[a:b], ct, back, status[a:b], max_len,
                               uniform=uniform, after_seal=True)
            return
        for i in range(K):
            a, b = cuts[i], cuts[i + 1]
            with torch.cuda.stream(side[i]):
                eng.seal(d_desc[a:b], pt, ct, max_len, uniform=uniform)
                eng.open(d_desc[a:b], ct, back, status[a:b], max_len, uniform=uniform)

    def fork():
        if K > 1:
            for s_ in side:
                s_.wait_stream(main_stream)

    def join():
        if K > 1:
            for s_ in side:
                main_stream.wait_stream(s_)

    if args.mode == "duplex":
        if K != 1:
            raise SystemExit("--mode duplex uses one stream")
        eng.seal(d_desc, pt, cts[1], max_len, uniform=uniform)  # the first step opens this
    fork()
    t_ramp = time.perf_counter()
    ramp_steps = 0
    while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        run_steps(16)
        ramp_steps += 16
        torch.cuda.synchronize()
    run_steps(args.warmup)
    join()
    torch.cuda.synchronize()
    launches_before = launch_count[0]

    # HIP events on the stream the kernels are launched on (torch's current stream,
    # which Engine passes to wg_seal_batch / wg_open_batch), around the whole region
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if args.graph:
        if args.mode == "duplex":
            raise SystemExit("--graph captures step launches (--mode step|serial)")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cap = torch.cuda.current_stream()
            if K > 1:  # the K streams' chains fork from and join back into the capture stream
                for s_ in side:
                    s_.wait_stream(cap)
            for _ in range(args.steps):
                step()
            if K > 1:
                for s_ in side:
                    cap.wait_stream(s_)
        graph.replay()  # warm: the graph's first launch
        torch.cuda.synchronize()
    # every output the check below reads is poisoned first, so the check certifies what the timed
    # launches themselves wrote (not a ramp, warmup or graph-warm step); duplex mode opens the previous
    # step's ciphertext, so its buffers stay as the warmup left them
    if args.mode != "duplex":
        ct.fill_(0x5A)
        back.fill_(0xA5)
        status.fill_(-1)
        if st2 is not None:
            st2.fill_(-1)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        fork()  # the K streams start after ev0 ...
        run_steps(args.steps)
        join()  # ... and ev1 waits for all of them
    t_enq = time.perf_counter()  # host time to enqueue the steps (the GPU idles if it is ~ ms_per_step)
    ev1.record()
    if args.spin_sync:
        while not ev1.query():  # every kernel of the region has completed once the last event has
            pass
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    elapsed = t1 - t0
    gpu_step_ms = ev0.elapsed_time(ev1) / args.steps  # = t_seal + t_open (back-to-back launches), or t_duplex

    # correctness guard on the device, on the buffers the timed launches wrote (nothing has run since):
    # open(seal(x)) == x with every tag verified, and below the ct||tag of a seeded sample against the
    # oracle. The re-timing and the per-kernel trains after this overwrite ct / back / status.
    window_launches = launch_count[0] - launches_before
    if st2 is not None:  # stream B's packets report through its ring of statuses
        ok_status = int(status[:cuts[1]].abs().sum().item()) == 0 and int(st2[:st2_used].abs().sum().item()) == 0
    else:
        ok_status = int(status.abs().sum().item()) == 0
    if uniform:  # equal strides: compare the [n, L] payload views directly
        s0, L0 = int(S[0]), int(lengths[0])
        ok_data = bool(torch.equal(back.view(n, s0)[:, :L0], pt.view(n, s0)[:, :L0]))
    else:
        d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lengths).to(dev)
        idx = torch.arange(total, device=dev)
        pkt = torch.searchsorted(d_off, idx, right=True) - 1
        mask = (idx - d_off[pkt]) < d_len[pkt]
        ok_data = bool(torch.equal(back[mask], pt[mask]))
        del idx, pkt, mask

    # a seeded sample of the timed batch, copied out for the oracle check (every rank checks its own
    # shard; the oracle is the checker, never the thing measured)
    sample = None
    if not args.no_cpu_baseline:
        pick = np.sort(np.random.default_rng(4242).choice(n, min(n, 2048), replace=False))
        sd = desc[pick].copy()
        SS = S[pick]
        so = np.concatenate([[0], np.cumsum(SS)[:-1]]).astype(np.uint64)
        sd["in_off"] = sd["out_off"] = so
        spt = np.zeros(int(SS.sum()), np.uint8)
        sct = np.zeros(int(SS.sum()), np.uint8)
        if uniform:  # equal strides: gather the sampled rows on the device (C3's buffers are 12 GB)
            s0 = int(S[0])
            idx = torch.from_numpy(pick.astype(np.int64)).to(dev)
            spt[:] = pt.view(n, s0).index_select(0, idx).cpu().numpy().reshape(-1)
            sct[:] = ct.view(n, s0).index_select(0, idx).cpu().numpy().reshape(-1)
            del idx
        else:
            pt_h, ct_h = pt.cpu().numpy(), ct.cpu().numpy()
            for k, i in enumerate(pick):
                o, ln = int(off[i]), int(lengths[i])
                spt[int(so[k]):int(so[k]) + ln] = pt_h[o:o + ln]
                sct[int(so[k]):int(so[k]) + ln + 16] = ct_h[o:o + ln + 16]
            del pt_h, ct_h
        sample = (sd, spt, sct)

    # K > 1: the launches of a step overlap, so a launch's duration is not its share of the step; the
    # roofline of the dominant kernel comes from the same steps on ONE stream, timed right after (the
    # kernel alone, back to back), and the value from the K-stream steps above
    single_ms = None
    if K > 1 and graph is None and args.mode == "step":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the checks above left the GPU idle for a few ms: ramp the clocks again before timing (a re-timing
        # straight after them measured the kernel 10% slow, gpurun_out/r05a)
        t_r = time.perf_counter()
        while (time.perf_counter() - t_r) * 1e3 < args.ramp_ms:
            for _ in range(8):
                eng.duplex(d_desc, pt, ct, max_len, d_desc, ct, back, status, max_len, uniform=uniform, after_seal=True)
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.steps):
            eng.duplex(d_desc, pt, ct, max_len, d_desc, ct, back, status, max_len, uniform=uniform, after_seal=True)
        e1.record()
        torch.cuda.synchronize()
        single_ms = e0.elapsed_time(e1) / args.steps

    # per-kernel split (not in the timed region): seal-only and open-only launch trains
    def train(fn, k=10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(k):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / k
    seal_ms = train(lambda: eng.seal(d_desc, pt, ct, max_len, uniform=uniform))
    open_ms = train(lambda: eng.open(d_desc, ct, back, status, max_len, uniform=uniform))

    # achievable streaming bandwidth for context: a device-to-device copy of the
    # plaintext buffer, read + write bytes per copy time (after the check above, untimed)
    copy_ms = train(lambda: back.copy_(pt))
    copy_gbs = 2.0 * pt.numel() / (copy_ms * 1e-3) / 1e9

    # the oracle check of this rank's sample (before the reductions: a mismatch on any rank fails the line)
    sample_res = oracle_sample_check(sample, keys) if sample is not None else None
    sample_ok = sample_res is None or sample_res["bit_exact"]

    payload = 2.0 * float(lengths.sum())  # sealed + opened bytes per step on this rank
    D = importlib.import_module("wireguard-java_amd.dist")
    # transport kernel launches per step: k_duplex, or k_step (one WG_F_AFTER_SEAL step), or seal + open
    fused_step = args.mode == "step" and args.kernel in ("default", "transport") and args.variant == 0
    launches = (1 if (args.mode == "duplex" or fused_step) else 2) * (K if args.mode != "duplex" else 1)
    # this rank's own figures, gathered before the max-over-ranks reduction (BASELINE configs[3]:
    # per-GPU and aggregate GiB/s)
    per_gpu = D.gather_per_rank(dist if use_dist else None, rdev, {
        "elapsed_s": elapsed, "payload_bytes": payload * args.steps, "packets": n, "seal_ms": seal_ms,
        "open_ms": open_ms, "kernel_ms": gpu_step_ms / launches})
    if use_dist:
        (elapsed, seal_ms, open_ms, gpu_step_ms), payload_all, all_ok = D.reduce_report(
            dist, rdev, [elapsed, seal_ms, open_ms, gpu_step_ms], payload, ok_status and ok_data and sample_ok)
    else:
        payload_all = payload
        all_ok = ok_status and ok_data and sample_ok

    value = payload_all * args.steps / elapsed / GIB
    # seal reads L, writes L+16; open reads L+16, writes L -> 4L+32 per packet
    step_alg = float((4 * lengths + 32).sum())
    step_rate = step_alg / (gpu_step_ms * 1e-3) / 1e9  # the whole step (all K streams), GPU time
    # the dominant kernel's roofline: one launch's algorithmic bytes over its duration (K = 1: the steps
    # above; K > 1: the same steps on one stream, single_ms)
    if single_ms is not None:
        k_launches, k_ms = 1, single_ms
    else:
        k_launches, k_ms = launches, gpu_step_ms / launches
    achieved = step_alg / k_launches / (k_ms * 1e-3) / 1e9
    pmc_mode = "fused" if fused_step else args.mode
    traffic = pmc_traffic(args.workload, pmc_mode)
    valu = pmc_valu_insts(args.workload, pmc_mode)

    if args.mode == "duplex":
        kname = "k_duplex (seal + open halves)"
        knames = ["k_duplex"]
    elif fused_step:
        kname = "k_step (seal, then open of the same packets, per wave)"
        knames = ["k_step"]
    else:
        kname = "k_transport<SEAL|OPEN>" if args.kernel == "default" else args.kernel
        base = {"default": "k_transport", "transport": "k_transport", "wave1": "k_wave", "tile": "k_tile"}[args.kernel]
        knames = [base + "<seal>", base + "<open>"]
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ramp_ms": args.ramp_ms,
            "ramp_steps": ramp_steps,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "host_enqueue_ms_per_step": round((t_enq - t0) * 1e3 / args.steps, 4),
            "graph": bool(args.graph),
            "graph_warm_steps": args.steps if args.graph else 0,  # the graph's warm replay, before the timed one
            # transport-kernel launches enqueued before the timed region and inside it (tools/prof_window.py)
            "launches_before_window": launches_before if graph is None else None,
            "window_launches": window_launches if graph is None else None,
            "stagger": bool(stagger),
            "spin_sync": bool(args.spin_sync),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c3" else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (random payload in HBM, splitmix64 keys, sequential counters)",
            "config": {"workload": wdesc, "packets_per_gpu": n, "payload_bytes": int(lengths.mean()), "step": args.mode,
                       "streams": K,
                       "sessions_per_gpu": nkeys, "parallelism": f"dp{world} sharded by session, no collective",
                       **({"rehearsal": f"{world} ranks on cuda:0, report over {args.dist_backend}"}
                          if args.same_device else {})},
            "roofline": {"bound": "hbm", "kernel": kname + (", one stream" if single_ms is not None else ""),
                         "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "alg_bytes_per_launch": int(step_alg / k_launches),
                         "launches_per_step": k_launches, "kernel_names": knames,
                         "kernel_ms": round(k_ms, 5), "seal_ms": round(seal_ms, 5),
                         "open_ms": round(open_ms, 5), "copy_gbs": round(copy_gbs, 1),
                         "frac_of_copy": round(achieved / copy_gbs, 4),
                         # the timed K-stream steps: their launches overlap (one stream's kernel tail is
                         # filled by the next step on the other stream), so the rate per step is higher
                         "step": {"streams": K, "launches": launches, "achieved": round(step_rate, 1),
                                  "frac": round(step_rate / HBM_PEAK_GBS, 4), "ms": round(gpu_step_ms, 5)}},
            "verified": all_ok,
            "verified_on": ("the timed launches' own outputs: ct / back / status poisoned before the timed region, "
                            "checked (and the oracle sample gathered) before any other launch"
                            if args.mode != "duplex" else "the last timed step's outputs"),
            "per_gpu": [{"rank": r["rank"], "gib_s": round(r["gib_s"], 2), "packets_per_step": r["packets"],
                         "elapsed_s": round(r["elapsed_s"], 6), "seal_ms": round(r["seal_ms"], 5),
                         "open_ms": round(r["open_ms"], 5), "kernel_ms": round(r["kernel_ms"], 5)} for r in per_gpu],
        }
        if valu:
            rate = valu / (k_ms * 1e-3)
            line["valu_roofline"] = {"insts_per_launch": round(valu), "achieved": round(rate / 1e12, 4),
                                     "peak": round(VALU_PEAK_WIPS / 1e12, 4), "unit": "T wave-instr/s",
                                     "frac": round(rate / VALU_PEAK_WIPS, 4), "source": "SQ_INSTS_VALU, profiles/pmc_*.json"}
        if sample_res is not None:
            line["oracle_sample"] = dict(sample_res, ranks=world, all_ranks_verified=bool(all_ok))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(lengths, slots, counters, keys)
        print(json.dumps(line), flush=True)
    eng.close()
    if use_dist:
        dist.destroy_process_group()
    if not all_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
