"""Per-phase cycle split of k_transport (diagnostic library, make -C wireguard-java_amd/csrc diag).

Runs C1 seal (or --mode open) launches on cuda:0 with libwgaead_diag.so, whose kernel
accumulates s_memtime deltas per phase of the round loop per wave, and prints the mean
cycles per wave and per round for each phase:
  desc wait (until the next descriptor has landed), start (key load + record sync), dma+chacha, xor/store/image, scan (round 0 only),
  poly, finish, loop.
Stamps themselves cost cycles (MI355X_MICROARCH.md: ~11%); compare phases, not totals with
the product build."""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("WG_LIB_PATH", os.path.join(ROOT, "wireguard-java_amd", "libwgaead_diag.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="seal", choices=["seal", "open", "step"])
    ap.add_argument("--workload", default="c1", choices=["c1", "c2"])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--keys", type=int, default=256, help="session keys (C1: 1)")
    args = ap.parse_args()
    import torch
    torch.cuda.is_available()
    wg = importlib.import_module("wireguard-java_amd")
    lib = wg.lib()
    lib.wg_diag_stamps.argtypes = [ctypes.c_void_p]
    n = 65536
    if args.workload == "c1":
        lengths = np.full(n, 1420, np.int64)
    else:
        rng = np.random.default_rng(1)
        lengths = rng.integers(64, 9001, n)
    S = ((lengths + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    eng = wg.Engine(0, key_slots=256)
    eng.set_keys(0, np.random.default_rng(2).integers(0, 256, 32 * 256, dtype=np.uint8).tobytes())
    desc = wg.pack_desc(off, off, np.arange(n, dtype=np.uint64), lengths, np.arange(n) % args.keys)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(wg.desc_as_int64(desc)).to(dev)
    total = int(S.sum())
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    ct = torch.zeros_like(pt)
    back = torch.zeros_like(pt)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    ml = int(lengths.max())
    uni = args.workload == "c1"
    eng.seal(d, pt, ct, ml, uniform=uni)
    stamps = torch.zeros(2 * 16384 * 10, dtype=torch.int64, device=dev)

    def launch():
        if args.mode == "seal":
            eng.seal(d, pt, ct, ml, uniform=uni)
        elif args.mode == "step":  # one k_step launch: each wave seals, then opens (stamps: seal half, open half)
            eng.duplex(d, pt, ct, ml, d, ct, back, st, ml, uniform=uni, after_seal=True)
        else:
            eng.open(d, ct, back, st, ml, uniform=uni)

    for _ in range(args.reps):  # ramp the clocks with stamps off
        launch()
    torch.cuda.synchronize()
    lib.wg_diag_stamps(stamps.data_ptr())
    launch()
    torch.cuda.synchronize()
    lib.wg_diag_stamps(None)
    a = stamps.cpu().numpy().reshape(-1, 10)  # 7 phase sums, unused, start time, end time
    if not (a != 0).any():
        raise SystemExit(f"no stamps written (lib {os.environ.get('WG_LIB_PATH')}, ptr {stamps.data_ptr():#x})")
    if args.mode == "step":  # wave w: seal half at w, open half at w + waves: life = seal start .. open end
        waves = int(np.argmax(a[:, 9] == 0)) // 2  # the seal half's rows, then as many open rows
        sa, oa = a[:waves], a[waves:2 * waves]
        a = sa.copy()
        a[:, :7] += oa[:, :7]
        a[:, 9] = oa[:, 9]
    a = a[a[:, 9] > 0]
    rounds = (6 if args.mode == "step" else 3) if args.workload == "c1" else None
    names = ["start", "dma+chacha", "xor/store/img", "scan", "poly", "finish", "desc wait"]
    mean = a[:, :7].mean(axis=0)
    # wave lifetimes from s_memrealtime (100 MHz): start / end relative to the first wave
    t0 = a[:, 8].min()
    st_us = (a[:, 8] - t0) / 100.0
    en_us = (a[:, 9] - t0) / 100.0
    span = float(en_us.max())
    grid = np.linspace(0, span, 41)
    live = [int(((st_us <= t) & (en_us > t)).sum()) for t in grid]
    # idle share of the launch after each wave's end: sum over waves of (span - end) / (waves x span)
    tail_idle = float((span - en_us).sum() / (len(en_us) * span)) if span > 0 else 0.0
    out = {"mode": args.mode, "workload": args.workload, "waves": int(len(a)),
           "cycles_per_wave": {k: round(float(mean[i]), 1) for i, k in enumerate(names)},
           "kernel_span_us": round(span, 2), "wave_life_us_mean": round(float((en_us - st_us).mean()), 2),
           "wave_start_us": [round(float(np.percentile(st_us, p)), 2) for p in (0, 25, 50, 75, 100)],
           "wave_end_us": [round(float(np.percentile(en_us, p)), 2) for p in (0, 10, 25, 50, 75, 90, 100)],
           "tail_idle_frac": round(tail_idle, 4), "live_waves_over_time": live}
    if rounds:
        out["cycles_per_round"] = {k: round(float(mean[i]) / rounds, 1) for i, k in enumerate(names)}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
