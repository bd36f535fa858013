"""k_step_mixed time per step for single-length batches and the IMIX mix, with the 2-lane tiny part on or off
(WG_SLOT2 from the environment). Diagnostic for where the IMIX step's time goes: 65,536 packets each of
40, 576 and 1,500 B and bench.py's IMIX batch, 256 keys, WG_F_AFTER_SEAL steps timed with HIP events over
--reps steps after a warmup. Prints one JSON line per batch."""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    import torch

    import bench
    wg = importlib.import_module("wireguard-java_amd")
    dev = torch.device("cuda", 0)
    eng = wg.Engine(0, key_slots=256)
    eng.set_keys(0, bench.splitmix_np(0xC0FFEE, 32 * 256).tobytes())
    n = 65536
    batches = {f"{L}B": np.full(n, L, np.int64) for L in (40, 576, 1500)}
    batches["imix"] = bench.build_workload("imix", 0, 1)[0]
    for name, lengths in batches.items():
        S = ((lengths + 16 + 15) // 16) * 16
        off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
        desc = wg.pack_desc(off, off, np.arange(n, dtype=np.uint64) // 256, lengths, np.arange(n) % 256)
        d = torch.from_numpy(wg.desc_as_int64(desc)).to(dev)
        total = int(S.sum())
        pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
        ct = torch.zeros_like(pt)
        back = torch.zeros_like(pt)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        ml = int(lengths.max())
        step = eng.prepare_duplex(d, pt, ct, ml, d, ct, back, st, ml, uniform=False, after_seal=True,
                                  stream=torch.cuda.current_stream().cuda_stream)
        for _ in range(10):
            step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / args.reps
        print(json.dumps({"slot2": int(os.environ.get("WG_SLOT2", "0")), "batch": name, "us_per_step": round(us, 2),
                          "GiB_s": round(2 * int(lengths.sum()) / (us * 1e-6) / 2**30, 1),
                          "ok": int(st.abs().sum()) == 0}))


if __name__ == "__main__":
    main()
