"""Times wg_frame_seal and wg_parse_open on a C1-shaped batch (65536 packets, 1452-B
wire packets in 4096-B ring slots) with HIP events on torch's current stream, the
stream both calls launch on. Usage: python tools/bench_framing.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import importlib  # noqa: E402

W = importlib.import_module("wireguard-java_amd")


def main():
    n, L, slot, reps = 65536, 1420, 4096, 200
    dev = torch.device("cuda", 0)
    e = W.Engine(0, key_slots=256)
    desc = np.zeros(n, W.WG_PKT_DTYPE)
    desc["out_off"] = np.arange(n, dtype=np.uint64) * slot + 16
    desc["counter"] = np.arange(n, dtype=np.uint64)
    desc["len"] = L
    desc["key_slot"] = np.arange(n) % 256
    dt = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    rx = torch.arange(256, dtype=torch.int32, device=dev)
    ring = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    wl = torch.full((n,), L + 32, dtype=torch.int32, device=dev)
    ks = torch.zeros(n, dtype=torch.int32, device=dev)
    od = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    out = {}
    for name, fn in [("frame_seal", lambda: e.frame_seal(dt, rx, ring)),
                     ("parse_open", lambda: e.parse_open(ring, off, wl, ks, od, pst))]:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(a.elapsed_time(b) * 1000.0 / reps, 2)
    assert int(pst.sum()) == 0 and int(od[:, 3].min()) >= 0
    out.update({"packets": n, "wire_bytes": L + 32, "slot": slot})
    print(json.dumps(out))
    e.close()


if __name__ == "__main__":
    main()
