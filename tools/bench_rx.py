"""Timing of the receive side on a C1-shaped batch (65536 x 1420 B IPv4 plaintexts, one key slot
with a 3-prefix AllowedIPs filter), after a 150-ms clock ramp:
  open, open with the fused filter (wg_open_batch WG_F_RX_FILTER), open then wg_rx_check(FILTER);
  wg_rx_check alone: filter, replay, both; replay over 1024 key slots.
HIP events on the launch stream around each of 200 calls (open variants: 200 calls each,
alternating between the variants); the replay window is re-enabled (emptied, untimed) before each
replay call so every call sees fresh counters. WG_RX_LAUNCHES=5 times the five-launch replay path
(the default: three launches for tables of at most 512 key slots, four above)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import importlib
    import torch
    W = importlib.import_module("wireguard-java_amd")
    dev = torch.device("cuda", 0)
    n, L, S = 65536, 1420, 1440
    eng = W.Engine(0, key_slots=16)
    eng.filter_set(0, [("10.0.0.0", 8), ("192.168.0.0", 16), ("2001:db8::", 32)])
    eng.slot_filters_set(0, [0])
    pt = np.zeros((n, S), np.uint8)
    pt[:, 0] = 0x45
    rng = np.random.default_rng(1)
    pt[:, 16] = np.where(rng.random(n) < 0.9, 10, 11)
    pt[:, 17:20] = rng.integers(0, 256, (n, 3))
    d = torch.from_numpy(W.desc_as_int64(W.pack_desc(np.arange(n) * S, np.arange(n) * S, np.arange(n), L, 0))).to(dev)
    dpt = torch.from_numpy(pt.reshape(-1)).to(dev)
    st0 = torch.zeros(n, dtype=torch.int32, device=dev)
    st = st0.clone()
    out = {"n": n, "rx_launches": 5 if os.environ.get("WG_RX_LAUNCHES") == "5" else 3}
    eng.set_keys(0, bytes(range(32)))
    ct = torch.zeros_like(dpt)
    back = torch.zeros_like(dpt)
    eng.seal(d, dpt, ct, L, uniform=True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:  # clock ramp
        eng.open(d, ct, back, st, L, uniform=True, rx_filter=True)
        eng.rx_check(d, back, st, 1)
        torch.cuda.synchronize()
    variants = {
        "open": lambda: eng.open(d, ct, back, st, L, uniform=True),
        "open_fused_filter": lambda: eng.open(d, ct, back, st, L, uniform=True, rx_filter=True),
        "open_then_rx_filter": lambda: (eng.open(d, ct, back, st, L, uniform=True), eng.rx_check(d, back, st, 1)),
    }
    tot = {k: 0.0 for k in variants}
    for _ in range(200):
        for k, f in variants.items():
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            tot[k] += a.elapsed_time(b)
    for k in variants:
        out[k + "_us"] = round(tot[k] / 200 * 1e3, 2)
    variants["open_fused_filter"]()
    torch.cuda.synchronize()
    out["open_fused_filter_status_hist"] = np.bincount(st.cpu().numpy(), minlength=7).tolist()
    for name, flags in (("filter", 1), ("replay", 2), ("filter+replay", 3)):
        if flags & 2:
            eng.replay_enable(8192)
        reps = 200
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(10):
            st.copy_(st0)
            eng.rx_check(d, dpt, st, flags)
        torch.cuda.synchronize()
        tot = 0.0
        for _ in range(reps):
            st.copy_(st0)
            if flags & 2:
                eng.replay_enable(8192)  # fresh window (untimed): every counter is new again
            a.record()
            eng.rx_check(d, dpt, st, flags)
            b.record()
            torch.cuda.synchronize()
            tot += a.elapsed_time(b)
        out[name + "_us"] = round(tot / reps * 1e3, 2)
        out[name + "_status_hist"] = np.bincount(st.cpu().numpy(), minlength=7).tolist()
    # the replay window over 1024 key slots (64 packets per slot, slot = i mod 1024)
    eng2 = W.Engine(0, key_slots=1024)
    d2 = torch.from_numpy(W.desc_as_int64(W.pack_desc(np.arange(n) * S, np.arange(n) * S, np.arange(n) // 1024, L,
                                                      np.arange(n) % 1024))).to(dev)
    eng2.replay_enable(8192)
    for _ in range(10):
        st.copy_(st0)
        eng2.rx_check(d2, dpt, st, 2)
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(200):
        st.copy_(st0)
        eng2.replay_enable(8192)
        a.record()
        eng2.rx_check(d2, dpt, st, 2)
        b.record()
        torch.cuda.synchronize()
        tot += a.elapsed_time(b)
    out["replay_1024_slots_us"] = round(tot / 200 * 1e3, 2)
    out["replay_1024_slots_status_hist"] = np.bincount(st.cpu().numpy(), minlength=7).tolist()
    print(json.dumps(out))
    eng2.close()
    eng.close()


if __name__ == "__main__":
    main()
