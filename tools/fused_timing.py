"""Where the time of one k_step_mixed_fused launch goes (diagnostic library: make -C wireguard-java_amd/csrc diag).

Runs the IMIX step (bench.py --workload imix, one stream) through the diagnostic build, whose fused kernel stamps
s_memrealtime (100 MHz) per workgroup: a planner's start and publication, a consumer's arrival, release from
its wait and end. Prints, for the last of --reps launches, in microseconds from the first workgroup's start:
the planners' first start / last publication, the consumers' first / last arrival and first / last release,
and the last end. The build's per-wave phase stamps cost cycles: read the planning and wait figures, not the
total."""
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

OFF = 400000  # kFusedStampOff (wg_transport.hip)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch

    import bench
    torch.cuda.is_available()
    wg = importlib.import_module("wireguard-java_amd")
    lib = wg.lib()
    lib.wg_diag_stamps.argtypes = [ctypes.c_void_p]
    lengths, slots, counters, nkeys, _, uniform = bench.build_workload("imix", 0, 1)
    n = len(lengths)
    dev = torch.device("cuda", 0)
    eng = wg.Engine(0, key_slots=max(nkeys, 1))
    eng.set_keys(0, bench.splitmix_np(0xC0FFEE, 32 * nkeys).tobytes())
    S = ((lengths + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    d = torch.from_numpy(wg.desc_as_int64(wg.pack_desc(off, off, counters, lengths, slots))).to(dev)
    total = int(S.sum())
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    ct = torch.zeros_like(pt)
    back = torch.zeros_like(pt)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    ml = int(lengths.max())
    stamps = torch.zeros(OFF + 3 * 8192, dtype=torch.int64, device=dev)
    lib.wg_diag_stamps(ctypes.c_void_p(stamps.data_ptr()))
    step = eng.prepare_duplex(d, pt, ct, ml, d, ct, back, st, ml, uniform=uniform, after_seal=True,
                              stream=torch.cuda.current_stream().cuda_stream)
    for _ in range(args.reps):
        step()
    torch.cuda.synchronize()
    ok = int(st.abs().sum()) == 0  # every packet opened (statuses 0)
    s = stamps[OFF:].view(-1, 3).cpu().numpy().astype(np.int64)
    np_ = max(1, min(64, (n + 1023) // 1024))
    if int(os.environ.get("WG_FUSED_NP", "0")):
        np_ = min(int(os.environ["WG_FUSED_NP"]), max(1, n // 256))
    used = s[:, 0] > 0
    t0 = s[used, 0].min()
    pl, co = s[:np_], s[np_:][used[np_:]]
    us = lambda v: round(float(v - t0) / 100.0, 2)  # noqa: E731  100 MHz ticks -> us
    out = {"poll": int(os.environ.get("WG_FUSED_POLL", "0")), "packets": n, "planners": np_, "consumers_stamped": int(len(co)), "verified": ok,
           "planner_first_start_us": us(pl[:, 0].min()), "planner_last_start_us": us(pl[:, 0].max()),
           "planner_last_publish_us": us(pl[:, 1].max()),
           "planner_mean_span_us": round(float((pl[:, 1] - pl[:, 0]).mean()) / 100.0, 2),
           "consumer_first_arrival_us": us(co[:, 0].min()), "consumer_last_arrival_us": us(co[:, 0].max()),
           "consumer_first_release_us": us(co[:, 1].min()), "consumer_last_release_us": us(co[:, 1].max()),
           "last_end_us": us(co[:, 2].max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
