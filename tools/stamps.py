"""Phase timing of k_tile from the diagnostic library's in-kernel s_memtime stamps.
Run with WG_LIB_PATH=wireguard-java_amd/libwgaead_diag.so. Shares, not absolute speed."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
wg = importlib.import_module("wireguard-java_amd")
E = importlib.import_module("wireguard-java_amd.engine")
lib = wg.lib()
lib.wg_diag_stamps.argtypes = [ctypes.c_void_p]
n, L, S = 65536, int(os.environ.get("L", 1420)), 1440
eng = wg.Engine(0, key_slots=4)
eng.set_keys(0, bytes(range(32)))
dev = torch.device("cuda", 0)
off = np.arange(n, dtype=np.uint64) * S
tdesc = torch.from_numpy(E.desc_as_int64(wg.pack_desc(off, off, np.arange(n, dtype=np.uint64), np.full(n, L), 0))).to(dev)
buf = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=dev)
out = torch.zeros_like(buf)
st = torch.zeros(n, dtype=torch.int32, device=dev)
stamps = torch.zeros(8 * 70000, dtype=torch.int64, device=dev)
for mode in ["seal", "open"]:
    fn = (lambda: eng.seal(tdesc, buf, out, L, uniform=True)) if mode == "seal" else (lambda: eng.open(tdesc, out, buf, st, L, uniform=True))
    lib.wg_diag_stamps(None)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    stamps.zero_()
    lib.wg_diag_stamps(stamps.data_ptr())
    fn()
    torch.cuda.synchronize()
    lib.wg_diag_stamps(None)
    s = stamps.view(-1, 8).cpu().numpy()
    s = s[s[:, 0] != 0]
    t = s[:, :4].astype(np.float64)
    rec, cha, pol = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    real = (s[:, 5] - s[:, 5].min()) * 10.0  # ns (100 MHz)
    print(f"{mode}: tiles={len(s)}  cycles/tile: records {rec.mean():.0f} (p90 {np.percentile(rec,90):.0f})  "
          f"chacha {cha.mean():.0f} (p90 {np.percentile(cha,90):.0f})  poly {pol.mean():.0f} (p90 {np.percentile(pol,90):.0f})  "
          f"total {(t[:,3]-t[:,0]).mean():.0f}")
    print(f"   start spread {real.max()/1e3:.1f} us; tiles started per us (first/last 10us): "
          f"{(real < 10e3).sum()/10:.0f} / {(real > real.max()-10e3).sum()/10:.0f}")
    t0r, t1r = s[:, 5].astype(np.int64), s[:, 4].astype(np.int64)
    hw = s[:, 6]
    cu_key = (s[:, 7] & 0xF) * 1024 + ((hw >> 13) & 0x7) * 64 + ((hw >> 8) & 0xF) * 4 + ((hw >> 6) & 0x3) * 0
    ev = sorted([(a, 1, k) for a, k in zip(t0r, cu_key)] + [(b, -1, k) for b, k in zip(t1r, cu_key)])
    cur, mx = {}, {}
    for tt, d, k in ev:
        cur[k] = cur.get(k, 0) + d
        mx[k] = max(mx.get(k, 0), cur[k])
    print(f"   tile wall (realtime) mean {(t1r-t0r).mean()*10/1e3:.2f} us; CUs seen {len(mx)}; max concurrent tiles/CU "
          f"mean {np.mean(list(mx.values())):.1f} max {max(mx.values())}; kernel span {(t1r.max()-t0r.min())*10/1e3:.1f} us")
    xcc = s[:, 7] & 0xF
    cu = (s[:, 6] >> 8) & 0xF
    se = (s[:, 6] >> 13) & 0x7
    print("   per-XCC tile counts:", np.bincount(xcc.astype(int), minlength=8).tolist())
