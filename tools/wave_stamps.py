"""Per-wave timeline of k_stream from the diagnostic library (make diag):
wave start/end (s_memrealtime, 100 MHz) and cycles per phase (s_memtime).
Run: WG_LIB_PATH=wireguard-java_amd/libwgaead_diag.so N=65536 python tools/wave_stamps.py"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

torch.cuda.is_available()  # torch's HIP runtime first (tests/conftest.py)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
wg = importlib.import_module("wireguard-java_amd")
E = importlib.import_module("wireguard-java_amd.engine")
lib = wg.lib()
lib.wg_diag_stamps.argtypes = [ctypes.c_void_p]
n, L, S = int(os.environ.get("N", 65536)), int(os.environ.get("L", 1420)), 1440
NK = int(os.environ.get("NKEYS", 1))
eng = wg.Engine(0, key_slots=max(NK, 4))
eng.set_keys(0, bytes(range(32)) * max(NK, 4))
dev = torch.device("cuda", 0)
off = np.arange(n, dtype=np.uint64) * S
tdesc = torch.from_numpy(E.desc_as_int64(wg.pack_desc(off, off, np.arange(n, dtype=np.uint64), np.full(n, L), np.arange(n) % NK))).to(dev)
buf = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=dev)
out = torch.zeros_like(buf)
waves = (n + 7) // 8
stamps = torch.zeros(8 * waves, dtype=torch.int64, device=dev)
fn = lambda: eng.seal(tdesc, buf, out, L, uniform=True)
for _ in range(3):
    fn()
torch.cuda.synchronize()
lib.wg_diag_stamps(stamps.data_ptr())
fn()
torch.cuda.synchronize()
lib.wg_diag_stamps(None)
s = stamps.view(-1, 8).cpu().numpy()
s = s[s[:, 0] != 0]
t0, t1 = s[:, 0].astype(np.int64), s[:, 1].astype(np.int64)
base = t0.min()
st, en = (t0 - base) * 10 / 1e3, (t1 - base) * 10 / 1e3  # us
life = en - st
ph = s[:, 2:6].astype(np.float64)
tot = ph.sum(1)
print(f"N={n} waves={len(s)} kernel span {en.max():.1f} us; wave life mean {life.mean():.1f} p10 {np.percentile(life,10):.1f} "
      f"p90 {np.percentile(life,90):.1f} us")
print("  start-time percentiles (us): " + " ".join(f"p{p}={np.percentile(st,p):.1f}" for p in (0, 10, 25, 50, 75, 90, 100)))
print("  end-time percentiles (us):   " + " ".join(f"p{p}={np.percentile(en,p):.1f}" for p in (0, 10, 25, 50, 75, 90, 100)))
names = ["pkt-start", "chacha", "poly", "finish"]
print("  cycles/wave: " + "  ".join(f"{nm} {ph[:, i].mean():.0f} ({ph[:, i].mean() / tot.mean() * 100:.0f}%)" for i, nm in enumerate(names))
      + f"  total {tot.mean():.0f}; clock {tot.mean() / (life.mean() * 1e3):.2f} GHz-equiv")
# concurrency over time (resident waves), 20 buckets
edges = np.linspace(0, en.max(), 21)
conc = [((st <= m) & (en > m)).sum() for m in (edges[:-1] + edges[1:]) / 2]
print("  resident waves over time:", conc)
# where did the waves run: (XCC, SE, CU, SIMD) from HW_ID / XCC_ID
hw, xcc = s[:, 6].astype(np.int64), s[:, 7].astype(np.int64) & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
u, inv = np.unique(key, return_inverse=True)
per = np.bincount(inv)
first = np.array([(st[inv == i] < 1.0).sum() for i in range(len(u))])
last_end = np.array([en[inv == i].max() for i in range(len(u))])
busy = np.array([life[inv == i].sum() for i in range(len(u))])
print(f"  SIMDs used {len(u)}; waves per SIMD min/mean/max {per.min()}/{per.mean():.1f}/{per.max()}; "
      f"started in first 1us per SIMD min/mean/max {first.min()}/{first.mean():.1f}/{first.max()}")
print(f"  per-SIMD last wave end (us) p0/p10/p50/p90/p100: "
      + "/".join(f"{np.percentile(last_end, p):.1f}" for p in (0, 10, 50, 90, 100)))
cus = np.unique(key // 4)
print(f"  CUs used {len(cus)}; XCCs {np.unique(xcc).tolist()}; waves per XCC {np.bincount(xcc, minlength=8).tolist()}")
