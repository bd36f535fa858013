"""Ablation timings on the GPU: ChaCha-only (CIPHER), Poly-only (MAC), full SEAL/OPEN,
all over 65536 x 1420 B device-resident packets. Prints µs per launch."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
wg = importlib.import_module("wireguard-java_amd")
E = importlib.import_module("wireguard-java_amd.engine")
n, L, S = int(os.environ.get("N", 65536)), int(os.environ.get("L", 1420)), 1440
NK = int(os.environ.get("NKEYS", 1))
eng = wg.Engine(0, key_slots=max(NK, 4))
eng.set_keys(0, np.random.default_rng(1).integers(0, 256, 32 * max(NK, 4), dtype=np.uint8).tobytes())
dev = torch.device("cuda", 0)
off = np.arange(n, dtype=np.uint64) * S
tdesc = torch.from_numpy(E.desc_as_int64(wg.pack_desc(off, off, np.arange(n, dtype=np.uint64), np.full(n, L),
                                                      np.arange(n) % NK))).to(dev)
g = np.zeros(n, E.WG_AEAD_DTYPE)
g["in_off"] = g["out_off"] = off
g["len"] = L
g["nonce"][:, 0] = np.arange(n)
gdesc = torch.from_numpy(E.desc_as_int64(g)).to(dev)
mdesc_np = g.copy(); mdesc_np["out_off"] = np.arange(n, dtype=np.uint64) * 16
mdesc = torch.from_numpy(E.desc_as_int64(mdesc_np)).to(dev)
buf = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=dev)
out = torch.zeros_like(buf)
st = torch.zeros(n, dtype=torch.int32, device=dev)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


if os.environ.get("ABLATE") == "transport":
    for name, fn in [("seal", lambda: eng.seal(tdesc, buf, out, L, uniform=True)),
                     ("open", lambda: eng.open(tdesc, out, buf, st, L, uniform=True))]:
        print(f"{name:32s} {t(fn, 5):9.2f} us")
    sys.exit(0)

res = {
    "seal(transport,uniform)": t(lambda: eng.seal(tdesc, buf, out, L, uniform=True)),
    "open(transport,uniform)": t(lambda: eng.open(tdesc, out, buf, st, L, uniform=True)),
    "seal(transport,plan)": t(lambda: eng.seal(tdesc, buf, out, L, uniform=False)),
    "seal(general)": t(lambda: eng.aead(0, gdesc, buf, None, out, None, L)),
    "cipher(general) chacha-only": t(lambda: eng.aead(2, gdesc, buf, None, out, None, L)),
    "mac(general) poly-only": t(lambda: eng.aead(3, mdesc, buf, None, out, None, L)),
}
for k, v in res.items():
    print(f"{k:32s} {v:9.2f} us")
