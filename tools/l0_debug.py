"""Debug: L=0 uniform seal vs the oracle (which packets differ). Diagnostic only."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_gpu_parity import make_batch, run_device, O, wg
from wgtest import noise, splitmix_bytes
if os.environ.get("L0_PP", "1") == "1":  # start the per-packet server of the default engine first
    n_ = noise()
    a = n_.SymmetricKeypair(splitmix_bytes(11, 32), splitmix_bytes(12, 32))
    dst = bytearray(16 + 20)
    a.cipher(bytes(20), dst)
    a.clean()
eng = wg().Engine(0, key_slots=4096)
for L in (0, 1, 0):
    for uni in (True, False, True):
        n = 300
        desc, keys, inp, out_size = make_batch(n, [L] * n, 3, seed=L + 17)
        sealed, _ = run_device(eng, torch, desc, keys, inp, out_size, uniform=uni)
        ref = np.zeros(out_size, np.uint8)
        O.seal_batch(desc, inp, ref, keys, threads=8)
        bad = [i for i in range(n) if not np.array_equal(sealed[desc["out_off"][i]:desc["out_off"][i] + L + 16],
                                                        ref[desc["out_off"][i]:desc["out_off"][i] + L + 16])]
        print("L", L, "uniform", uni, "bad", len(bad), bad[:12], flush=True)
        for i in bad[:3]:
            o = int(desc["out_off"][i])
            print("   pkt", i, "key", int(desc["key_slot"][i]), "dev", sealed[o:o + L + 16].tobytes().hex(), "ref", ref[o:o + L + 16].tobytes().hex())
