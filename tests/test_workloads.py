"""bench.py's workloads as the parity tests rebuild them: sizes, key slots and
per-session counters, and the IMIX mix's ratio (CPU only, no GPU)."""
import numpy as np

import bench


def test_c1_c2_shapes():
    L, slots, ctr, k, _, uniform = bench.build_workload("c1", 0, 1)
    assert uniform and k == 1 and len(L) == 65536 and (L == 1420).all()
    assert np.array_equal(ctr, np.arange(65536, dtype=np.uint64))
    L, slots, ctr, k, _, uniform = bench.build_workload("c2", 0, 1)
    assert not uniform and k == 256 and L.min() >= 64 and L.max() <= 9000
    # every session counts its own packets from 0, as SymmetricKeypair issues them
    for s in (0, 17, 255):
        assert np.array_equal(ctr[slots == s], np.arange(256, dtype=np.uint64))


def test_imix_mix():
    L, slots, ctr, k, desc, uniform = bench.build_workload("imix", 0, 1)
    assert not uniform and k == 256 and len(L) == 65536 and "IMIX" in desc
    sizes, counts = np.unique(L, return_counts=True)
    assert sizes.tolist() == [40, 576, 1500]
    frac = counts / counts.sum()
    assert np.allclose(frac, [7 / 12, 4 / 12, 1 / 12], atol=0.01)
    again = bench.build_workload("imix", 0, 1)[0]
    assert np.array_equal(L, again)                      # seeded: every run times the same batch
    assert not np.array_equal(L, bench.build_workload("imix", 1, 2)[0])  # each rank its own draw
    for s in (0, 255):
        assert np.array_equal(ctr[slots == s], np.arange(256, dtype=np.uint64))
