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


def _cgroup(tmp_path, quota_cpus):
    """A cgroup v2 root whose cpu.max allows `quota_cpus` CPUs of time (None: no quota)."""
    root = tmp_path / f"cg{quota_cpus}"
    root.mkdir()
    (root / "cpu.max").write_text("max 100000\n" if quota_cpus is None else f"{quota_cpus * 100000} 100000\n")
    return str(root)


def test_host_cpus_follows_quota_and_affinity(tmp_path, monkeypatch):
    """cpu_baseline's thread count: the affinity mask capped by the cgroup quota, with
    the binding limit named, instead of a fixed cap of 16."""
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(64)))
    assert bench.host_cpus(_cgroup(tmp_path, 8)) == (8, "quota")
    assert bench.host_cpus(_cgroup(tmp_path, 32)) == (32, "quota")
    assert bench.host_cpus(_cgroup(tmp_path, None)) == (64, "affinity")
    assert bench.host_cpus(_cgroup(tmp_path, 128)) == (64, "affinity")   # quota above the affinity
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("1200000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.host_cpus(str(v1)) == (12, "quota")
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(4)))
    assert bench.host_cpus(str(v1)) == (4, "affinity")                   # affinity below the quota


def test_cpu_baseline_cores_follow_quota(tmp_path, monkeypatch):
    """The reported `cores` is the number of threads the timing actually used."""
    used = []
    from oracle import oracle as O
    real = O.seal_batch

    def spy(desc, inp, out, keys, threads=1):
        used.append(threads)
        return real(desc, inp, out, keys, threads=threads)

    monkeypatch.setattr(O, "seal_batch", spy)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(64)))
    L = np.full(64, 1420, np.int64)
    keys = bench.splitmix_np(7, 32)
    for q in (8, 32):
        used.clear()
        cb = bench.cpu_baseline(L, np.zeros(64, np.int64), np.arange(64, dtype=np.uint64), keys, budget_s=0.02,
                                cgroup_root=_cgroup(tmp_path, q))
        assert cb["cores"] == q and cb["cores_source"] == "quota"
        assert used[0] == q and used[-1] == 1          # the multi-thread run, then the single-thread one
