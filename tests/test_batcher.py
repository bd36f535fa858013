"""Per-packet wg_seal1 / wg_open1 through the persistent per-packet server k_pp (SURVEY §8f
rank 1, realised under the unchanged per-packet API): many threads call concurrently, as the
reference's ForkJoinPool workers call SymmetricKeypair.cipher / decipher
(TransportManager.java:41,79,152-158); one resident kernel serves all of them without a launch
per packet, and every result is bit-exact vs the oracle."""
import threading
import time

import numpy as np
import pytest

from wgtest import oracle, splitmix_bytes, splitmix_np, wg

O = oracle()


@pytest.mark.gpu
def test_sixteen_threads_mixed_seal_open_bit_exact():
    W = wg()
    eng = W.Engine(0, key_slots=64)
    try:
        keys = splitmix_np(1601, 32 * 64)
        eng.set_keys(0, keys.tobytes())
        T, N = 16, 2000
        errors = []

        def worker(t):
            try:
                rng = np.random.default_rng(t)
                for i in range(N):
                    L = int(rng.integers(0, 1500)) if i % 5 else 1420
                    slot = int(rng.integers(0, 64))
                    ctr = (t << 32) | i
                    key = keys[32 * slot:32 * slot + 32].tobytes()
                    pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                    if i % 2 == 0:
                        got = eng.seal1(slot, ctr, pt)
                        assert got == O.c_aead_seal(key, O.transport_nonce(ctr), pt), (t, i, L)
                    else:
                        sealed = bytearray(O.c_aead_seal(key, O.transport_nonce(ctr), pt))
                        forged = i % 7 == 1
                        if forged:
                            sealed[L] ^= 0x20
                        got = eng.open1(slot, ctr, bytes(sealed))
                        assert got == (None if forged else pt), (t, i, L, forged)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:3]
        launches, packets = eng.batcher_stats()
        assert packets == T * N
        assert launches < packets  # one resident kernel served many packets
    finally:
        eng.close()


@pytest.mark.gpu
def test_keypair_api_through_batcher_with_window():
    """SymmetricKeypair.cipher / decipher (the unchanged reference API) on two threads with a
    4-wave server that goes idle after 200 us (so it exits and is relaunched between bursts);
    counters are claimed atomically (getAndAdd, :64)."""
    n = __import__("wgtest").noise()
    W = wg()
    eng = W.Engine(0, key_slots=8)
    try:
        eng.batcher_config(waves=4, idle_us=200)
        k1, k2 = splitmix_bytes(1701, 32), splitmix_bytes(1702, 32)
        a = n.SymmetricKeypair(k1, k2, engine=eng)
        b = n.SymmetricKeypair(k2, k1, engine=eng)
        used = []
        lock = threading.Lock()

        def send(t):
            for i in range(300):
                pt = splitmix_bytes(t * 1000 + i, (i * 37) % 1500)
                dst = bytearray(len(pt) + 16)
                c = a.cipher(pt, dst)
                out = bytearray(len(pt))
                b.decipher(c, bytes(dst), out)
                assert bytes(out) == pt
                assert bytes(dst) == O.c_aead_seal(k1, O.transport_nonce(c), pt)
                with lock:
                    used.append(c)
                if i % 50 == 49:
                    time.sleep(0.002)  # let the server go idle and exit

        th = [threading.Thread(target=send, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert sorted(used) == list(range(600))
        a.clean(); b.clean()
    finally:
        eng.close()


@pytest.mark.gpu
def test_per_packet_edges_bit_exact():
    """Keepalive (0 B), the largest slot packet (4080 B), packets past a slot (4081, 9000,
    65535 B: the host batch path), a key change and wg_keys_zero between calls, and a forged
    tag that must leave the caller's buffer untouched (ChaCha20Poly1305.java:51-55)."""
    import ctypes
    W = wg()
    eng = W.Engine(0, key_slots=4)
    try:
        keys = splitmix_np(1801, 32 * 4)
        eng.set_keys(0, keys.tobytes())
        for L in (0, 1, 15, 16, 17, 63, 64, 65, 1420, 2032, 4080, 4081, 9000, 65535):
            for slot in (0, 3):
                key = keys[32 * slot:32 * slot + 32].tobytes()
                ctr = (L << 20) | slot
                pt = splitmix_bytes(L * 7 + slot, L)
                want = O.c_aead_seal(key, O.transport_nonce(ctr), pt)
                assert eng.seal1(slot, ctr, pt) == want, L
                assert eng.open1(slot, ctr, want) == pt, L
        # rekey slot 1, then zero it: the next calls use the new / zero key
        k_new = splitmix_bytes(1802, 32)
        eng.set_keys(1, k_new)
        pt = splitmix_bytes(1803, 700)
        assert eng.seal1(1, 5, pt) == O.c_aead_seal(k_new, O.transport_nonce(5), pt)
        eng.zero_keys(1, 1)
        assert eng.seal1(1, 6, pt) == O.c_aead_seal(bytes(32), O.transport_nonce(6), pt)
        # forged tag: return 1, dst untouched
        lib = W.lib()
        for L in (100, 5000):
            key = keys[:32].tobytes()
            sealed = bytearray(O.c_aead_seal(key, O.transport_nonce(9), splitmix_bytes(L, L)))
            sealed[L + 3] ^= 1
            src = (ctypes.c_uint8 * len(sealed)).from_buffer_copy(bytes(sealed))
            dst = (ctypes.c_uint8 * L)(*([0xA5] * L))
            assert lib.wg_open1(eng.ctx, 0, 9, src, L, dst) == 1
            assert bytes(dst) == b"\xa5" * L
    finally:
        eng.close()


@pytest.mark.gpu
def test_new_context_while_another_server_runs():
    """A context created while another context's per-packet server is resident: its key table
    is zeroed on its own stream, so the first wg_keys_set is not overwritten by a late
    zero-fill (found on the box: every tag of the first batch came from the all-zero key).
    Also reports how long a batch launch takes while the server is resident."""
    import torch
    W = wg()
    a = W.Engine(0, key_slots=2)
    b = None
    try:
        a.batcher_config(waves=4, idle_us=300000)  # keep the server resident for the whole test
        ka = splitmix_bytes(1950, 32)
        a.set_keys(0, ka)
        pt = splitmix_bytes(1951, 100)
        assert a.seal1(0, 1, pt) == O.c_aead_seal(ka, O.transport_nonce(1), pt)
        b = W.Engine(0, key_slots=8)
        keys = splitmix_np(1952, 32 * 3)
        b.set_keys(0, keys.tobytes())
        n = 300
        dev = torch.device("cuda", 0)
        off = np.arange(n, dtype=np.uint64) * 32
        desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64) + 7, np.zeros(n, np.int64), np.arange(n) % 3)
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        inp = torch.zeros(32 * n, dtype=torch.uint8, device=dev)
        out = torch.zeros(32 * n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.seal(d, inp, out, 0, uniform=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        got = out.cpu().numpy()
        for i in range(n):
            k = keys[32 * (i % 3):32 * (i % 3) + 32].tobytes()
            assert got[32 * i:32 * i + 16].tobytes() == O.c_aead_seal(k, O.transport_nonce(i + 7), b""), i
        print(f"batch seal while another context's server is resident: {dt * 1e3:.2f} ms")
        assert a.seal1(0, 2, pt) == O.c_aead_seal(ka, O.transport_nonce(2), pt)
    finally:
        if b is not None:
            b.close()
        a.close()


@pytest.mark.gpu
def test_failed_server_launch_is_not_sticky(monkeypatch):
    """A failed launch of the per-packet server fails only the call that hit it; the next
    call launches again and succeeds (test hook WG_PP_TEST_FAIL_LAUNCHES)."""
    monkeypatch.setenv("WG_PP_TEST_FAIL_LAUNCHES", "1")
    W = wg()
    eng = W.Engine(0, key_slots=1)
    try:
        key = splitmix_bytes(1901, 32)
        eng.set_keys(0, key)
        pt = splitmix_bytes(1902, 300)
        with pytest.raises(W.WgError):
            eng.seal1(0, 1, pt)
        assert eng.seal1(0, 2, pt) == O.c_aead_seal(key, O.transport_nonce(2), pt)
        assert eng.seal1(0, 3, pt) == O.c_aead_seal(key, O.transport_nonce(3), pt)
    finally:
        eng.close()


def test_batcher_entry_points_reject_bad_arguments():
    W = wg()
    lib = W.lib()
    E = W._lib.WG_EINVAL
    assert lib.wg_seal1(None, 0, 0, None, 0, None) == E
    assert lib.wg_open1(None, 0, 0, None, 0, None) == E
    assert lib.wg_batcher_config(None, 16, 0) == E
    assert lib.wg_batcher_stats(None, None, None) == E
