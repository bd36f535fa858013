"""Per-packet wg_seal1 / wg_open1 through the batcher (realised under the
unchanged per-packet API): many threads call concurrently, as the reference's ForkJoinPool
workers call SymmetricKeypair.cipher / decipher (TransportManager.java:41,79,152-158);
their packets share device launches, and every result is bit-exact vs the oracle."""
import threading

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
        assert launches < packets  # concurrent callers shared launches
    finally:
        eng.close()


@pytest.mark.gpu
def test_keypair_api_through_batcher_with_window():
    """SymmetricKeypair.cipher / decipher (the unchanged reference API) on two threads with
    an accumulation window configured; counters are claimed atomically (getAndAdd, :64)."""
    n = __import__("wgtest").noise()
    W = wg()
    eng = W.Engine(0, key_slots=8)
    try:
        eng.batcher_config(max_batch=256, window_us=50)
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

        th = [threading.Thread(target=send, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert sorted(used) == list(range(600))
        a.clean(); b.clean()
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
