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
        eng.pp_config(waves=4, idle_us=200)
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
        # clean(): the next call is refused, never sealed under the all-zero key (the
        # reference's cipher() throws once the key arena is closed, SymmetricKeypair.java:85-93)
        for fn, data in ((eng.seal1, pt), (eng.open1, pt + bytes(16))):
            for big in (False, True):  # a ring slot, and the host batch path past it
                with pytest.raises(W.WgError) as ei:
                    fn(1, 6, data if not big else data * 8)
                assert ei.value.code == W._lib.WG_ENOKEY
        eng.set_keys(1, k_new)
        assert eng.seal1(1, 6, pt) == O.c_aead_seal(k_new, O.transport_nonce(6), pt)
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
def test_per_packet_random_lengths_bit_exact():
    """400 calls of random length 0..4080 in random order from two threads (a unit reads the whole slot
    at once after a packet past 1,984 B, and its first 2 KB otherwise: every switch between the two,
    both ways, and the second round trip), seal against the oracle and open back, every 7th open
    with a forged tag that must leave the buffer untouched. Reference: ChaCha20Poly1305.java:31-60."""
    import ctypes
    W = wg()
    eng = W.Engine(0, key_slots=2)
    errors = []
    try:
        keys = splitmix_np(1901, 64)
        eng.set_keys(0, keys.tobytes())
        lib = W.lib()

        def caller(t):
            try:
                rng = np.random.default_rng(190 + t)
                for i in range(200):
                    L = int(rng.choice([int(rng.integers(0, 4081)), int(rng.integers(1900, 2100)),
                                        int(rng.integers(0, 64))]))
                    slot = i % 2
                    key = keys[32 * slot:32 * slot + 32].tobytes()
                    ctr = (t << 40) | i
                    pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                    want = O.c_aead_seal(key, O.transport_nonce(ctr), pt)
                    got = eng.seal1(slot, ctr, pt)
                    assert got == want, (t, i, L)
                    if i % 7 == 3:
                        bad = bytearray(want)
                        bad[L + (i % 16)] ^= 0x10
                        src = (ctypes.c_uint8 * len(bad)).from_buffer_copy(bytes(bad))
                        dst = (ctypes.c_uint8 * max(L, 1))(*([0x5C] * max(L, 1)))
                        assert lib.wg_open1(eng.ctx, slot, ctr, src, L, dst) == 1, (t, i, L)
                        assert bytes(dst) == b"\x5c" * max(L, 1), (t, i, L)
                    else:
                        assert eng.open1(slot, ctr, want) == pt, (t, i, L)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=caller, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not errors, errors[:3]
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
        a.pp_config(waves=4, idle_us=300000)  # keep the server resident for the whole test
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
    """A failed launch of the per-packet server fails only the call that hit it (test hook
    WG_PP_TEST_FAIL_LAUNCHES). That call's ring entry was already published: it is left to the
    next server, which completes it, and is then reused, so no entry is lost. 1,200 further calls
    from 4 threads (more than twice the 512-entry ring) all succeed, bit-exact."""
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
        errors = []

        def worker(t):
            try:
                for i in range(300):
                    ctr = (t + 1) << 20 | i
                    p = pt[:(i * 13) % 300]
                    if eng.seal1(0, ctr, p) != O.c_aead_seal(key, O.transport_nonce(ctr), p):
                        errors.append((t, i))
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:3]
    finally:
        eng.close()


def _batcher_bench(*args, timeout=120):
    """tools/batcher_bench (C callers over libwgaead, built by __graft_entry__.build()): one JSON line."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "batcher_bench")
    assert os.path.exists(exe), "tools/batcher_bench is built by __graft_entry__.build()"
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [1, 4, 8, 16, 64])
def test_every_wave_count_serves_every_entry(waves):
    """wg_pp_config with each power-of-two wave count (a wave owns 512 / waves ring entries: 512 in
    8 doorbell words down to 8 in a sub-word) and a 200-us idle timeout (the server leaves and is
    relaunched between bursts): 4 threads x 600 calls reach every entry, including doorbell bits
    31 and 32 (a sign-extension bug in the 64-bit doorbell handling once lost every entry past
    bit 31 of a wave's word)."""
    j = _batcher_bench(4, 600, 0, f"waves={waves}", "idle_us=200")
    assert j["failures"] == 0 and j["calls"] == 2400, j


@pytest.mark.gpu
def test_held_caller_delays_nobody():
    """One caller is held 50 ms between claiming its ring entry and publishing it (a caller
    descheduled mid-call, test hook WG_PP_TEST_HOLD_*) while 16 others run: with out-of-order
    service nobody waits for it (the round-3 in-order ticket server stalled every later ticket of
    its wave for the whole 50 ms)."""
    j = _batcher_bench(16, 2000, 1420, "hold_us=50000", "stamps=1")
    print(j)
    assert j["failures"] == 0 and j["held_rc"] == 0
    assert j["held_us"] >= 50000
    assert j["lat_us"]["p999"] < 2000, j["lat_us"]
    # The single slowest of the 32,000 calls, with its stages (wg_pp_last_call) and the caller thread's
    # context switches. Waiting for the held entry would add 50 ms, so the slowest call must stay far
    # below that. It usually stays under 2 ms (the device serves a call in ~8 us; round 5 traced every
    # 0.2-ms outlier to an OS preemption of the caller), but one round-6 box stalled the
    # device itself for 3.75 ms under 16 concurrent calls (device_service_us 3754.8, no preemption, no
    # throttling): a device-wide pause, not a wait for the held entry, so the bound is 10 ms.
    slow = j["slowest"]
    assert j["lat_us"]["max"] < 10000, (j["lat_us"], slow, j["throttled_periods"])


@pytest.mark.gpu
def test_refused_launch_loses_no_entry_under_load():
    """The same failure through the C callers: the warm-up call's launch is refused, then 4
    threads x 300 calls (1,200, > 2 x 512 entries) all succeed."""
    j = _batcher_bench(4, 300, 1420, "fail_launches=1")
    assert j["failures"] == 0 and j["calls"] == 1200


@pytest.mark.gpu
def test_low_call_rate_latency():
    """A quiet tunnel: one call every 2 ms keeps the server resident (the whole server leaves
    only after 20 ms without work anywhere, so no call lands on a wave that has already left:
    round 3 stranded about every 16th call for up to 20 ms); and with a 1-ms idle timeout every
    call relaunches the server, which must cost a launch, not an idle period."""
    j = _batcher_bench(1, 300, 1420, "gap_us=2000")
    print(j)
    assert j["failures"] == 0
    assert j["lat_us"]["p99"] < 500, j["lat_us"]
    assert j["launches"] <= 5  # a launch lives at most 250 ms
    j = _batcher_bench(1, 100, 1420, "gap_us=3000", "idle_us=1000")
    print(j)
    assert j["failures"] == 0
    assert j["lat_us"]["p99"] < 3000, j["lat_us"]


def test_batcher_entry_points_reject_bad_arguments():
    W = wg()
    lib = W.lib()
    E = W._lib.WG_EINVAL
    assert lib.wg_seal1(None, 0, 0, None, 0, None) == E
    assert lib.wg_open1(None, 0, 0, None, 0, None) == E
    assert lib.wg_batcher_config(None, 16, 0) == E
    assert lib.wg_pp_config(None, 16, 0) == E
    assert lib.wg_batcher_stats(None, None, None) == E


@pytest.mark.gpu
@pytest.mark.parametrize("callers", [64, 128])
def test_more_callers_than_cpus_tail_latency(callers):
    """More synchronous callers than the CPUs the process may use (the GPU box: 16 CPUs of cgroup
    quota): only that many poll for their completion, the rest sleep on a futex, so the process
    never exhausts its quota and no call waits out a throttled period (polling callers had p999
    74 / 88 ms at 64 / 128)."""
    j = _batcher_bench(callers, 160000 // callers, 1420)
    print(j)
    assert j["failures"] == 0
    assert j["lat_us"]["p999"] < 2000, (j["lat_us"], j["throttled_periods"])
