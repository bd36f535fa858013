"""Asynchronous batch submission (wg_queue): producers submit packets and return
at once, one dispatcher thread per queue batches them into k_transport launches over a pinned ring,
and the consumer reaps completions. The batching replacement for TransportManager's per-packet
ForkJoinPool submission (TransportManager.java:41,70-93,137-158; EstablishedSession.java:88-90).

-m gpu: every sealed packet against the oracle (oracle/liboracle.so), every opened plaintext against
the input, forged tags refused; the C producers/consumers harness (tools/queue_bench) bit-checks a
longer run. Without a GPU: the argument contract."""
import json
import os
import subprocess
import threading
import time

import numpy as np
import pytest

from wgtest import oracle, splitmix_bytes, splitmix_np, wg

O = oracle()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_queue_seal_then_open_bit_exact():
    W = wg()
    eng = W.Engine(0, key_slots=16)
    qs = qo = None
    try:
        keys = splitmix_np(2101, 32 * 16)
        eng.set_keys(0, keys.tobytes())
        qs, qo = eng.queue("seal", capacity=4096), eng.queue("open", capacity=4096)
        T, N = 4, 3000
        sent = {}
        errors = []
        lock = threading.Lock()

        def producer(t):
            try:
                rng = np.random.default_rng(t)
                for i in range(N):
                    L = int(rng.integers(0, 2033)) if i % 7 else (0 if i % 2 else 2032)
                    user = (t << 32) | i
                    pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                    with lock:
                        sent[user] = (i % 16, (t << 40) | i, pt)
                    qs.submit(i % 16, (t << 40) | i, pt, user)
            except Exception as e:  # pragma: no cover - reported by the reaping loop
                errors.append(repr(e))

        th = [threading.Thread(target=producer, args=(t,), daemon=True) for t in range(T)]
        for x in th:
            x.start()
        sealed = {}
        deadline = time.monotonic() + 60
        while len(sealed) < T * N:
            assert not errors, errors[:3]
            assert time.monotonic() < deadline, (len(sealed), qs.stats())
            for user, ctr, st, data in qs.reap(4096, 200000):
                assert st == 0, st
                sealed[user] = (ctr, data)
        for x in th:
            x.join()
        assert len(sealed) == T * N
        for user, (slot, ctr, pt) in sent.items():
            key = keys[32 * slot:32 * slot + 32].tobytes()
            assert sealed[user][0] == ctr
            assert sealed[user][1] == O.c_aead_seal(key, O.transport_nonce(ctr), pt), user
        # the peer's side: open every packet, about 2% with a flipped tag bit; the main thread
        # submits (more packets than the queue has slots) while a consumer thread reaps
        forged = set()
        got = {}
        stop = threading.Event()

        def consumer():
            try:
                while not stop.is_set() and len(got) < T * N:
                    for user, ctr, st, data in qo.reap(4096, 20000):
                        got[user] = (st, data)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        rc = threading.Thread(target=consumer, daemon=True)
        rc.start()
        for k, (user, (slot, ctr, pt)) in enumerate(sorted(sent.items())):
            ct = bytearray(sealed[user][1])
            if k % 50 == 7:
                ct[len(pt) + (k % 16)] ^= 0x04
                forged.add(user)
            qo.submit(slot, ctr, bytes(ct), user)
        rc.join(timeout=60)
        stop.set()
        assert not errors, errors[:3]
        assert len(got) == T * N, (len(got), qo.stats())
        for user, (slot, ctr, pt) in sent.items():
            st, data = got[user]
            if user in forged:
                assert st == W._lib.WG_PKT_BADTAG and data is None, user
            else:
                assert st == 0 and data == pt, user
        b, p = qs.stats()
        assert p == T * N and 1 <= b <= p
    finally:
        for q in (qs, qo):
            if q is not None:
                q.close()
        eng.close()


@pytest.mark.gpu
def test_one_producer_uses_the_whole_ring():
    """One producer thread submits 3,000 packets into a 4,096-slot queue before anything is reaped:
    its own lane holds 64 slots (4096 / 64 lanes), so the other 2,936 come from other lanes'
    free rings, 32 at a time through the lane's stash; every sealed packet is then compared with
    the oracle, and the slots go back to their home lanes (a second round fits again)."""
    W = wg()
    eng = W.Engine(0, key_slots=4)
    q = None
    try:
        keys = splitmix_np(2201, 32 * 4)
        eng.set_keys(0, keys.tobytes())
        q = eng.queue("seal", capacity=4096)
        for rnd in range(2):
            sent = {}
            for i in range(3000):
                L = (i * 37 + rnd) % 1500
                pt = splitmix_bytes(rnd * 100000 + i, L)
                sent[i] = (i % 4, (rnd << 32) | i, pt)
                q.submit(i % 4, (rnd << 32) | i, pt, i)
            got = {}
            deadline = time.monotonic() + 30
            while len(got) < 3000:
                assert time.monotonic() < deadline, (len(got), q.stats())
                for user, ctr, st, data in q.reap(4096, 100000):
                    assert st == 0, st
                    got[user] = (ctr, data)
            for i, (slot, ctr, pt) in sent.items():
                key = keys[32 * slot:32 * slot + 32].tobytes()
                assert got[i][0] == ctr
                assert got[i][1] == O.c_aead_seal(key, O.transport_nonce(ctr), pt), (rnd, i)
    finally:
        if q is not None:
            q.close()
        eng.close()


@pytest.mark.gpu
def test_queue_c_harness_transport_manager_shape():
    """tools/queue_bench: 16 producer threads submit 1420-B packets to a seal queue, a forwarder
    reaps them and submits each ct || tag to an open queue (one by one, or per reap with
    wg_submit_open_n), a verifier checks every status and byte of the plaintexts (the reference's FJP
    workers -> UDP worker -> peer -> tun writer)."""
    exe = os.path.join(ROOT, "tools", "queue_bench")
    assert os.path.exists(exe), "tools/queue_bench is built by __graft_entry__.build()"
    # the last two: two forwarders and two verifiers, each forwarder handing a whole reap to the open
    # queue in one wg_submit_open_n (fwd_batch=1)
    for args in (["16", "20000", "1420"], ["4", "20000", "0"], ["16", "20000", "0", "8192", "2", "2", "fwd_batch=1"],
                 ["8", "20000", "1420", "8192", "1", "1", "fwd_batch=1"]):
        r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
        j = json.loads(r.stdout.strip().splitlines()[-1])
        print(j)
        assert j["bad"] == 0 and j["packets"] == int(args[0]) * int(args[1])


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _reap_all(q, n, timeout_s=30):
    got = {}
    deadline = time.monotonic() + timeout_s
    while len(got) < n:
        assert time.monotonic() < deadline, (len(got), q.stats())
        for user, ctr, st, data in q.reap(4096, 100000):
            got[user] = (ctr, st, data)
    return got


@pytest.mark.gpu
def test_queued_packets_keep_the_key_they_were_submitted_with():
    """A packet queued before wg_keys_zero / wg_keys_set of its key slot is sealed with the key the
    slot held at the submit, never the zero key or the next keypair's (the kernel used to
    read the device key table when the batch launched, so clean() between submit and launch sealed
    packets under an all-zero key). The batching window is stretched to 300 ms (WG_QUEUE_WINDOW_US)
    so every packet is still queued when the key changes. Reference: SymmetricKeypair.java:63-74, 85-93."""
    W = wg()
    eng = W.Engine(0, key_slots=4)
    q = None
    try:
        k_old, k_new = splitmix_bytes(2301, 32), splitmix_bytes(2302, 32)
        eng.set_keys(1, k_old)
        q = _with_env({"WG_QUEUE_WINDOW_US": "300000", "WG_QUEUE_MIN_BATCH": "100000"},
                      lambda: eng.queue("seal", capacity=1024))
        pts = {i: splitmix_bytes(2400 + i, 100 + 13 * i) for i in range(40)}
        for i in range(20):
            q.submit(1, i, pts[i], i)
        eng.zero_keys(1, 1)  # clean(): the queued packets keep k_old
        for i in range(20, 30):
            # submitted after the zeroing: refused (sealing under the all-zero key was fail-open;
            # the reference's cipher() throws once clean() has closed the key arena)
            with pytest.raises(W.WgError) as ei:
                q.submit(1, i, pts[i], i)
            assert ei.value.code == W._lib.WG_ENOKEY
        with pytest.raises(W.WgError) as ei:  # a batched submit with one such entry queues nothing
            q.submit_n([(1, 20, pts[20], 20)])
        assert ei.value.code == W._lib.WG_ENOKEY
        eng.set_keys(1, k_new)
        for i in range(30, 40):
            q.submit(1, i, pts[i], i)
        got = _reap_all(q, 30)
        assert sorted(got) == list(range(20)) + list(range(30, 40))
        for i in got:
            key = k_old if i < 20 else k_new
            ctr, st, data = got[i]
            assert st == 0 and ctr == i
            assert data == O.c_aead_seal(key, O.transport_nonce(i), pts[i]), i
        # every completed batch's key copies are wiped from the pinned ring (they stayed until
        # the queue was freed, so a zeroed session's key outlived clean() in pinned memory)
        assert W.lib().wg_queue_key_residue(q.q) == 0
    finally:
        if q is not None:
            q.close()
        eng.close()


@pytest.mark.gpu
def test_submit_timeout_returns_eagain_when_nobody_reaps():
    """wg_queue_set_submit_timeout: with every slot of a 64-slot queue sealed but not reaped, the next
    submit returns WG_EAGAIN after the timeout instead of waiting for ever (the round-4 hang was a
    caller that submitted more packets than the ring holds before reaping any); after the consumer
    reaps, submits succeed again."""
    W = wg()
    eng = W.Engine(0, key_slots=1)
    q = None
    try:
        eng.set_keys(0, splitmix_bytes(2501, 32))
        q = eng.queue("seal", capacity=64)
        q.set_submit_timeout(5000)
        for i in range(64):
            q.submit(0, i, b"x" * 64, i)
        t0 = time.monotonic()
        with pytest.raises(W.WgError) as ei:
            q.submit(0, 64, b"x" * 64, 64)
        assert ei.value.code == W._lib.WG_EAGAIN
        assert time.monotonic() - t0 < 2.0
        got = _reap_all(q, 64)
        assert all(st == 0 for _, st, _ in got.values())
        q.submit(0, 65, b"y" * 64, 65)
        assert _reap_all(q, 1)[65][1] == 0
    finally:
        if q is not None:
            q.close()
        eng.close()


@pytest.mark.gpu
def test_queue_beside_batch_calls_with_timing_and_another_kernel():
    """A queue runs while another thread makes wg_seal_batch calls with timing on and the k_tile
    kernel selected (the dispatcher launched without c->mu through whatever kernel the
    context selected, racing the shared plan workspace and the timing-event list). The queue's
    launches are now the transport kernel with their own keys and no timing events: both paths stay
    bit-exact, and the timing list holds exactly the batch calls' launches."""
    import torch
    W = wg()
    eng = W.Engine(0, key_slots=8)
    q = None
    try:
        keys = splitmix_np(2601, 32 * 8)
        eng.set_keys(0, keys.tobytes())
        eng.set_kernel("tile")
        q = eng.queue("seal", capacity=4096)
        errors, sent = [], {}

        def producer():
            try:
                for i in range(6000):
                    pt = splitmix_bytes(2700 + i, (i * 53) % 1500)
                    sent[i] = (i % 8, pt)
                    q.submit(i % 8, i, pt, i)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        got = {}

        def consumer():
            try:
                deadline = time.monotonic() + 60
                while len(got) < 6000 and time.monotonic() < deadline:
                    for user, ctr, st, data in q.reap(4096, 20000):
                        got[user] = (st, data)
            except Exception as e:  # pragma: no cover
                errors.append(repr(e))

        th = [threading.Thread(target=producer, daemon=True), threading.Thread(target=consumer, daemon=True)]
        for t in th:
            t.start()
        dev = torch.device("cuda", 0)
        n, L = 2048, 700
        off = np.arange(n, dtype=np.uint64) * 720
        desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), L, np.arange(n) % 8)
        pt = splitmix_np(2801, n * 720)
        ref = np.zeros_like(pt)
        O.seal_batch(desc, pt, ref, keys, threads=8)
        d_desc = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        d_pt = torch.from_numpy(pt).to(dev)
        eng.timing(True)
        eng.timing_read()
        calls = 0
        while th[0].is_alive() and calls < 400:
            d_ct = torch.zeros_like(d_pt)
            eng.seal(d_desc, d_pt, d_ct, L)
            torch.cuda.synchronize()
            ct = d_ct.cpu().numpy().reshape(n, 720)
            assert np.array_equal(ct[:, :L + 16], ref.reshape(n, 720)[:, :L + 16])
            calls += 1
        for t in th:
            t.join(timeout=60)
        _, launches = eng.timing_read()
        eng.timing(False)
        assert not errors, errors[:3]
        assert launches == calls, (launches, calls)  # k_tile's mixed plan: one timed launch per call
        assert len(got) == 6000
        for i, (slot, p) in sent.items():
            key = keys[32 * slot:32 * slot + 32].tobytes()
            assert got[i][0] == 0 and got[i][1] == O.c_aead_seal(key, O.transport_nonce(i), p), i
    finally:
        if q is not None:
            q.close()
        eng.close()


@pytest.mark.gpu
def test_batched_submits_bit_exact_beside_single_submits():
    """wg_submit_seal_n / wg_submit_open_n: 3 producer threads submit 2,000 packets of 0..1500 B each in
    runs of 1..300 (more than a lane's share of the 1,024-slot ring, so runs span several free-slot
    runs and wait for the consumer), a fourth submits one at a time; every sealed packet matches the
    oracle, then the forwarder shape: reaped completions submitted to an open queue in batches of
    what one wg_reap returned (every 50th with a forged tag: WG_PKT_BADTAG, no data), every other
    plaintext equal to the input."""
    W = wg()
    eng = W.Engine(0, key_slots=8)
    qs = qo = None
    try:
        keys = splitmix_np(2701, 32 * 8)
        eng.set_keys(0, keys.tobytes())
        qs, qo = eng.queue("seal", capacity=1024), eng.queue("open", capacity=1024)
        T, N = 4, 2000
        sent, errors, lock = {}, [], threading.Lock()

        def producer(t):
            try:
                rng = np.random.default_rng(40 + t)
                i = 0
                while i < N:
                    run = 1 if t == 3 else int(rng.integers(1, 301))
                    batch = []
                    for _ in range(min(run, N - i)):
                        L = int(rng.integers(0, 1501))
                        user = (t << 32) | i
                        pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                        with lock:
                            sent[user] = (i % 8, (t << 40) | i, pt)
                        batch.append((i % 8, (t << 40) | i, pt, user))
                        i += 1
                    if t == 3:
                        qs.submit(*batch[0])
                    else:
                        assert qs.submit_n(batch) == len(batch)
            except Exception as e:  # pragma: no cover - reported by the reaping loop
                errors.append(repr(e))

        got, stop = {}, threading.Event()

        def consumer():  # the open queue's reaper (the forwarder below outruns its 1,024 slots)
            try:
                while not stop.is_set() and len(got) < T * N:
                    for user, ctr, st, data in qo.reap(4096, 20000):
                        got[user] = (ctr, st, data)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=producer, args=(t,), daemon=True) for t in range(T)]
        rc = threading.Thread(target=consumer, daemon=True)
        for x in th + [rc]:
            x.start()
        sealed = {}
        deadline = time.monotonic() + 60
        while len(sealed) < T * N:
            assert not errors, errors[:3]
            assert time.monotonic() < deadline, (len(sealed), qs.stats())
            done = qs.reap(4096, 200000)
            for user, ctr, st, data in done:
                assert st == 0, st
                sealed[user] = (ctr, data)
            # forward what this reap returned to the open queue in one call, every 50th with a
            # flipped tag bit
            if done:
                fwd = []
                for u, c, _, d in done:
                    if (u & 0xffffffff) % 50 == 7:
                        d = bytearray(d)
                        d[-1 - (u % 16)] ^= 0x20
                        d = bytes(d)
                    fwd.append((sent[u][0], c, d, u))
                assert qo.submit_n(fwd) == len(done)
        for x in th:
            x.join()
        for user, (slot, ctr, pt) in sent.items():
            key = keys[32 * slot:32 * slot + 32].tobytes()
            assert sealed[user] == (ctr, O.c_aead_seal(key, O.transport_nonce(ctr), pt)), user
        rc.join(timeout=60)
        stop.set()
        assert not errors, errors[:3]
        assert len(got) == T * N, (len(got), qo.stats())
        for user, (slot, ctr, pt) in sent.items():
            if (user & 0xffffffff) % 50 == 7:
                assert got[user] == (ctr, W._lib.WG_PKT_BADTAG, None), user
            else:
                assert got[user] == (ctr, 0, pt), user
    finally:
        for q in (qs, qo):
            if q is not None:
                q.close()
        eng.close()


@pytest.mark.gpu
def test_batched_submit_stops_at_the_timeout_and_checks_every_entry_first():
    """A 64-slot queue nobody reaps: a batch of 100 queues 64 and returns 64 once the 5-ms submit timeout
    runs out; the next batch gets WG_EAGAIN; a batch with one oversized entry queues nothing."""
    W = wg()
    eng = W.Engine(0, key_slots=1)
    q = None
    try:
        eng.set_keys(0, splitmix_bytes(2801, 32))
        q = eng.queue("seal", capacity=64, max_len=256)
        q.set_submit_timeout(5000)
        with pytest.raises(W.WgError) as ei:
            q.submit_n([(0, 0, b"a" * 16, 0), (0, 1, b"b" * 300, 1)])
        assert ei.value.code == W._lib.WG_E2BIG
        t0 = time.monotonic()
        assert q.submit_n([(0, i, bytes([i]) * 32, i) for i in range(100)]) == 64
        assert time.monotonic() - t0 < 2.0
        with pytest.raises(W.WgError) as ei:
            q.submit_n([(0, 100, b"z", 100)])
        assert ei.value.code == W._lib.WG_EAGAIN
        got = _reap_all(q, 64)
        assert sorted(got) == list(range(64)) and all(st == 0 for _, st, _ in got.values())
    finally:
        if q is not None:
            q.close()
        eng.close()


def test_queue_argument_contract():
    W = wg()
    lib = W.lib()
    E = W._lib.WG_EINVAL
    import ctypes
    q = ctypes.c_void_p()
    assert lib.wg_queue_create(None, 0, 0, 0, 0, ctypes.byref(q)) == E
    assert lib.wg_submit_seal(None, 0, 0, None, 0, 0) == E
    assert lib.wg_submit_open(None, 0, 0, None, 0, 0) == E
    assert lib.wg_submit_seal_n(None, None, 0) == E
    assert lib.wg_submit_open_n(None, None, 0) == E
    assert lib.wg_reap(None, None, 0, 0) == E
    assert lib.wg_reap_done(None, None, 0) == E
    assert lib.wg_queue_stats(None, None, None) == E
    assert lib.wg_queue_set_submit_timeout(None, 0) == E
    assert lib.wg_queue_destroy(None) == 0


@pytest.mark.gpu
def test_no_key_left_in_the_ring_after_reap():
    """After a batch completes, its slots' key copies are zeroed: keys_zero followed by a reap leaves no
    key bytes in the queue's pinned key ring (SymmetricKeypair.clean zeroes its keys,
    SymmetricKeypair.java:85-89). A slot that never held a key is refused as well."""
    W = wg()
    eng = W.Engine(0, key_slots=4)
    q = None
    try:
        eng.set_keys(0, splitmix_bytes(2601, 64))
        for mode in ("seal", "open"):
            q = eng.queue(mode, capacity=256)
            extra = 16 if mode == "open" else 0
            for i in range(200):
                q.submit(i % 2, i, splitmix_bytes(2700 + i, 64 + i + extra), i)
            eng.zero_keys(0, 1)
            got = _reap_all(q, 200)
            assert len(got) == 200
            if mode == "seal":
                assert all(st == 0 for _, st, _ in got.values())
            assert W.lib().wg_queue_key_residue(q.q) == 0
            with pytest.raises(W.WgError) as ei:
                q.submit(2, 0, b"x" * (8 + extra), 0)  # never set
            assert ei.value.code == W._lib.WG_ENOKEY
            q.close()
            q = None
            eng.set_keys(0, splitmix_bytes(2602, 32))
    finally:
        if q is not None:
            q.close()
        eng.close()
