"""wg_rx_check on the MI355X against oracle/rx.py (pytest -m gpu): keepalives, IP version /
length, AllowedIPs per key slot (TransportManager.java:98-130, util/IPFilter.java:30-61),
and the replay window over several batches (window state compared word for word)."""
import ipaddress

import numpy as np
import pytest

from oracle import rx
from wgtest import oracle, splitmix_np, wg

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    assert torch.cuda.is_available()
    return torch, torch.device("cuda", 0)


def _random_prefixes(rng, k):
    out = []
    for _ in range(k):
        if rng.random() < 0.6:
            a = ipaddress.IPv4Address(int(rng.integers(0, 1 << 32)))
            p = int(rng.choice([0, 1, 7, 8, 9, 16, 20, 24, 31, 32]))
        else:
            a = ipaddress.IPv6Address(int.from_bytes(rng.bytes(16), "big"))
            p = int(rng.choice([0, 8, 32, 48, 64, 100, 127, 128]))
        out.append((a, p))
    return out


def _packet(rng, prefixes):
    """An IP-ish plaintext: mostly v4/v6 with destinations near the filter's prefixes."""
    kind = rng.random()
    if kind < 0.05:
        return b""
    if kind < 0.10:
        return bytes([int(rng.choice([0x00, 0x50, 0x85, 0xF0]))]) + rng.bytes(int(rng.integers(0, 60)))
    v6 = kind > 0.55
    base, plen = prefixes[int(rng.integers(0, len(prefixes)))] if prefixes else (None, 0)
    nbytes = 16 if v6 else 4
    if base is not None and (base.version == 6) == v6 and rng.random() < 0.7:
        addr = bytearray(base.packed)
        flip = int(rng.integers(max(plen - 3, 0), nbytes * 8)) if rng.random() < 0.5 else None
        if flip is not None:
            addr[flip // 8] ^= 1 << (7 - flip % 8)
        dst = bytes(addr)
    else:
        dst = rng.bytes(nbytes)
    at = 24 if v6 else 16
    total = int(rng.integers(at + nbytes - 2, 200)) if rng.random() < 0.1 else int(rng.integers(at + nbytes, 300))
    p = bytearray(rng.bytes(max(total, 1)))
    p[0] = (0x60 if v6 else 0x45) | (p[0] & 0x0F)
    p[at:at + nbytes] = dst[:max(0, min(nbytes, total - at))] if total >= at else b""
    return bytes(p[:total])


def _run(engine, torch, dev, W, slots, counters, pts, status, flags):
    n = len(pts)
    lens = np.array([len(p) for p in pts], np.int64)
    S = ((lens + 15) // 16) * 16 + 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(S.sum()), np.uint8)
    for i, p in enumerate(pts):
        buf[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    desc = W.pack_desc(off, off, counters, lens, slots)
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    st = torch.from_numpy(np.asarray(status, np.int32)).to(dev)
    engine.rx_check(d, torch.from_numpy(buf).to(dev), st, flags)
    torch.cuda.synchronize()
    return st.cpu().numpy().astype(np.int64).tolist()


def test_filter_parity_random(engine):
    torch, dev = _dev()
    W = wg()
    rng = np.random.default_rng(7)
    nf = 6
    filters = {}
    for f in range(nf):
        pre = _random_prefixes(rng, int(rng.integers(0, 12)))
        if f == 1:
            pre = [(ipaddress.ip_address("0.0.0.0"), 32), (ipaddress.ip_address("::"), 128)]  # allowingAll()
        engine.filter_set(f, pre)
        o = rx.IPFilter()
        for a, p in pre:
            o.insert(a.packed, p)
        filters[f] = (pre, o)
    # slots 0..9: filter f = slot % 6, slot 7 -> no filter, slot 8 -> an id never set
    ids = [s % nf for s in range(10)]
    ids[7] = W._lib.WG_NO_FILTER
    ids[8] = 4242
    engine.slot_filters_set(0, ids)
    n = 20000
    slots = rng.integers(0, 10, n)
    pts = []
    for s in slots:
        f = ids[int(s)]
        pts.append(_packet(rng, filters[f][0] if f in filters else []))
    status = np.where(rng.random(n) < 0.03, 1, 0)
    got = _run(engine, torch, dev, W, slots, np.arange(n), pts, status, W._lib.WG_RX_FILTER)
    of = {s: (filters[ids[s]][1] if ids[s] in filters else (rx.IPFilter() if ids[s] != W._lib.WG_NO_FILTER else None))
          for s in range(10)}
    want = rx.rx_check(slots, np.arange(n), [len(p) for p in pts], pts, status, of, None)
    assert got == want
    kinds = set(want)
    assert {rx.PKT_OK, rx.PKT_FILTERED, rx.PKT_BADIP, rx.PKT_KEEPALIVE, rx.PKT_BADTAG} <= kinds


@pytest.mark.parametrize("uniform", [False, True])
def test_open_with_fused_filter_matches_open_then_rx_check(engine, uniform):
    """wg_open_batch(..., WG_F_RX_FILTER): the open kernel writes the receive-side verdict itself.
    Sealed IP-ish packets (3% forged tags) over 10 key slots and 6 filters; statuses equal
    oracle open + oracle rx_check, plaintexts equal the inputs."""
    torch, dev = _dev()
    W = wg()
    O = oracle()
    rng = np.random.default_rng(17)
    nf = 6
    filters = {}
    for f in range(nf):
        pre = _random_prefixes(rng, int(rng.integers(1, 12)))
        engine.filter_set(f, pre)
        o = rx.IPFilter()
        for a, p in pre:
            o.insert(a.packed, p)
        filters[f] = (pre, o)
    ids = [s % nf for s in range(10)]
    ids[7] = W._lib.WG_NO_FILTER
    ids[8] = 4242
    engine.slot_filters_set(0, ids)
    keys = splitmix_np(0xF11, 32 * 10)
    engine.set_keys(0, keys.tobytes())
    n = 8000
    slots = rng.integers(0, 10, n)
    pts = [_packet(rng, filters[ids[int(s)]][0] if ids[int(s)] in filters else []) for s in slots]
    if uniform:  # equal lengths (the one-packet-per-slot dispatch)
        pts = [(p + bytes(300))[:300] if len(p) else bytes(300) for p in pts]
    lens = np.array([len(p) for p in pts], np.int64)
    S = ((lens + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    total = int(S.sum())
    buf = np.zeros(total, np.uint8)
    for i, p in enumerate(pts):
        buf[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), lens, slots)
    ct = np.zeros(total, np.uint8)
    O.seal_batch(desc, buf, ct, keys, threads=16)
    forged = rng.random(n) < 0.03
    for i in np.nonzero(forged)[0]:
        ct[int(off[i]) + int(lens[i])] ^= 0x10
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    back = torch.zeros(total, dtype=torch.uint8, device=dev)
    st = torch.full((n,), 9, dtype=torch.int32, device=dev)
    engine.open(d, torch.from_numpy(ct).to(dev), back, st, int(lens.max()), uniform=uniform, rx_filter=True)
    torch.cuda.synchronize()
    got = st.cpu().numpy().astype(np.int64).tolist()
    of = {s: (filters[ids[s]][1] if ids[s] in filters else (rx.IPFilter() if ids[s] != W._lib.WG_NO_FILTER else None))
          for s in range(10)}
    want = rx.rx_check(slots, np.arange(n), lens.tolist(), pts, forged.astype(np.int64), of, None)
    assert got == want
    b = back.cpu().numpy()
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        exp = np.zeros(L, np.uint8) if forged[i] else buf[o:o + L]
        assert np.array_equal(b[o:o + L], exp), i


def test_reference_filter_known_answers_on_device(engine):
    torch, dev = _dev()
    W = wg()
    engine.filter_set(0, [("192.168.1.0", 24), ("2001:db8::", 32)])
    engine.slot_filters_set(0, [0])
    pts = []
    for a in ("192.168.1.55", "192.168.2.1", "2001:db8::abcd", "2001:db9::abcd"):
        ip = ipaddress.ip_address(a)
        if ip.version == 4:
            pts.append(bytes([0x45]) + bytes(15) + ip.packed + bytes(4))
        else:
            pts.append(bytes([0x60]) + bytes(23) + ip.packed)
    got = _run(engine, torch, dev, W, [0] * 4, [0, 1, 2, 3], pts, [0] * 4, W._lib.WG_RX_FILTER)
    assert got == [rx.PKT_OK, rx.PKT_FILTERED, rx.PKT_OK, rx.PKT_FILTERED]  # IPFilter.java:85-88


@pytest.fixture(params=["three_launches", "four_launches", "five_launches"])
def rp_engine(request):
    """An engine whose replay checks take each launch structure: three launches (judge with the
    windows advanced by its last block, insert, fix-up + mark; at most 512 key slots), four (the
    same with a separate advance launch; more than 512 key slots), or the five-launch path
    (WG_RX_LAUNCHES=5, read when the context's receive state is created)."""
    import os
    old = os.environ.get("WG_RX_LAUNCHES")
    os.environ["WG_RX_LAUNCHES"] = "5" if request.param == "five_launches" else "3"
    try:
        e = wg().Engine(0, key_slots=1024 if request.param == "four_launches" else 512)
        e.replay_enable(64)
    finally:
        if old is None:
            del os.environ["WG_RX_LAUNCHES"]
        else:
            os.environ["WG_RX_LAUNCHES"] = old
    yield e
    e.close()


def test_replay_window_batches_match_oracle(rp_engine):
    engine = rp_engine
    torch, dev = _dev()
    W = wg()
    Wb = 256
    engine.replay_enable(Wb)
    engine.set_keys(0, splitmix_np(5, 32 * 8).tobytes())  # also empties the windows
    o = rx.ReplayWindow(Wb)
    rng = np.random.default_rng(11)
    base = np.zeros(8, np.int64)
    for b in range(6):
        n = 3000
        slots = rng.integers(0, 8, n)
        # mostly increasing per slot, with duplicates, stragglers, old replays and jumps
        c64 = base[slots] + rng.integers(0, 400, n)
        dup = rng.random(n) < 0.05
        c64[dup] = np.maximum(c64[dup] - rng.integers(0, 600, dup.sum()), 0)
        np.maximum.at(base, slots, c64)
        ctr = c64.astype(np.uint64)
        if b == 3:  # Reject-After-Messages and beyond
            ctr[:5] = np.array([rx.REJECT_AFTER - 1 + k for k in range(5)], dtype=np.uint64)
        status = np.where(rng.random(n) < 0.02, 1, 0)
        pts = [b""] * n
        got = _run(engine, torch, dev, W, slots, ctr, pts, status, W._lib.WG_RX_REPLAY)
        want = o.check_batch(slots, [int(x) for x in ctr], status)
        assert got == want, b
        for s in range(8):
            top, words = engine.replay_state(s, Wb)
            otop, owords = o.bitmap(s)
            assert top == otop and [int(x) for x in words] == owords, (b, s)
    assert any(x == rx.PKT_REPLAY for x in want)


def test_replay_sorted_batches_match_oracle(rp_engine):
    """Batches whose (slot, counter) pairs strictly increase with the index skip the duplicate
    table (k_rp_order); replays of earlier batches, old counters and window jumps must still be
    judged exactly as the oracle does. One batch repeats a pair (not strictly increasing) and
    so takes the table path."""
    engine = rp_engine
    torch, dev = _dev()
    W = wg()
    Wb = 512
    engine.replay_enable(Wb)
    engine.set_keys(0, splitmix_np(6, 32 * 64).tobytes())
    o = rx.ReplayWindow(Wb)
    rng = np.random.default_rng(23)
    base = np.zeros(64, np.int64)
    for b in range(6):
        n = 20000
        slots = np.sort(rng.integers(0, 64, n))
        c64 = base[slots] + rng.integers(-700, 900, n)
        c64 = np.maximum(c64, 0)
        order = np.lexsort((c64, slots))
        slots, c64 = slots[order], c64[order]
        keep = np.ones(n, bool)
        keep[1:] = (slots[1:] != slots[:-1]) | (c64[1:] != c64[:-1])
        slots, c64 = slots[keep], c64[keep]
        if b == 4:  # one repeated pair: the batch is no longer strictly increasing
            slots = np.insert(slots, 10, slots[10])
            c64 = np.insert(c64, 10, c64[10])
        np.maximum.at(base, slots, c64)
        ctr = c64.astype(np.uint64)
        status = np.where(rng.random(len(slots)) < 0.01, 1, 0)
        got = _run(engine, torch, dev, W, slots, ctr, [b""] * len(slots), status, W._lib.WG_RX_REPLAY)
        want = o.check_batch(slots, [int(x) for x in ctr], status)
        assert got == want, b
        for s_ in range(64):
            top, words = engine.replay_state(s_, Wb)
            otop, owords = o.bitmap(s_)
            assert top == otop and [int(x) for x in words] == owords, (b, s_)
    assert any(x == rx.PKT_REPLAY for x in want)


@pytest.mark.parametrize("sorted_batch", [False, True])
def test_replay_large_batches_many_slots(rp_engine, sorted_batch):
    """Batches of 300,000 packets over 512 key slots (1,172 blocks racing to be the last of
    k_rp_judge, every slot's new top spread over 8 copies): interleaved slots (the table path,
    with duplicates) or the same packets sorted by (slot, counter) (no table)."""
    engine = rp_engine
    torch, dev = _dev()
    W = wg()
    Wb = 1024
    engine.replay_enable(Wb)
    engine.set_keys(0, splitmix_np(8, 32 * 512).tobytes())
    o = rx.ReplayWindow(Wb)
    rng = np.random.default_rng(31 + sorted_batch)
    base = np.zeros(512, np.int64)
    for b in range(3):
        n = 300000
        slots = rng.integers(0, 512, n)
        c64 = base[slots] + rng.integers(0, 700, n)
        dup = rng.random(n) < 0.03
        c64[dup] = np.maximum(c64[dup] - rng.integers(0, 1500, dup.sum()), 0)
        if sorted_batch:
            order = np.lexsort((c64, slots))
            slots, c64 = slots[order], c64[order]
            keep = np.ones(n, bool)
            keep[1:] = (slots[1:] != slots[:-1]) | (c64[1:] != c64[:-1])
            slots, c64 = slots[keep], c64[keep]
        np.maximum.at(base, slots, c64)
        ctr = c64.astype(np.uint64)
        status = np.where(rng.random(len(slots)) < 0.01, 1, 0)
        got = _run(engine, torch, dev, W, slots, ctr, [b""] * len(slots), status, W._lib.WG_RX_REPLAY)
        want = o.check_batch(slots, [int(x) for x in ctr], status)
        assert got == want, b
        for s_ in range(0, 512, 17):
            top, words = engine.replay_state(s_, Wb)
            otop, owords = o.bitmap(s_)
            assert top == otop and [int(x) for x in words] == owords, (b, s_)
    assert any(x == rx.PKT_REPLAY for x in want)


def test_replay_then_filter_and_key_reset(engine):
    """WG_RX_REPLAY | WG_RX_FILTER on opened packets: replay first (keepalives count), then
    the filter; a new key for a slot empties its window."""
    torch, dev = _dev()
    W = wg()
    O = oracle()
    engine.replay_enable(128)
    keys = splitmix_np(9, 32 * 2)
    engine.set_keys(0, keys.tobytes())
    engine.filter_set(0, [("10.0.0.0", 8)])
    engine.slot_filters_set(0, [0, W._lib.WG_NO_FILTER])
    pts = [bytes([0x45]) + bytes(15) + ipaddress.ip_address(a).packed + bytes(20)
           for a in ("10.1.2.3", "11.1.2.3", "10.9.9.9")] + [b""]
    slots = [0, 0, 0, 0]
    ctrs = [5, 6, 5, 7]
    lens = np.array([len(p) for p in pts], np.int64)
    S = ((lens + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    desc = W.pack_desc(off, off, ctrs, lens, slots)
    buf = np.zeros(int(S.sum()), np.uint8)
    for i, p in enumerate(pts):
        buf[int(off[i]):int(off[i]) + len(p)] = np.frombuffer(p, np.uint8)
    sealed = np.zeros_like(buf)
    O.seal_batch(desc, buf, sealed, keys, threads=1)
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    out = torch.zeros(len(buf), dtype=torch.uint8, device=dev)
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    engine.open(d, torch.from_numpy(sealed).to(dev), out, st, int(lens.max()))
    engine.rx_check(d, out, st, W._lib.WG_RX_FILTER | W._lib.WG_RX_REPLAY)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [rx.PKT_OK, rx.PKT_FILTERED, rx.PKT_REPLAY, rx.PKT_KEEPALIVE]
    assert engine.replay_state(0, 128)[0] == 8
    engine.set_keys(0, keys[:32].tobytes())
    assert engine.replay_state(0, 128)[0] == 0


def test_rekey_is_ordered_after_replay_checks_on_another_stream():
    """A replay check queued on a side stream, then wg_keys_set for its slot with no
    synchronisation in between: the window reset must land after the queued check,
    so the new session's counters from 0 are accepted, not rejected as too old."""
    torch, dev = _dev()
    W = wg()
    eng = W.Engine(0, key_slots=4)
    try:
        eng.replay_enable(256)
        eng.set_keys(0, splitmix_np(21, 32 * 4).tobytes())
        n = 60000
        desc = W.pack_desc(np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.arange(1_000_000, 1_000_000 + n),
                           np.zeros(n, np.int64), np.zeros(n, np.int64))
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        pt = torch.zeros(64, dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(device=dev)
        for _ in range(3):
            st = torch.zeros(n, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                eng.rx_check(d, pt, st, W._lib.WG_RX_REPLAY)  # old session: top -> 1,060,000
            eng.set_keys(0, splitmix_np(22, 32).tobytes())      # new session, no sync before it
            fresh = W.pack_desc(np.zeros(4, np.uint64), np.zeros(4, np.uint64), np.arange(4), np.zeros(4, np.int64),
                                np.zeros(4, np.int64))
            st2 = torch.zeros(4, dtype=torch.int32, device=dev)
            eng.rx_check(torch.from_numpy(W.desc_as_int64(fresh)).to(dev), pt, st2, W._lib.WG_RX_REPLAY)
            torch.cuda.synchronize()
            assert (st.cpu().numpy() == rx.PKT_OK).all()  # the old batch: all fresh counters
            assert st2.cpu().tolist() == [rx.PKT_OK] * 4  # counters 0..3 of the new session accepted
            assert eng.replay_state(0, 256)[0] == 4
    finally:
        eng.close()


def test_rx_argument_contract(engine):
    torch, dev = _dev()
    W = wg()
    lib = W.lib()
    d = torch.zeros((1, 4), dtype=torch.int64, device=dev)
    s = torch.zeros(1, dtype=torch.int32, device=dev)
    b = torch.zeros(64, dtype=torch.uint8, device=dev)
    E = W._lib.WG_EINVAL
    assert lib.wg_rx_check(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, s.data_ptr(), 0x10, None) == E
    assert lib.wg_rx_check(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, None, 1, None) == E
    assert lib.wg_replay_enable(engine.ctx, 100) == E
    assert lib.wg_replay_enable(engine.ctx, 0) == 0  # disabled: WG_RX_REPLAY is refused
    assert lib.wg_rx_check(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, s.data_ptr(), 2, None) == E
    assert lib.wg_rx_check(engine.ctx, d.data_ptr(), 0, None, 0, None, 3, None) == 0  # n = 0
    assert lib.wg_slot_filters_set(engine.ctx, engine.key_slots, 1, None) == E  # NULL ids with n > 0
    assert lib.wg_filter_set(engine.ctx, W._lib.WG_MAX_FILTERS, None, 0) == W._lib.WG_ERANGE


def _skew_check(mutant: bool) -> dict:
    """Body of test_replay_flag_protocol_under_block_skew, run in a child process that loads the test
    library (the hooks exist only there) with the hook variables set: four duplicate-laden replay
    checks, each compared with the oracle (statuses and every slot's window)."""
    torch, dev = _dev()
    W = wg()
    engine = W.Engine(0, key_slots=512)
    engine.replay_enable(256)
    try:
        engine.set_keys(0, splitmix_np(9, 32 * 16).tobytes())
        o = rx.ReplayWindow(256)
        rng = np.random.default_rng(77)
        base = np.zeros(16, np.int64)
        agree, replays = [], []
        for b in range(4):
            n = 20000  # 79 blocks
            slots = rng.integers(0, 16, n)
            c64 = base[slots] + rng.integers(0, 300, n)
            dup = rng.random(n) < 0.08
            c64[dup] = np.maximum(c64[dup] - rng.integers(0, 200, dup.sum()), 0)
            np.maximum.at(base, slots, c64)
            ctr = c64.astype(np.uint64)
            status = np.zeros(n, np.int64)
            got = _run(engine, torch, dev, W, slots, ctr, [b""] * n, status, W._lib.WG_RX_REPLAY)
            want = o.check_batch(slots, [int(x) for x in ctr], status)
            same = got == want
            for s_ in range(16):
                top, words = engine.replay_state(s_, 256)
                otop, owords = o.bitmap(s_)
                same = same and top == otop and [int(x) for x in words] == owords
            agree.append(bool(same))
            replays.append(any(x == rx.PKT_REPLAY for x in want))
        return {"agree": agree, "replays": replays, "lib": W._lib.LIB_PATH}
    finally:
        engine.close()


@pytest.mark.parametrize("mutant", [False, True])
def test_replay_flag_protocol_under_block_skew(mutant):
    """Regression test of the order-flag race fixed in round 4 (98a2832): k_rp_fixmark cleared the
    order flag that its own later-starting blocks still read, so they skipped their duplicate
    fix-ups and a repeated (slot, counter) could be accepted twice. WG_RX_TEST_SKEW delays every
    block but block 0 of each replay launch by 30 us, so block 0 always finishes first.
    Consecutive duplicate-laden checks must then still match the oracle (flag words, done counts,
    group counts and new-top copies all read after the skew). WG_RX_TEST_MUTANT=1 puts the old flag
    clearing back: the same checks must then disagree with the oracle, which shows that the skew
    exposes the race. The hooks exist only in the test library, so the check runs in a
    child process that loads it. Reference: TransportManager.java:98-119 (the window itself is unpinned)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    test_lib = os.path.join(root, "wireguard-java_amd", "libwgaead_test.so")
    assert os.path.exists(test_lib), "build the test library first (__graft_entry__.build())"
    env = dict(os.environ, WG_LIB_PATH=test_lib, WG_RX_LAUNCHES="3", WG_RX_TEST_SKEW="30",
               WG_RX_TEST_MUTANT="1" if mutant else "0")
    code = ("import json, sys; sys.path[:0] = ['tests', '.']; import test_gpu_rx as t; "
            f"print(json.dumps(t._skew_check({bool(mutant)})), flush=True)")
    p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=100)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stderr[-2000:]
    r = json.loads(lines[-1])
    assert r["lib"] == test_lib
    if mutant:
        assert not all(r["agree"]), "the skew did not expose the round-4 flag race"
    else:
        assert all(r["agree"]), r
        assert all(r["replays"])

