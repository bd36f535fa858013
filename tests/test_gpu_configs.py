"""BASELINE configs at full size on the MI355X (pytest -m gpu), every compared byte against
the oracle (oracle/liboracle.so), plus the batch API's argument contract.

  C2 = configs[2]: 65536 packets of 64..9000 B over 256 session keys, every packet compared
  C3 = configs[3]: 8,388,608 x 1420 B sharded by session (dist.shard_packets), 1024 keys on
       one GPU: full seal -> open round trip on the device, a seeded 65536-packet subset
       compared byte for byte with the oracle
"""
import importlib

import numpy as np
import pytest

from wgtest import oracle, splitmix_np, wg

pytestmark = pytest.mark.gpu
O = oracle()


def _dev():
    import torch
    assert torch.cuda.is_available()
    return torch, torch.device("cuda", 0)


def _c2_batch(W, n=65536):
    """configs[2] exactly as bench.py --workload c2 builds it: 64..9000 B, key slot i mod 256,
    counters i div 256 (each session counting its own packets)."""
    lengths = (64 + splitmix_np(0x5EED2026, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
    S = ((lengths + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64) // 256, lengths, np.arange(n) % 256)
    return lengths, S, off, int(S.sum()), desc


@pytest.mark.parametrize("path", ["separate", "after_seal"])
def test_c2_full_every_packet(engine, path):
    """Every C2 packet sealed against the oracle, then opened with 1% forged tags.
    path "separate": wg_seal_batch then wg_open_batch (k_transport launches);
    "after_seal": wg_duplex_batch(seal, open | WG_F_AFTER_SEAL), the ONE k_step launch the C2
    bench line times (8-lane longest-first pairs at 65,536 packets, 9000-B packets up to 18
    rounds, one issue-priority schedule over both halves): its ciphertext is compared with the
    oracle byte for byte and its plaintext with the input, so a self-consistent seal bug (a
    wrong tag the same code recomputes on open) cannot pass."""
    torch, dev = _dev()
    W = wg()
    n = 65536
    lengths, S, off, total, desc = _c2_batch(W, n)
    keys = splitmix_np(0xC0FFEE, 32 * 256)
    pt = splitmix_np(0x5EED2027, total)
    engine.set_keys(0, keys.tobytes())
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    dpt = torch.from_numpy(pt).to(dev)
    dct = torch.zeros(total, dtype=torch.uint8, device=dev)
    if path == "separate":
        engine.seal(d, dpt, dct, 9000)
    else:
        back = torch.zeros(total, dtype=torch.uint8, device=dev)
        st = torch.full((n,), 7, dtype=torch.int32, device=dev)
        engine.duplex(d, dpt, dct, 9000, d, dct, back, st, 9000, uniform=False, after_seal=True)
    torch.cuda.synchronize()
    ref = np.zeros(total, np.uint8)
    O.seal_batch(desc, pt, ref, keys, threads=16)
    got = dct.cpu().numpy()
    assert np.array_equal(got, ref)  # every packet's ct || tag (and untouched slack)
    if path == "after_seal":
        assert int(st.abs().sum().item()) == 0
        b = back.cpu().numpy()
        want = pt.copy()
        for i in range(n):
            o, L = int(off[i]), int(lengths[i])
            want[o + L:o + int(S[i])] = 0  # slack between packets: never written
        assert np.array_equal(b, want)
        del back
    # open every packet, 1% tampered
    bad = np.nonzero(splitmix_np(99, n) < 3)[0]
    for i in bad:
        got[int(off[i]) + int(lengths[i])] ^= 0x10
    back = torch.zeros(total, dtype=torch.uint8, device=dev)
    st = torch.full((n,), 7, dtype=torch.int32, device=dev)
    engine.open(d, torch.from_numpy(got).to(dev), back, st, 9000)
    torch.cuda.synchronize()
    exp = np.zeros(n, np.int32)
    exp[bad] = 1
    assert np.array_equal(st.cpu().numpy(), exp)
    b = back.cpu().numpy()
    want = pt.copy()
    bad_set = set(bad.tolist())
    for i in range(n):
        o, L = int(off[i]), int(lengths[i])
        want[o + L:o + int(S[i])] = 0  # slack between packets: never written
        if i in bad_set:
            want[o:o + L] = 0  # unauthenticated plaintext scrubbed
    assert np.array_equal(b, want)


@pytest.mark.parametrize("packets", [65536, 32768, 131072])
def test_imix_every_packet(engine, packets):
    """bench.py --workload imix (SURVEY.md §8d's IMIX-like mix: 40 / 576 / 1500 B at 7 : 4 : 1, 256
    sessions) through the one k_step launch its line times (65,536 packets; 32,768 and 131,072 take the
    same plan, long packets in 16-lane and the rest in 4-lane slots): every ct || tag against the
    oracle, every plaintext back, 1% forged tags rejected with their plaintext scrubbed."""
    import bench
    torch, dev = _dev()
    W = wg()
    lengths, slots, counters, nkeys, _, uniform = bench.build_workload("imix", 0, 1, packets)
    assert not uniform and nkeys == 256
    n = len(lengths)
    S = ((lengths + 16 + 15) // 16) * 16
    off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    total = int(S.sum())
    desc = W.pack_desc(off, off, counters, lengths, slots)
    keys = splitmix_np(0xC0FFEE, 32 * nkeys)
    pt = splitmix_np(0x5EED2028, total)
    engine.set_keys(0, keys.tobytes())
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    dct = torch.zeros(total, dtype=torch.uint8, device=dev)
    back = torch.zeros(total, dtype=torch.uint8, device=dev)
    st = torch.full((n,), 7, dtype=torch.int32, device=dev)
    engine.duplex(d, torch.from_numpy(pt).to(dev), dct, 1500, d, dct, back, st, 1500, uniform=False, after_seal=True)
    torch.cuda.synchronize()
    ref = np.zeros(total, np.uint8)
    O.seal_batch(desc, pt, ref, keys, threads=16)
    got = dct.cpu().numpy()
    assert np.array_equal(got, ref)
    assert int(st.abs().sum().item()) == 0
    want = pt.copy()
    for i in range(n):
        want[int(off[i]) + int(lengths[i]):int(off[i]) + int(S[i])] = 0  # slack: never written
    assert np.array_equal(back.cpu().numpy(), want)
    bad = np.nonzero(splitmix_np(98, n) < 3)[0]
    for i in bad:
        got[int(off[i]) + int(lengths[i]) + 15] ^= 0x80
    back.zero_()
    st.fill_(7)
    engine.open(d, torch.from_numpy(got).to(dev), back, st, 1500)
    torch.cuda.synchronize()
    exp = np.zeros(n, np.int32)
    exp[bad] = 1
    assert np.array_equal(st.cpu().numpy(), exp)
    for i in bad:
        want[int(off[i]):int(off[i]) + int(lengths[i])] = 0  # unauthenticated plaintext scrubbed
    assert np.array_equal(back.cpu().numpy(), want)


@pytest.mark.parametrize("n", [65536, 131072, 50000])
def test_k_step_claim_every_packet(n):
    """WG_CLAIM=1: mixed-length WG_F_AFTER_SEAL steps through k_step_claim, whose slots claim their
    packets dynamically from 64 interleaved longest-first sub-orders and whose open half replays the
    seal half's log. Three steps in a row (the counters are reset by every step's k_lpt_scatter): every
    ct || tag against the oracle, every plaintext against the input, every status OK. n = 50,000 takes
    a grid that 64 does not divide (fewer sub-orders)."""
    import os
    torch, dev = _dev()
    W = wg()
    old = os.environ.get("WG_CLAIM")
    os.environ["WG_CLAIM"] = "1"
    try:
        eng = W.Engine(0, key_slots=256)
    finally:
        if old is None:
            del os.environ["WG_CLAIM"]
        else:
            os.environ["WG_CLAIM"] = old
    try:
        lengths, S, off, total, desc = _c2_batch(W, n)
        keys = splitmix_np(0xC1A1, 32 * 256)
        pt = splitmix_np(0x5EED2028 + n, total)
        eng.set_keys(0, keys.tobytes())
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        dpt = torch.from_numpy(pt).to(dev)
        ref = np.zeros(total, np.uint8)
        O.seal_batch(desc, pt, ref, keys, threads=16)
        want = pt.copy()
        for i in range(n):
            want[int(off[i]) + int(lengths[i]):int(off[i]) + int(S[i])] = 0
        for rep in range(3):
            dct = torch.zeros(total, dtype=torch.uint8, device=dev)
            back = torch.zeros(total, dtype=torch.uint8, device=dev)
            st = torch.full((n,), 7, dtype=torch.int32, device=dev)
            eng.duplex(d, dpt, dct, 9000, d, dct, back, st, 9000, uniform=False, after_seal=True)
            torch.cuda.synchronize()
            assert np.array_equal(dct.cpu().numpy(), ref), rep
            assert int(st.abs().sum().item()) == 0, rep
            assert np.array_equal(back.cpu().numpy(), want), rep
    finally:
        eng.close()


@pytest.mark.parametrize("path", ["separate", "after_seal"])
def test_c3_sharded_roundtrip_and_oracle_subset(path):
    """configs[3] on one GPU: 8M x 1420 B, session s -> rank s mod world (world 1 here),
    each session counting its packets from 0; 1024 keys. path "after_seal" is the k_step launch
    the C3 bench line times (one packet per 8-lane slot, 8M packets)."""
    torch, dev = _dev()
    W = wg()
    D = importlib.import_module("wireguard-java_amd.dist")
    total, L, sessions, stride = 8 * 1024 * 1024, 1420, 1024, 1440
    slots, _, counters = D.shard_packets(total, sessions, 0, 1)
    n = len(slots)
    assert n == total
    off = np.arange(n, dtype=np.uint64) * stride
    desc = W.pack_desc(off, off, counters, L, slots)
    keys = splitmix_np(0xC3C3, 32 * sessions)
    eng = W.Engine(0, key_slots=sessions)
    try:
        eng.set_keys(0, keys.tobytes())
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        g = torch.Generator(device=dev)
        g.manual_seed(1234)
        pt = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
        ct = torch.zeros_like(pt)
        back = torch.zeros_like(pt)
        st = torch.full((n,), 7, dtype=torch.int32, device=dev)
        if path == "separate":
            eng.seal(d, pt, ct, L, uniform=True)
            eng.open(d, ct, back, st, L, uniform=True)
        else:
            eng.duplex(d, pt, ct, L, d, ct, back, st, L, uniform=True, after_seal=True)
        torch.cuda.synchronize()
        assert int(st.abs().sum().item()) == 0
        assert torch.equal(back.view(n, stride)[:, :L], pt.view(n, stride)[:, :L])
        # seeded 65536-packet subset, every byte of ct || tag against the oracle
        pick = np.sort(np.random.default_rng(33).choice(n, 65536, replace=False))
        idx = torch.from_numpy(pick.astype(np.int64)).to(dev)
        sub_pt = pt.view(n, stride).index_select(0, idx).cpu().numpy()
        sub_ct = ct.view(n, stride).index_select(0, idx).cpu().numpy()
        sd = desc[pick].copy()
        sd["in_off"] = sd["out_off"] = np.arange(len(pick), dtype=np.uint64) * stride
        ref = np.zeros(len(pick) * stride, np.uint8)
        O.seal_batch(sd, sub_pt.reshape(-1), ref, keys, threads=16)
        ref = ref.reshape(len(pick), stride)
        assert np.array_equal(sub_ct[:, :L + 16], ref[:, :L + 16])
        del pt, ct, back
    finally:
        eng.close()


def test_k_step_mixed_c2_shape_default_plan():
    """wg_duplex_batch(... WG_F_AFTER_SEAL) on 65,536 packets of 64..9000 B over 256 keys with
    the default size-based plan (8-lane longest-first pairs in ONE k_step launch), on a fresh
    context, a different seed from test_c2_full_every_packet and odd (4-B aligned) offsets, so the
    pairs' snake order across the seal -> open boundary is exercised with other lengths; every
    ciphertext byte against the oracle, every plaintext byte against the input, three calls in a
    row."""
    torch, dev = _dev()
    W = wg()
    n = 65536
    lengths = (64 + splitmix_np(0xACE1, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
    S = ((lengths + 16 + 3) // 4) * 4 + 4
    off = (np.concatenate([[0], np.cumsum(S)[:-1]]) + 4).astype(np.uint64)
    total = int(S.sum()) + 8
    desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64) // 256 + (1 << 40), lengths, np.arange(n) % 256)
    keys = splitmix_np(0xBEEF, 32 * 256)
    pt = splitmix_np(0xF00D, total)
    eng = W.Engine(0, key_slots=256)
    try:
        eng.set_keys(0, keys.tobytes())
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        dpt = torch.from_numpy(pt).to(dev)
        dct = torch.zeros(total, dtype=torch.uint8, device=dev)
        back = torch.zeros(total, dtype=torch.uint8, device=dev)
        st = torch.full((n,), 7, dtype=torch.int32, device=dev)
        for _ in range(3):
            back.zero_()
            eng.duplex(d, dpt, dct, 9000, d, dct, back, st, 9000, uniform=False, after_seal=True)
        torch.cuda.synchronize()
        ref = np.zeros(total, np.uint8)
        O.seal_batch(desc, pt, ref, keys, threads=16)
        assert np.array_equal(dct.cpu().numpy(), ref)
        assert int(st.abs().sum().item()) == 0
        b = back.cpu().numpy()
        want = np.zeros(total, np.uint8)
        for i in range(n):
            o, L = int(off[i]), int(lengths[i])
            want[o:o + L] = pt[o:o + L]
        assert np.array_equal(b, want)
    finally:
        eng.close()


@pytest.mark.parametrize("n", [40, 32768])
@pytest.mark.parametrize("shift", [0, -8, -1])
@pytest.mark.parametrize("uniform", [True, False])
def test_in_place_open_keeps_forged_packets(engine, shift, uniform, n):
    """Batch open whose plaintext range overlaps the ciphertext || tag range (in place, shift 0,
    or moved back by a few bytes, which a byte-sequential decrypt also allows; a forward move is
    undefined, as for the reference's sequential cipher): every such packet is verified before
    any byte is written
    (verify-first: the tag pass, then a decrypt pass), as ChaCha20Poly1305.java:40-56 verifies
    before it decrypts. A good packet decrypts in place; a forged one comes back WG_PKT_BADTAG
    with its ciphertext || tag untouched. Mixed lengths (uniform False) include 0-byte and
    multi-round packets. 32,768 mixed packets of at most 2,000 B take the verify-first body of the
    16 / 4-lane split (k_transport_mixed<OPEN, true, 4>)."""
    torch, dev = _dev()
    W = wg()
    rng = np.random.default_rng(70 + shift)
    top = 3000 if n == 40 else 2000
    lengths = np.full(n, 300, np.int64) if uniform else rng.integers(0, top, n).astype(np.int64)
    lengths[3] = 0 if not uniform else lengths[3]
    S = ((lengths + 16 + 15) // 16) * 16 + 32
    off = (np.concatenate([[0], np.cumsum(S)[:-1]]) + 16).astype(np.uint64)
    total = int(S.sum()) + 64
    keys = splitmix_np(61, 32)
    pt = splitmix_np(62 + shift, total)
    sd = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), lengths, np.zeros(n, np.int64))
    sealed = pt.copy()
    O.seal_batch(sd, pt, sealed, keys, threads=8)
    forged = rng.random(n) < 0.3
    forged[0], forged[1] = True, False
    for i in np.nonzero(forged)[0]:
        sealed[int(off[i]) + int(lengths[i])] ^= 1  # a tag bit
    od = sd.copy()
    od["out_off"] = (off.astype(np.int64) + shift).astype(np.uint64)
    engine.set_keys(0, keys.tobytes())
    buf = torch.from_numpy(sealed.copy()).to(dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    engine.open(torch.from_numpy(W.desc_as_int64(od)).to(dev), buf, buf, st, int(lengths.max()), uniform=uniform)
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == forged.astype(np.int32).tolist()
    got = buf.cpu().numpy()
    want = sealed.copy()
    for i in range(n):
        o, L = int(off[i]), int(lengths[i])
        if not forged[i]:
            want[o + shift:o + shift + L] = pt[o:o + L]
        elif not (o < o + shift + L and o + shift < o + L + 16):
            # a packet too short to overlap its own ciphertext || tag (L <= -shift) is an out-of-place
            # open: its plaintext range is zero-filled on a bad tag (include/wgaead.h)
            want[o + shift:o + shift + L] = 0
    for i in range(n):  # packet by packet (a forged packet's bytes, a good one's plaintext)
        o, L = int(off[i]), int(lengths[i])
        lo, hi = min(o, o + shift), max(o + L + 16, o + shift + L)
        assert np.array_equal(got[lo:hi], want[lo:hi]), (i, bool(forged[i]))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kernel", ["tile", "wave1"])
def test_other_kernels_in_place_open_and_rx_filter(kernel):
    """with wg_ctx_set_kernel("tile" / "wave1") an open whose buffers overlap still runs
    the verify-first transport kernel (a forged packet's bytes stay as they were, as every kernel
    must write identical bytes), and WG_F_RX_FILTER is refused (WG_EINVAL) instead of silently
    skipping the AllowedIPs verdict."""
    torch, dev = _dev()
    W = wg()
    eng = W.Engine(0, key_slots=2)
    try:
        eng.set_kernel(kernel)
        n, L = 24, 700
        S = ((L + 16 + 15) // 16) * 16
        off = np.arange(n, dtype=np.uint64) * S
        keys = splitmix_np(81, 32)
        pt = splitmix_np(82, n * S)
        sd = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), L, 0)
        sealed = pt.copy()
        O.seal_batch(sd, pt, sealed, keys, threads=1)
        forged = np.arange(n) % 5 == 2
        for i in np.nonzero(forged)[0]:
            sealed[int(off[i]) + L] ^= 1
        eng.set_keys(0, keys.tobytes())
        buf = torch.from_numpy(sealed.copy()).to(dev)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        d = torch.from_numpy(W.desc_as_int64(sd)).to(dev)
        eng.open(d, buf, buf, st, L, uniform=True)
        torch.cuda.synchronize()
        assert st.cpu().numpy().tolist() == forged.astype(np.int32).tolist()
        got = buf.cpu().numpy()
        for i in range(n):
            o = int(off[i])
            want = sealed[o:o + L + 16] if forged[i] else np.concatenate([pt[o:o + L], sealed[o + L:o + L + 16]])
            assert np.array_equal(got[o:o + L + 16], want), (i, bool(forged[i]))
        out = torch.zeros_like(buf)
        with pytest.raises(W.WgError) as e:
            eng.open(d, buf, out, st, L, uniform=True, rx_filter=True)
        assert e.value.code == W._lib.WG_EINVAL
    finally:
        eng.close()


def test_batch_argument_contract(engine):
    """open needs a status array; unknown flag bits and WG_F_FRAME on open are
    refused (WG_EINVAL) instead of silently ignored."""
    torch, dev = _dev()
    W = wg()
    lib = W.lib()
    d = torch.from_numpy(W.desc_as_int64(W.pack_desc([0], [0], [0], 16, 0))).to(dev)
    b = torch.zeros(64, dtype=torch.uint8, device=dev)
    s = torch.zeros(1, dtype=torch.int32, device=dev)
    E = W._lib.WG_EINVAL
    assert lib.wg_open_batch(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, b.data_ptr(), 64, None, 16, 0, None) == E
    assert lib.wg_open_batch(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, b.data_ptr(), 64, s.data_ptr(), 16,
                             W._lib.WG_F_FRAME, None) == E
    assert lib.wg_seal_batch(engine.ctx, d.data_ptr(), 1, b.data_ptr(), 64, b.data_ptr(), 64, 16, 0x80, None) == E
    assert lib.wg_open_batch(engine.ctx, d.data_ptr(), 0, b.data_ptr(), 64, b.data_ptr(), 64, None, 16, 0, None) == 0


def test_mixed_batch_on_two_streams_shares_plan_workspace(engine):
    """Two mixed-length (longest-first ordered) batches enqueued on two different streams of
    one context: the second waits for the first's plan workspace, both bit-exact."""
    torch, dev = _dev()
    W = wg()
    outs = []
    refs = []
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    keys = splitmix_np(71, 32 * 4)
    engine.set_keys(0, keys.tobytes())
    for k, stream in enumerate((s1, s2)):
        n = 40000 + 5000 * k  # more packets than resident slots: the LPT order is used
        lengths = (splitmix_np(72 + k, 4 * n).view("<u4") % 1500).astype(np.int64)
        S = ((lengths + 16 + 15) // 16) * 16
        off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
        desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), lengths, np.arange(n) % 4)
        pt = splitmix_np(80 + k, int(S.sum()))
        ref = np.zeros_like(pt)
        O.seal_batch(desc, pt, ref, keys, threads=16)
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        dp = torch.from_numpy(pt).to(dev)
        out = torch.zeros_like(dp)
        torch.cuda.synchronize()
        engine.seal(d, dp, out, int(lengths.max()), stream=stream.cuda_stream)
        outs.append((out, d, dp))
        refs.append(ref)
    torch.cuda.synchronize()
    for (out, _, _), ref in zip(outs, refs):
        assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("slot2,workload", [(1, "imix"), (2, "imix"), (0, "ragged"), (1, "ragged"), (2, "ragged")])
def test_two_lane_slots_every_packet(slot2, workload):
    """WG_SLOT2=k (default 1): the short-packet split plan's step (k_step_mixed<4, false, 2>) puts the packets
    of at most 8 k blocks (keys <= k) in 2-lane slots, after the 16-lane and 4-lane parts (0: no 2-lane part,
    k_step_mixed<4>). 80-B slot records, the key read from the key table each round. "imix" is bench.py's IMIX
    batch; "ragged" is 65,536 packets of 0..2,048 B (every partial-chunk shape in 2-lane slots, empty
    packets, and both other parts populated). Two steps in a row: every ct || tag against the oracle, every
    plaintext back, every status OK."""
    import os

    import bench
    torch, dev = _dev()
    W = wg()
    old = os.environ.get("WG_SLOT2")
    os.environ["WG_SLOT2"] = str(slot2)
    try:
        eng = W.Engine(0, key_slots=256)
    finally:
        if old is None:
            del os.environ["WG_SLOT2"]
        else:
            os.environ["WG_SLOT2"] = old
    try:
        if workload == "imix":
            lengths, slots, counters, nkeys, _, _ = bench.build_workload("imix", 0, 1)
        else:
            n = 65536
            lengths = (splitmix_np(0x5107 + slot2, 4 * n).view("<u4") % 2049).astype(np.int64)
            lengths[:64] = np.arange(64)  # 0..63 B: every partial first block
            slots, counters, nkeys = np.arange(n) % 256, np.arange(n, dtype=np.uint64) // 256, 256
        n = len(lengths)
        S = ((lengths + 16 + 15) // 16) * 16
        off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
        total = int(S.sum())
        desc = W.pack_desc(off, off, counters, lengths, slots)
        keys = splitmix_np(0x2A2E + slot2, 32 * nkeys)
        pt = splitmix_np(0x5EED2029 + slot2, total)
        eng.set_keys(0, keys.tobytes())
        ml = int(lengths.max())
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        dpt = torch.from_numpy(pt).to(dev)
        ref = np.zeros(total, np.uint8)
        O.seal_batch(desc, pt, ref, keys, threads=16)
        want = pt.copy()
        for i in range(n):
            want[int(off[i]) + int(lengths[i]):int(off[i]) + int(S[i])] = 0  # slack: never written
        for _ in range(2):
            dct = torch.zeros(total, dtype=torch.uint8, device=dev)
            back = torch.zeros(total, dtype=torch.uint8, device=dev)
            st = torch.full((n,), 7, dtype=torch.int32, device=dev)
            eng.duplex(d, dpt, dct, ml, d, dct, back, st, ml, uniform=False, after_seal=True)
            torch.cuda.synchronize()
            assert np.array_equal(dct.cpu().numpy(), ref)
            assert int(st.abs().sum().item()) == 0
            assert np.array_equal(back.cpu().numpy(), want)
    finally:
        eng.close()


def test_short_plan_steps_on_destroyed_and_recreated_streams():
    """Per-stream plan workspaces (WG_STREAM_WS) are keyed by stream handle; each use waits for the workspace's
    last use (an event, WG_WSEV=3). A step on a stream that is destroyed while its launches run, then a step on
    a new stream (which may get the same handle) with a DIFFERENT batch, must not plan into the workspace the
    first step's kernel is still reading. Four rounds of create / step / destroy, each with its own
    0..2,048-B batch, then every output against the oracle."""
    import ctypes
    torch, dev = _dev()
    W = wg()
    hip = ctypes.CDLL("libamdhip64.so")
    eng = W.Engine(0, key_slots=256)
    keys = splitmix_np(0x57EA, 32 * 256)
    eng.set_keys(0, keys.tobytes())
    runs = []
    try:
        for r in range(4):
            n = 65536
            lengths = (splitmix_np(0x5700 + r, 4 * n).view("<u4") % 2049).astype(np.int64)
            S = ((lengths + 16 + 15) // 16) * 16
            off = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
            desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64) // 256, lengths, np.arange(n) % 256)
            total = int(S.sum())
            pt = splitmix_np(0x5701 + r, total)
            d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
            dpt = torch.from_numpy(pt).to(dev)
            dct = torch.zeros(total, dtype=torch.uint8, device=dev)
            back = torch.zeros(total, dtype=torch.uint8, device=dev)
            st = torch.full((n,), 7, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            step = eng.prepare_duplex(d, dpt, dct, 2048, d, dct, back, st, 2048, uniform=False, after_seal=True,
                                      stream=s.value)
            step()
            assert hip.hipStreamDestroy(s) == 0  # while the step may still run
            runs.append((lengths, S, off, total, desc, pt, d, dpt, dct, back, st))
        torch.cuda.synchronize()
        for lengths, S, off, total, desc, pt, d, dpt, dct, back, st in runs:
            ref = np.zeros(total, np.uint8)
            O.seal_batch(desc, pt, ref, keys, threads=16)
            assert np.array_equal(dct.cpu().numpy(), ref)
            assert int(st.abs().sum().item()) == 0
            want = pt.copy()
            for i in range(len(lengths)):
                want[int(off[i]) + int(lengths[i]):int(off[i]) + int(S[i])] = 0
            assert np.array_equal(back.cpu().numpy(), want)
    finally:
        eng.close()


def test_c2_wide_one_launch_plan_every_packet():
    """WG_LPT_WIDE=1 (A/B knob, off by default): C2's step planned by ONE k_lpt_one launch over 32 round keys
    (a sparse longest-first order) and run by k_step<8, 4, ..., kWideBins>, which maps its positions through the
    counts. Two steps in a row (double-buffered counters): every ct || tag against the oracle, every plaintext
    back, every status OK."""
    import os
    torch, dev = _dev()
    W = wg()
    old = os.environ.get("WG_LPT_WIDE")
    os.environ["WG_LPT_WIDE"] = "1"
    try:
        eng = W.Engine(0, key_slots=256)
    finally:
        if old is None:
            del os.environ["WG_LPT_WIDE"]
        else:
            os.environ["WG_LPT_WIDE"] = old
    try:
        n = 65536
        lengths, S, off, total, desc = _c2_batch(W, n)
        keys = splitmix_np(0xC0FFEE, 32 * 256)
        pt = splitmix_np(0x5EED2030, total)
        eng.set_keys(0, keys.tobytes())
        d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
        dpt = torch.from_numpy(pt).to(dev)
        ref = np.zeros(total, np.uint8)
        O.seal_batch(desc, pt, ref, keys, threads=16)
        want = pt.copy()
        for i in range(n):
            want[int(off[i]) + int(lengths[i]):int(off[i]) + int(S[i])] = 0
        for _ in range(2):
            dct = torch.zeros(total, dtype=torch.uint8, device=dev)
            back = torch.zeros(total, dtype=torch.uint8, device=dev)
            st = torch.full((n,), 7, dtype=torch.int32, device=dev)
            eng.duplex(d, dpt, dct, 9000, d, dct, back, st, 9000, uniform=False, after_seal=True)
            torch.cuda.synchronize()
            assert np.array_equal(dct.cpu().numpy(), ref)
            assert int(st.abs().sum().item()) == 0
            assert np.array_equal(back.cpu().numpy(), want)
    finally:
        eng.close()
