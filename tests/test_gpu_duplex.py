"""wg_duplex_batch (pytest -m gpu): one launch that seals one batch and opens another must
write exactly the bytes of wg_seal_batch + wg_open_batch, checked against the oracle
(oracle/liboracle.so) byte for byte.

The reference runs a node's outgoing cipher and incoming decipher on one ForkJoinPool
(TransportManager.java:41,79); the duplex launch is that pair of batches in one kernel.
"""
import numpy as np
import pytest

from wgtest import oracle, splitmix_np, wg

pytestmark = pytest.mark.gpu
O = oracle()


def _dev():
    import torch
    assert torch.cuda.is_available()
    return torch, torch.device("cuda", 0)


def _batch(seed, n, lengths, nkeys, ctr_base=0, pre=0):
    """Packets at 16-B aligned strides; `pre` bytes of header room in front of each."""
    W = wg()
    S = ((lengths + 16 + 15) // 16) * 16 + pre
    off = (np.cumsum(S) - S + pre).astype(np.uint64)
    total = int(S.sum())
    desc = W.pack_desc(off, off, ctr_base + np.arange(n, dtype=np.uint64), lengths, np.arange(n) % nkeys)
    pt = splitmix_np(seed, total)
    return desc, off, total, pt


def _run(engine, n_seal, n_open, lens_seal, lens_open, nkeys, uniform, forge_every=0, frame=False):
    torch, dev = _dev()
    W = wg()
    keys = splitmix_np(0xD0D0 + nkeys, 32 * nkeys)
    engine.set_keys(0, keys.tobytes())
    sdesc, soff, stotal, spt = _batch(0xA11CE, n_seal, lens_seal, nkeys, pre=16 if frame else 0)
    odesc, ooff, ototal, opt = _batch(0xB0B, n_open, lens_open, nkeys, ctr_base=1 << 33)
    # the open batch's input: its plaintexts sealed by the oracle, some tags forged
    oct_ = np.zeros(ototal, np.uint8)
    if n_open:
        O.seal_batch(odesc, opt, oct_, keys, threads=16)
    bad = np.arange(0, n_open, forge_every) if forge_every else np.zeros(0, np.int64)
    for i in bad:
        oct_[int(ooff[i]) + int(lens_open[i])] ^= 0x01
    ds = torch.from_numpy(W.desc_as_int64(sdesc)).to(dev)
    do = torch.from_numpy(W.desc_as_int64(odesc)).to(dev)
    dspt = torch.from_numpy(spt).to(dev)
    dsct = torch.zeros(max(stotal, 1), dtype=torch.uint8, device=dev)
    doct = torch.from_numpy(oct_).to(dev) if ototal else torch.zeros(1, dtype=torch.uint8, device=dev)
    dback = torch.zeros(max(ototal, 1), dtype=torch.uint8, device=dev)
    st = torch.full((max(n_open, 1),), 7, dtype=torch.int32, device=dev)
    rx = None
    if frame:
        rx = torch.arange(1000, 1000 + engine.key_slots, dtype=torch.int32, device=dev)
        engine.set_receivers(rx)
    maxs = int(lens_seal.max()) if n_seal else 0
    maxo = int(lens_open.max()) if n_open else 0
    engine.duplex(ds, dspt, dsct, maxs, do, doct, dback, st, maxo, uniform=uniform, frame=frame)
    torch.cuda.synchronize()
    if frame:
        engine.set_receivers(None)
    # seal half: ct || tag of every packet, slack untouched (or the header when framed)
    ref = np.zeros(max(stotal, 1), np.uint8)
    if n_seal:
        O.seal_batch(sdesc, spt, ref[:stotal], keys, threads=16)
    got = dsct.cpu().numpy()
    if frame:
        O.frame_headers(sdesc, np.arange(1000, 1000 + engine.key_slots, dtype=np.uint32), ref, engine.key_slots,
                        in_size=stotal,
                        max_len=maxs)
    assert np.array_equal(got, ref)
    # open half: statuses, plaintexts, forged packets zero-filled
    if n_open:
        exp = np.zeros(n_open, np.int32)
        exp[bad] = 1
        assert np.array_equal(st.cpu().numpy()[:n_open], exp)
        b = dback.cpu().numpy()
        want = np.zeros(ototal, np.uint8)
        for i in range(n_open):
            o, L_ = int(ooff[i]), int(lens_open[i])
            if i % forge_every if forge_every else True:
                want[o:o + L_] = opt[o:o + L_]
        assert np.array_equal(b[:ototal], want)


def test_duplex_uniform_c1_shape(engine):
    n = 65536
    L_ = np.full(n, 1420, np.int64)
    _run(engine, n, n, L_, L_, 1, uniform=True, forge_every=97)


def test_duplex_mixed_lengths_many_keys(engine):
    n = 20000
    ls = (64 + splitmix_np(1, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
    lo = (splitmix_np(2, 4 * n).view("<u4") % 1501).astype(np.int64)
    _run(engine, n, n, ls, lo, 256, uniform=False, forge_every=13)


def test_duplex_unequal_sizes_and_empty_sides(engine):
    a = np.full(5000, 1420, np.int64)
    b = np.full(300, 64, np.int64)
    _run(engine, 5000, 300, a, b, 4, uniform=True, forge_every=7)
    _run(engine, 300, 5000, b, a, 4, uniform=True, forge_every=11)
    _run(engine, 700, 0, a[:700], a[:0], 2, uniform=True)
    _run(engine, 0, 700, a[:0], a[:700], 2, uniform=True, forge_every=5)


def test_duplex_frame_flag(engine):
    L_ = np.full(3000, 1000, np.int64)
    _run(engine, 3000, 1000, L_, L_[:1000], 8, uniform=True, forge_every=3, frame=True)


def test_duplex_argument_contract(engine):
    torch, dev = _dev()
    W = wg()
    L = W._lib
    d = torch.zeros((4, 4), dtype=torch.int64, device=dev)
    buf = torch.zeros(4096, dtype=torch.uint8, device=dev)
    with pytest.raises(W.WgError) as e:  # open without a status array
        engine.duplex(d, buf, buf, 64, d, buf, buf, None, 64)
    assert e.value.code == L.WG_EINVAL
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    engine.set_receivers(None)
    with pytest.raises(W.WgError) as e:  # WG_F_FRAME without a receiver table
        engine.duplex(d, buf, buf, 64, d, buf, buf, st, 64, frame=True)
    assert e.value.code == L.WG_EINVAL


def _after_seal(engine, n, lengths, nkeys, uniform, forge=()):
    """wg_duplex_batch(seal, open | WG_F_AFTER_SEAL): seal a batch and, in the same call, open
    exactly what was sealed. Every ciphertext byte against the oracle, every plaintext byte
    against the input, statuses all OK."""
    torch, dev = _dev()
    W = wg()
    keys = splitmix_np(0xE0E0 + nkeys, 32 * nkeys)
    engine.set_keys(0, keys.tobytes())
    desc, off, total, pt = _batch(0xC0C0 + n, n, lengths, nkeys)
    d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    dpt = torch.from_numpy(pt).to(dev)
    dct = torch.zeros(total, dtype=torch.uint8, device=dev)
    dback = torch.zeros(total, dtype=torch.uint8, device=dev)
    st = torch.full((n,), 7, dtype=torch.int32, device=dev)
    m = int(lengths.max())
    for _ in range(3):  # repeated calls
        dback.zero_()
        engine.duplex(d, dpt, dct, m, d, dct, dback, st, m, uniform=uniform, after_seal=True)
    torch.cuda.synchronize()
    ref = np.zeros(total, np.uint8)
    O.seal_batch(desc, pt, ref, keys, threads=16)
    ct = dct.cpu().numpy()
    for i in range(n):
        o, L = int(off[i]), int(lengths[i])
        assert np.array_equal(ct[o:o + L + 16], ref[o:o + L + 16]), f"ct of packet {i}"
    back = dback.cpu().numpy()
    assert (st.cpu().numpy() == 0).all()
    for i in range(n):
        o, L = int(off[i]), int(lengths[i])
        assert np.array_equal(back[o:o + L], pt[o:o + L]), f"plaintext of packet {i}"


@pytest.mark.parametrize("variant", [0, 1])
def test_after_seal_c1_shaped(variant):
    """variant 0: one k_step launch; 1: the same step as a seal launch and an open launch."""
    W = wg()
    eng = W.Engine(0, key_slots=1)
    try:
        eng.set_kernel("default", variant=variant)
        _after_seal(eng, 65536, np.full(65536, 1420, np.int64), 1, uniform=True)
    finally:
        eng.close()


@pytest.mark.parametrize("n,L", [(1, 0), (31, 64), (33, 1420), (1000, 577), (4097, 1420)])
def test_after_seal_ragged_sizes(n, L):
    W = wg()
    eng = W.Engine(0, key_slots=8)
    try:
        _after_seal(eng, n, np.full(n, L, np.int64), 8, uniform=True)
    finally:
        eng.close()


@pytest.mark.parametrize("n", [3000, 30000, 40000])
@pytest.mark.parametrize("plan", [None, "WG_SLOT16=0", "WG_SLOT16=1", "WG_MIXED_SPLIT=4", "WG_SLOT4=1", "WG_SLOT4=2"])
def test_after_seal_mixed_lengths(n, plan, monkeypatch):
    """Mixed lengths, ordered longest-first once for both halves. plan None: the size-based plan
    (3000 packets: one per slot, 16-lane slots above one round; 40000: 16-lane longest-first
    pairs); the others force 8-lane pairs, 16-lane pairs, a split at 4 rounds, 4-lane slots or
    the long packets in 16-lane and the rest in 4-lane slots (read when the context is created; 30000 packets in 4-lane slots are 1875 waves, so the second,
    partial generation of 1024 waves takes its positions reversed)."""
    for var in ("WG_SLOT16", "WG_MIXED_SPLIT", "WG_SLOT4"):
        monkeypatch.delenv(var, raising=False)
    if plan:
        k, v = plan.split("=")
        monkeypatch.setenv(k, v)
    W = wg()
    eng = W.Engine(0, key_slots=16)
    try:
        lens = (64 + splitmix_np(77, 4 * n).view("<u4") % 3000).astype(np.int64)
        _after_seal(eng, n, lens, 16, uniform=False)
    finally:
        eng.close()


def test_after_seal_argument_contract():
    torch, dev = _dev()
    W = wg()
    eng = W.Engine(0, key_slots=1)
    try:
        d = torch.zeros((4, 4), dtype=torch.int64, device=dev)
        b = torch.zeros(64, dtype=torch.uint8, device=dev)
        st = torch.zeros(3, dtype=torch.int32, device=dev)
        with pytest.raises(W.WgError):  # unequal sizes
            eng.duplex(d, b, b, 0, d[:3], b, b, st, 0, uniform=True, after_seal=True)
    finally:
        eng.close()
