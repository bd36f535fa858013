"""Transport wire framing on device: wg_frame_seal writes the
16-B transport header in front of each sealed packet, wg_parse_open turns received
wire packets into open descriptors without a host parse.

Reference behaviour followed: TransportPacket.java:18-35 (header layout),
UnencryptedOutgoingTransport.java:14-18 and EncryptedOutgoingTransport.java:11-14
(type, receiver index, counter written on send), UndecryptedIncomingTransport.java:20-33
(type check, ctLen = packetLen - 16, plaintext right after the ciphertext, counter
from the header). The reference has no test vectors for the framing; the CPU tests pin
the oracle to the struct layout (native little-endian JAVA_INT / JAVA_LONG)."""
import struct

import numpy as np
import pytest

from wgtest import oracle, splitmix_np, wg

O = oracle()


def test_header_layout_matches_transport_packet():
    h = O.transport_header(0x11223344, 0x0102030405060708)
    assert len(h) == O.HEADER_SIZE == 16
    assert h[0] == 4 and h[1:4] == b"\x00\x00\x00"  # message_type, paddingLayout(3)
    assert h[4:8] == bytes([0x44, 0x33, 0x22, 0x11])  # receiver_index, LE u32
    assert h[8:16] == bytes(range(8, 0, -1))  # counter, LE u64
    assert O.transport_header(-1, -1)[4:] == b"\xff" * 12  # Java int / long wrap


def test_frame_then_parse_roundtrip_oracle():
    n, L, stride = 40, 100, 4096
    desc = np.zeros(n, O.WG_PKT)
    desc["out_off"] = np.arange(n, dtype=np.uint64) * stride + 16
    desc["counter"] = np.arange(n, dtype=np.uint64) * 7 + (1 << 40)
    desc["len"] = L
    desc["key_slot"] = np.arange(n) % 3
    receivers = np.array([5, 0xFFFFFFFF, 123456], np.uint32)
    wire = np.zeros(n * stride, np.uint8)
    O.frame_headers(desc, receivers, wire, key_slots=3)
    off = desc["out_off"].astype(np.uint64) - 16
    wl = np.full(n, 16 + L + 16, np.uint32)
    pd, st = O.parse_wire(wire, off, wl, desc["key_slot"])
    assert not st.any()
    assert np.array_equal(pd["counter"], desc["counter"])
    assert np.array_equal(pd["in_off"], desc["out_off"])
    assert np.array_equal(pd["len"], desc["len"])
    assert np.array_equal(pd["out_off"], off + wl)
    for i in range(n):
        rx = struct.unpack_from("<I", wire[int(off[i]) + 4:int(off[i]) + 8].tobytes())[0]
        assert rx == receivers[i % 3]


def test_parse_rejects_bad_type_short_and_overrun_oracle():
    wire = np.zeros(3 * 4096, np.uint8)
    for o in (0, 4096, 8192):
        wire[o:o + 16] = np.frombuffer(O.transport_header(1, 9), np.uint8)
    wire[4096] = 1  # handshake initiation type
    off = np.array([0, 4096, 8192, 8192], np.uint64)
    wl = np.array([31, 64, 64, 4096], np.uint32)  # short; bad type; ok; plaintext overruns
    pd, st = O.parse_wire(wire, off, wl, np.zeros(4, np.uint32))
    assert st.tolist() == [2, 2, 0, 2]
    assert pd["len"].tolist() == [0xFFFFFFFF, 0xFFFFFFFF, 32, 0xFFFFFFFF]


# ---- device parity (MI355X) --------------------------------------------------------

@pytest.mark.gpu
def test_device_frame_seal_and_parse_open(engine):
    """Seal + frame 2000 mixed-length packets into a UDP ring at 4096-B slots, check every
    byte of the ring against the oracle, then parse + open the ring on device (plaintext
    lands after each ciphertext, as the reference's incoming buffers hold it), with
    tampered tags and malformed headers mixed in."""
    import torch
    W = wg()
    dev = torch.device("cuda", 0)
    n, slot, nkeys = 2000, 4096, 16
    rng = np.random.default_rng(2026)
    lens = rng.integers(0, 2033, n).astype(np.uint32)  # L <= 2032 fits the 4096-B incoming buffer
    lens[:4] = [0, 1, 2032, 1420]
    keys = splitmix_np(901, 32 * nkeys)
    tun = splitmix_np(902, n * 2048)
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * 2048
    desc["out_off"] = np.arange(n, dtype=np.uint64) * slot + 16
    desc["counter"] = splitmix_np(903, 8 * n).view("<u8") >> np.uint64(8)
    desc["len"] = lens
    desc["key_slot"] = np.arange(n) % nkeys
    receivers = splitmix_np(904, 4 * engine.key_slots).view("<u4").copy()

    engine.set_keys(0, keys.tobytes())
    dt = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    rt = torch.from_numpy(receivers.view(np.int32)).to(dev)
    ring = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    engine.seal(dt, torch.from_numpy(tun).to(dev), ring, 2032)
    engine.frame_seal(dt, rt, ring, in_size=tun.size, max_len=2032)
    torch.cuda.synchronize()
    got = ring.cpu().numpy()

    ref = np.zeros(n * slot, np.uint8)
    O.seal_batch(desc, tun, ref, keys, threads=8)
    O.frame_headers(desc, receivers, ref, key_slots=engine.key_slots, in_size=tun.size, max_len=2032)
    assert np.array_equal(got, ref)

    # inbound: tamper 1% of tags, corrupt 3 type bytes, give one packet an overrunning length
    rx_wire = got.copy()
    tamper = rng.choice(np.arange(10, n), 20, replace=False)
    for i in tamper:
        rx_wire[int(desc["out_off"][i]) + int(lens[i])] ^= 0x01
    badtype = [4, 5, 6]
    for i in badtype:
        rx_wire[i * slot] = 3
    off = np.arange(n, dtype=np.uint64) * slot
    wl = (lens + 32).astype(np.uint32)
    wl[7] = slot  # plaintext would run past the end of its slot... and of the ring for the last one
    wl[n - 1] = slot
    exp_desc, exp_pst = O.parse_wire(rx_wire, off, wl, desc["key_slot"].astype(np.uint32))

    wt = torch.from_numpy(rx_wire).to(dev)
    od = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    pst = torch.full((n,), 9, dtype=torch.int32, device=dev)
    engine.parse_open(wt, torch.from_numpy(off.view(np.int64)).to(dev), torch.from_numpy(wl.view(np.int32)).to(dev),
                      torch.from_numpy(desc["key_slot"].astype(np.int32)).to(dev), od, pst)
    torch.cuda.synchronize()
    assert np.array_equal(od.cpu().numpy(), W.desc_as_int64(exp_desc))
    assert np.array_equal(pst.cpu().numpy().view(np.uint32), exp_pst)

    st = torch.full((n,), 9, dtype=torch.int32, device=dev)
    engine.open(od, wt, wt, st, 2032)  # in place: ciphertext and plaintext ranges of one ring
    torch.cuda.synchronize()
    # oracle open over the packets wg_open_batch accepts; the rest (parse rejects, and
    # packet 7 whose 4064-B ciphertext exceeds max_len) are skipped with WG_PKT_BADTAG
    take = np.nonzero((exp_pst == 0) & (exp_desc["len"] <= 2032))[0]
    exp_st = np.ones(n, np.uint32)
    exp_st[take] = O.open_batch(exp_desc[take].copy(), rx_wire, rx_wire.copy(), keys, threads=8)
    assert np.array_equal(st.cpu().numpy().view(np.uint32), exp_st)
    # wg_open_batch reports every skipped (malformed) packet as a bad tag
    assert set(np.nonzero(exp_st)[0].tolist()) == set(tamper.tolist()) | set(badtype) | {7, n - 1}
    opened = wt.cpu().numpy()
    good = [i for i in range(n) if exp_st[i] == 0]
    for i in good[:200] + good[-200:]:
        o = int(off[i]) + int(wl[i])
        assert np.array_equal(opened[o:o + int(lens[i])], tun[i * 2048:i * 2048 + int(lens[i])])


def test_framing_entry_points_reject_null_context():
    """Argument checks run before any HIP call, so they hold on a CPU-only host too."""
    W = wg()
    lib = W.lib()
    assert lib.wg_frame_seal(None, None, 1, None, None, 0, 0, 0, None) == W._lib.WG_EINVAL
    assert lib.wg_parse_open(None, None, 0, None, None, None, 1, None, None, None) == W._lib.WG_EINVAL
    assert b"context" in lib.wg_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["transport", "wave1", "tile"])
def test_device_seal_with_frame_flag(engine, kernel):
    """WG_F_FRAME: the seal kernel, then k_frame_seal on the same stream; the same ring
    bytes whichever transport kernel sealed."""
    import torch
    W = wg()
    dev = torch.device("cuda", 0)
    n, slot, nkeys = 3000, 1536, 8
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 1489, n).astype(np.uint32)
    keys = splitmix_np(911, 32 * nkeys)
    tun = splitmix_np(912, n * 1504)
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * 1504
    desc["out_off"] = np.arange(n, dtype=np.uint64) * slot + 16 + (np.arange(n, dtype=np.uint64) % 3)  # 4-B and 1-B aligned headers
    desc["counter"] = np.arange(n, dtype=np.uint64) * 3 + (1 << 33)
    desc["len"] = lens
    desc["key_slot"] = np.arange(n) % nkeys
    receivers = splitmix_np(913, 4 * engine.key_slots).view("<u4").copy()
    rt = torch.from_numpy(receivers.view(np.int32)).to(dev)
    engine.set_keys(0, keys.tobytes())
    engine.set_kernel(kernel)
    try:
        engine.set_receivers(rt)
        ring = torch.zeros(n * slot + 64, dtype=torch.uint8, device=dev)
        engine.seal(torch.from_numpy(W.desc_as_int64(desc)).to(dev), torch.from_numpy(tun).to(dev), ring, 1488,
                    frame=True)
        torch.cuda.synchronize()
    finally:
        engine.set_kernel("default")
        engine.set_receivers(None)
    ref = np.zeros(n * slot + 64, np.uint8)
    O.seal_batch(desc, tun, ref, keys, threads=8)
    O.frame_headers(desc, receivers, ref, key_slots=engine.key_slots, in_size=tun.size, max_len=1488)
    assert np.array_equal(ring.cpu().numpy(), ref)


@pytest.mark.gpu
def test_frame_flag_needs_receiver_table(engine):
    """seal(frame=True) without wg_ctx_set_receivers is refused (WG_EINVAL) before any launch,
    and the host path refuses WG_F_FRAME instead of ignoring it."""
    import torch
    W = wg()
    dev = torch.device("cuda", 0)
    engine.set_receivers(None)
    d = torch.from_numpy(W.desc_as_int64(W.pack_desc([0], [16], [0], 10, 0))).to(dev)
    buf = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(W.WgError) as e:
        engine.seal(d, buf, buf, 10, frame=True)
    assert e.value.code == W._lib.WG_EINVAL
    lib = W.lib()
    hd = W.pack_desc([0], [16], [0], 10, 0)
    hb = np.zeros(64, np.uint8)
    assert lib.wg_seal_host(engine.ctx, hd.ctypes.data, 1, hb.ctypes.data, 64, hb.ctypes.data, 64, 10,
                            W._lib.WG_F_FRAME) == W._lib.WG_EINVAL


@pytest.mark.gpu
def test_frame_flag_leaves_rejected_packets_untouched(engine):
    """A packet the seal skips (len > max_len, input or output range outside its buffer,
    key slot past the table) gets no header either: its 16 header bytes keep their value."""
    import torch
    W = wg()
    dev = torch.device("cuda", 0)
    n, slot, L = 6, 256, 100
    keys = splitmix_np(931, 32)
    tun = splitmix_np(932, n * 128)
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * 128
    desc["out_off"] = np.arange(n, dtype=np.uint64) * slot + 16
    desc["counter"] = np.arange(n, dtype=np.uint64) + 5
    desc["len"] = L
    desc["len"][1] = 120                   # > max_len
    desc["in_off"][2] = tun.size - 50      # input runs past the end of `in`
    desc["out_off"][3] = n * slot - 40     # ct||tag runs past the end of `out`
    desc["key_slot"][4] = engine.key_slots  # no such key slot
    receivers = np.arange(engine.key_slots, dtype=np.uint32) + 1000
    engine.set_keys(0, keys.tobytes())
    engine.set_receivers(torch.from_numpy(receivers.view(np.int32)).to(dev))
    try:
        ring = torch.full((n * slot,), 0xA5, dtype=torch.uint8, device=dev)
        engine.seal(torch.from_numpy(W.desc_as_int64(desc)).to(dev), torch.from_numpy(tun).to(dev), ring, L,
                    frame=True)
        torch.cuda.synchronize()
    finally:
        engine.set_receivers(None)
    got = ring.cpu().numpy()
    ref = np.full(n * slot, 0xA5, np.uint8)
    O.seal_batch(desc[[0, 5]].copy(), tun, ref, keys, threads=1)
    O.frame_headers(desc, receivers, ref, key_slots=engine.key_slots, in_size=tun.size, max_len=L)
    assert np.array_equal(got, ref)
    for i in (1, 2, 3, 4):
        o = int(desc["out_off"][i])
        assert (got[o - 16:o] == 0xA5).all(), i


@pytest.mark.gpu
def test_receiver_table_is_validated(engine):
    """wg_ctx_set_receivers refuses a table shorter than the key table or not in device memory."""
    import torch
    W = wg()
    with pytest.raises(W.WgError):
        engine.set_receivers(torch.zeros(engine.key_slots - 1, dtype=torch.int32, device="cuda"))
    with pytest.raises(W.WgError):
        engine.set_receivers(torch.zeros(engine.key_slots, dtype=torch.int32))  # host tensor
    lib = W.lib()
    host = np.zeros(engine.key_slots, np.uint32)
    assert lib.wg_ctx_set_receivers(engine.ctx, host.ctypes.data, engine.key_slots) == W._lib.WG_EINVAL
