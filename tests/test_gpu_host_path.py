"""Host-to-host transport path (BASELINE configs[4]): batches that
start and end in host memory, through wg_seal_host / wg_open_host.

Pageable numpy buffers take the chunked copy pipeline (H2D / kernel / D2H overlapped);
pinned buffers from wg_host_alloc take the zero-copy path (the kernel reads and writes
the rings over PCIe). Both must be bit-exact with the oracle and must leave the bytes
between packets (wire headers, ring slack) untouched."""
import numpy as np
import pytest

from wgtest import oracle, splitmix_np

pytestmark = pytest.mark.gpu
O = oracle()
SENTINEL = 0xA5


def wire_rings(n, L, seed):
    """tun ring: plaintext at a 1440-B stride; UDP ring: 16-B header then ct||tag at a
    1452-B stride (TransportPacket.java:30-35)."""
    tun_stride, wire = 1440, 16 + L + 16
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * tun_stride
    desc["out_off"] = np.arange(n, dtype=np.uint64) * wire + 16
    desc["counter"] = np.arange(n, dtype=np.uint64) + 1000
    desc["len"] = L
    keys = splitmix_np(seed, 32)
    tun = splitmix_np(seed + 1, n * tun_stride)
    return desc, keys, tun, n * wire


def check_open(engine, desc, keys, sealed, tun_size, alloc, tamper):
    od = desc.copy()
    od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
    bad = sealed.copy()
    for i in tamper:
        bad[int(desc["out_off"][i]) + int(desc["len"][i])] ^= 0x10
    src = alloc(len(bad))
    src[:] = bad
    back = alloc(tun_size)
    back[:] = SENTINEL
    st = engine.open_host(od, src, back, int(desc["len"].max()), uniform=len(set(desc["len"].tolist())) == 1)
    exp = np.zeros(len(desc), np.uint32)
    exp[list(tamper)] = 1
    assert np.array_equal(st, exp)
    return back


@pytest.mark.parametrize("pinned", [False, True])
def test_wire_rings_multi_chunk(engine, pinned):
    """16384 x 1420 B (24 MB, several pipeline chunks) tun ring -> UDP ring and back."""
    n, L = 16384, 1420
    desc, keys, tun, wire_size = wire_rings(n, L, seed=71 + pinned)
    engine.set_keys(0, keys.tobytes())
    pinned_bufs = []

    def alloc(nb):
        if pinned:
            a = engine.host_alloc(nb)
            pinned_bufs.append(a)
            return a
        return np.empty(nb, np.uint8)

    try:
        src = alloc(len(tun))
        src[:] = tun
        ring = alloc(wire_size)
        ring[:] = SENTINEL
        engine.seal_host(desc, src, ring, L, uniform=True)
        ref = np.full(wire_size, SENTINEL, np.uint8)
        O.seal_batch(desc, tun, ref, keys, threads=8)
        assert np.array_equal(ring, ref)  # packets bit-exact, headers untouched
        back = check_open(engine, desc, keys, np.array(ring), len(tun), alloc, tamper=[3, 9000])
        exp = tun.copy()
        for i in range(n):  # the 20 B of slack per tun slot keep the sentinel; bad packets are zero
            o = int(desc["in_off"][i])
            exp[o + L:o + 1440] = SENTINEL
            if i in (3, 9000):
                exp[o:o + L] = 0
        assert np.array_equal(back, exp)
    finally:
        for a in pinned_bufs:
            engine.host_free(a)


def test_mixed_lengths_gapped_layout(engine):
    """C2-like mix (64..9000 B, 256 keys) with gaps between packets: range copies with
    the gaps staged, several chunks."""
    n = 3000
    lengths = (64 + splitmix_np(5, 4 * n).view("<u4") % (9000 - 64 + 1)).astype(np.int64)
    in_stride = (lengths + 15) // 16 * 16 + 32
    out_stride = lengths + 16 + 48
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.concatenate([[0], np.cumsum(in_stride)[:-1]]).astype(np.uint64)
    desc["out_off"] = np.concatenate([[0], np.cumsum(out_stride)[:-1]]).astype(np.uint64) + 7
    desc["counter"] = np.arange(n, dtype=np.uint64) // 256
    desc["len"] = lengths
    desc["key_slot"] = np.arange(n) % 256
    keys = splitmix_np(6, 32 * 256)
    engine.set_keys(0, keys.tobytes())
    inp = splitmix_np(7, int(in_stride.sum()))
    out_size = int(out_stride.sum()) + 7
    out = np.full(out_size, SENTINEL, np.uint8)
    engine.seal_host(desc, inp, out, 9000)
    ref = np.full(out_size, SENTINEL, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=8)
    assert np.array_equal(out, ref)
    back = check_open(engine, desc, keys, out, len(inp), lambda nb: np.empty(nb, np.uint8), tamper=[0, 2999])
    for i in range(0, n, 5):
        o, l = int(desc["in_off"][i]), int(lengths[i])
        if i in (0, 2999):
            assert not back[o:o + l].any()
        else:
            assert np.array_equal(back[o:o + l], inp[o:o + l])
        assert (back[o + l:o + int(in_stride[i])] == SENTINEL).all()


def test_non_monotone_descriptors_single_chunk(engine):
    """Descriptors in reverse buffer order cannot be pipelined safely: still exact."""
    n, L = 8192, 1420
    desc, keys, tun, wire_size = wire_rings(n, L, seed=90)
    desc = desc[::-1].copy()
    engine.set_keys(0, keys.tobytes())
    ring = np.full(wire_size, SENTINEL, np.uint8)
    engine.seal_host(desc, tun, ring, L, uniform=True)
    ref = np.full(wire_size, SENTINEL, np.uint8)
    O.seal_batch(desc, tun, ref, keys, threads=8)
    assert np.array_equal(ring, ref)
