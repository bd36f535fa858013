"""Parity of the HIP path (through the C-ABI) with the oracle and with the
reference's own known-answer tests. Runs on an MI355X (pytest -m gpu)."""
import hashlib
import json
import os

import numpy as np
import pytest

from wgtest import ROOT, noise, oracle, splitmix_bytes, splitmix_np, wg

pytestmark = pytest.mark.gpu
O = oracle()
V = json.load(open(os.path.join(ROOT, "tests/golden/reference_vectors.json")))
T = json.load(open(os.path.join(ROOT, "tests/golden/transport_vectors.json")))
h = bytes.fromhex


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


# ---- the reference's own tests, through the mirrored API -------------------------

def test_selftest_on_device():
    assert wg().selftest(0)  # Poly1305.<clinit> power-on self test convention


def test_chacha20_block_rfc():
    n = noise()
    v = V["chacha20_block"]  # ChaCha20Test.chacha20Block
    state = bytearray(64)
    n.ChaCha20.initializeState(h(v["key"]), h(v["nonce"]), state, 1)
    out = bytearray(64)
    n.ChaCha20.chacha20Block(state, out, 1)
    assert bytes(out) == h(v["out"])


def test_chacha20_rfc():
    n = noise()
    v = V["chacha20"]  # ChaCha20Test.chacha20 (sunscreen, counter 1)
    out = bytearray(len(h(v["pt"])))
    n.ChaCha20.chacha20(h(v["key"]), h(v["nonce"]), h(v["pt"]), out, 1)
    assert bytes(out) == h(v["ct"])


def test_chacha20_matches_independent_cipher():
    n = noise()  # ChaCha20Test.testMatchesCipher: counter 0, zero nonce, random key
    key = splitmix_bytes(99, 32)
    pt = V["chacha20"]["pt"]
    out = bytearray(len(h(pt)))
    n.ChaCha20.chacha20(key, bytes(12), h(pt), out, 0)
    assert bytes(out) == O.py_chacha20(key, bytes(12), 0, h(pt))


def test_poly1305_rfc():
    n = noise()
    v = V["poly1305"]  # Poly1305Test.testPoly1305
    p = n.Poly1305()
    p.init(h(v["key"]))
    p.update(h(v["msg"]))
    assert p.finish() == h(v["tag"])
    with pytest.raises(n.IllegalStateException):
        p.update(b"x")


def test_poly1305_donna_selftest_vectors():
    n = noise()
    nacl = V["donna_nacl"]
    msg = h(nacl["msg"])
    p = n.Poly1305()
    p.init(h(nacl["key"]))
    for a, b in [(0, 32), (32, 96), (96, 112), (112, 120), (120, 124), (124, 126), (126, 127), (127, 128),
                 (128, 129), (129, 130), (130, 131)]:  # poly1305-donna.c:167-179 split updates
        p.update(msg[a:b])
    assert p.finish() == h(nacl["tag"])
    w = V["donna_wrap"]
    p.init(h(w["key"])); p.update(h(w["msg"]))
    assert p.finish() == h(w["tag"])
    total = n.Poly1305()
    total.init(h(V["donna_total"]["key"]))
    for i in range(256):
        q = n.Poly1305(); q.init(bytes([i]) * 32); q.update(bytes([i]) * i)
        total.update(q.finish())
    assert total.finish() == h(V["donna_total"]["tag"])


def test_poly1305_keygen_rfc():
    n = noise()
    v = V["poly1305_keygen"]
    assert n.ChaCha20Poly1305.poly1305ChaChaKeyGen(h(v["key"]), h(v["nonce"])) == h(v["otk"])


def test_aead_encrypt_rfc():
    n = noise()
    v = V["aead"]  # Poly1305Test.poly1305AeadEncrypt
    ct = bytearray(len(h(v["pt"])))
    tag = bytearray(16)
    n.ChaCha20Poly1305.poly1305AeadEncrypt(h(v["aad"]), h(v["key"]), h(v["nonce"]), h(v["pt"]), ct, tag)
    assert bytes(ct) == h(v["ct"]) and bytes(tag) == h(v["tag"])


def test_aead_decrypt_roundtrip_and_tamper():
    n = noise()  # Poly1305Test.poly1305AeadDecrypt
    pt = h(V["aead"]["pt"])
    aad = b"Cryptographic Forum Research Group"
    key, nonce = splitmix_bytes(5, 32), splitmix_bytes(6, 12)
    ct, tag = bytearray(len(pt)), bytearray(16)
    n.ChaCha20Poly1305.poly1305AeadEncrypt(aad, key, nonce, pt, ct, tag)
    res = bytearray(len(pt))
    n.ChaCha20Poly1305.poly1305AeadDecrypt(aad, key, nonce, bytes(ct), res, bytes(tag))
    assert bytes(res) == pt
    tag[0] ^= 0x01
    res2 = bytearray(b"\xaa" * len(pt))
    with pytest.raises(n.AEADBadTagException):
        n.ChaCha20Poly1305.poly1305AeadDecrypt(aad, key, nonce, bytes(ct), res2, bytes(tag))
    assert bytes(res2) == b"\xaa" * len(pt)  # untouched on failure


# ---- SymmetricKeypair: the drop-in boundary ----------------------------------------

def test_symmetric_keypair_roundtrip_and_nonce_layout():
    n = noise()
    k1, k2 = splitmix_bytes(11, 32), splitmix_bytes(12, 32)
    a = n.SymmetricKeypair(k1, k2)
    b = n.SymmetricKeypair(k2, k1)
    for i, L in enumerate([0, 1, 16, 63, 64, 65, 1420, 2032]):
        pt = splitmix_bytes(100 + i, L)
        dst = bytearray(L + 16)
        c = a.cipher(pt, dst)
        assert c == i  # counters start at 0 (SymmetricKeypair.java:37,64)
        assert bytes(dst) == O.py_aead_seal(k1, O.transport_nonce(c), pt)
        out = bytearray(L)
        b.decipher(c, bytes(dst), out)
        assert bytes(out) == pt
        with pytest.raises(n.BadPaddingException):
            b.decipher(c + 1, bytes(dst), bytearray(L))
    with pytest.raises(IndexError):
        b.decipher(0, b"\x00" * 15, bytearray(1))
    a.clean(); b.clean()


# ---- device batches vs the oracle ----------------------------------------------------

def make_batch(n, lengths, nkeys, seed, in_align=16, out_pad=16, tag_in=False):
    lengths = np.asarray(lengths, np.int64)
    in_sz = lengths + (16 if tag_in else 0)
    in_stride = (in_sz + in_align - 1) // in_align * in_align
    in_off = np.concatenate([[0], np.cumsum(in_stride)[:-1]]).astype(np.uint64)
    out_sz = lengths + 16 + out_pad
    out_off = np.concatenate([[0], np.cumsum(out_sz)[:-1]]).astype(np.uint64)
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"], desc["out_off"] = in_off, out_off
    desc["counter"] = splitmix_np(seed, 8 * n).view("<u8")
    desc["len"] = lengths
    desc["key_slot"] = np.arange(n) % nkeys
    keys = splitmix_np(seed + 1, 32 * nkeys)
    inp = splitmix_np(seed + 2, int(in_stride.sum()) + 64)
    return desc, keys, inp, int(out_sz.sum()) + 64


def run_device(engine, torch, desc, keys, inp, out_size, open_=False, uniform=False, max_len=None):
    W = wg()
    engine.set_keys(0, keys.tobytes())
    dev = torch.device("cuda", 0)
    dt = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    it = torch.from_numpy(inp).to(dev)
    ot = torch.zeros(out_size, dtype=torch.uint8, device=dev)
    ml = int(desc["len"].max()) if max_len is None else max_len
    if open_:
        st = torch.full((len(desc),), 7, dtype=torch.int32, device=dev)
        engine.open(dt, it, ot, st, ml, uniform=uniform)
        torch.cuda.synchronize()
        return ot.cpu().numpy(), st.cpu().numpy()
    engine.seal(dt, it, ot, ml, uniform=uniform)
    torch.cuda.synchronize()
    return ot.cpu().numpy(), None


@pytest.mark.parametrize("uniform", [True, False])
@pytest.mark.parametrize("L", [0, 1, 63, 64, 65, 1420, 4080])
def test_seal_open_uniform_lengths(engine, torch_dev, L, uniform):
    n = 300
    desc, keys, inp, out_size = make_batch(n, [L] * n, 3, seed=L + 17)
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size, uniform=uniform)
    ref = np.zeros(out_size, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=8)
    assert np.array_equal(sealed, ref)
    # open what we sealed (ct||tag now at out_off), flip one tag bit in packet 7
    od = desc.copy()
    od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
    tampered = sealed.copy()
    if n > 7:
        tampered[int(desc["out_off"][7]) + L] ^= 0x40
    pt, st = run_device(engine, torch_dev, od, keys, tampered, len(inp), open_=True, uniform=uniform)
    exp_status = np.zeros(n, np.int32); exp_status[7] = 1
    assert np.array_equal(st, exp_status)
    for i in range(n):
        o, l = int(desc["in_off"][i]), int(desc["len"][i])
        if i == 7:
            assert not pt[o:o + l].any()  # unauthenticated plaintext scrubbed
        else:
            assert np.array_equal(pt[o:o + l], inp[o:o + l])


def test_transport_golden_vectors_on_device(engine, torch_dev):
    cases = T["cases"]
    n = len(cases)
    lengths = [c["len"] for c in cases]
    desc, _, _, out_size = make_batch(n, lengths, n, seed=1)
    keys = np.frombuffer(b"".join(h(c["key"]) for c in cases), np.uint8).copy()
    desc["key_slot"] = np.arange(n)
    desc["counter"] = np.array([c["counter"] for c in cases], dtype=np.uint64)
    inp = np.zeros(int(desc["in_off"][-1]) + lengths[-1] + 64, np.uint8)
    for i, c in enumerate(cases):
        o = int(desc["in_off"][i])
        inp[o:o + c["len"]] = np.frombuffer(splitmix_bytes(c["pt_seed"], c["len"]), np.uint8)
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size)
    for i, c in enumerate(cases):
        o = int(desc["out_off"][i])
        got = sealed[o:o + c["len"] + 16].tobytes()
        assert hashlib.sha256(got).hexdigest() == c["sha256"], (i, c["len"], c["counter"])


def test_mixed_sizes_many_keys(engine, torch_dev):
    """C2 shape at reduced n: lengths 64..9000, 256 session keys, per-packet key/nonce gather;
    two tampered tags among 6000 packets come back BADTAG with their plaintext scrubbed."""
    n = 6000
    lengths = 64 + splitmix_np(77, 4 * n).view("<u4") % (9000 - 64 + 1)
    desc, keys, inp, out_size = make_batch(n, lengths, 256, seed=5)
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size)
    ref = np.zeros(out_size, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=8)
    assert np.array_equal(sealed, ref)
    od = desc.copy()
    od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
    tampered = sealed.copy()
    bad = [123, 4321]
    for i in bad:
        tampered[int(desc["out_off"][i]) + int(desc["len"][i])] ^= 0x80
    pt, st = run_device(engine, torch_dev, od, keys, tampered, len(inp), open_=True)
    exp = np.zeros(n, np.int32)
    exp[bad] = 1
    assert np.array_equal(st, exp)
    for i in list(range(0, n, 7)) + bad:
        o, l = int(desc["in_off"][i]), int(desc["len"][i])
        want = np.zeros(l, np.uint8) if i in bad else inp[o:o + l]
        assert np.array_equal(pt[o:o + l], want), i


def test_unaligned_offsets_and_lengths(engine, torch_dev):
    n = 200
    lengths = splitmix_np(3, 4 * n).view("<u4") % 700
    desc, keys, inp, out_size = make_batch(n, lengths, 5, seed=9, in_align=1, out_pad=3)
    desc["in_off"] += 1  # every packet starts at an odd address
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size)
    ref = np.zeros(out_size, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=4)
    assert np.array_equal(sealed, ref)


def test_wire_format_layout(engine, torch_dev):
    """Packed wire packets: 16-byte header, ct||tag at +16 (TransportPacket.java:30-35), 1452-byte stride."""
    n, L = 256, 1420
    wire = 16 + L + 16
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * L
    desc["out_off"] = np.arange(n, dtype=np.uint64) * wire + 16
    desc["counter"] = np.arange(n, dtype=np.uint64)
    desc["len"] = L
    keys = splitmix_np(21, 32)
    inp = splitmix_np(22, n * L)
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, n * wire, uniform=True)
    ref = np.zeros(n * wire, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=4)
    assert np.array_equal(sealed, ref)


def test_out_of_range_descriptors_are_rejected(engine, torch_dev):
    n, L = 4, 100
    desc, keys, inp, out_size = make_batch(n, [L] * n, 1, seed=31)
    desc["in_off"][1] = len(inp) + 1000      # input past the buffer
    desc["key_slot"][2] = engine.key_slots   # key slot past the table
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size)
    ref = np.zeros(out_size, np.uint8)
    good = desc[[0, 3]]
    O.seal_batch(good, inp, ref, keys, threads=1)
    assert np.array_equal(sealed, ref)  # rejected packets leave their output untouched (zero)
    od = desc.copy()
    od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
    od["in_off"][1] = out_size + 5
    _, st = run_device(engine, torch_dev, od, keys, sealed, len(inp) + 2000, open_=True)
    assert st.tolist() == [0, 1, 1, 0]


def test_max_packet_and_empty_batch(engine, torch_dev):
    n = 2
    desc, keys, inp, out_size = make_batch(n, [65535, 0], 1, seed=41)
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size)
    ref = np.zeros(out_size, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=2)
    assert np.array_equal(sealed, ref)
    W = wg()
    import torch
    e = torch.zeros(0, 4, dtype=torch.int64, device="cuda")
    b = torch.zeros(16, dtype=torch.uint8, device="cuda")
    engine.seal(e, b, b, 1420, uniform=True)  # n = 0 is a no-op


def test_full_c1_roundtrip(engine, torch_dev):
    """BASELINE configs[1]: 65536 x 1420 B, one session key, counters 0..65535 — every packet bit-exact."""
    torch = torch_dev
    W = wg()
    n, L, S = 65536, 1420, 1440
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = desc["out_off"] = np.arange(n, dtype=np.uint64) * S
    desc["counter"] = np.arange(n, dtype=np.uint64)
    desc["len"] = L
    keys = splitmix_np(0x5EED2026, 32)
    inp = splitmix_np(0x5EED2027, n * S)
    sealed, _ = run_device(engine, torch, desc, keys, inp, n * S, uniform=True)
    ref = np.zeros(n * S, np.uint8)
    O.seal_batch(desc, inp, ref, keys, threads=16)
    assert np.array_equal(sealed, ref)
    pt, st = run_device(engine, torch, desc, keys, sealed, n * S, open_=True, uniform=True)
    assert not st.any()
    mask = np.zeros(S, bool); mask[:L] = True
    m = np.tile(mask, n)
    assert np.array_equal(pt[m], inp[m])


# ---- every selectable transport kernel (wg_ctx_set_kernel) --------------------------

KERNELS = [("transport", 0, 0), ("wave1", 0, 0), ("tile", 0, 0)]


@pytest.mark.parametrize("kern,lanes,variant", KERNELS)
def test_every_transport_kernel_bit_exact(torch_dev, kern, lanes, variant):
    """each selectable transport kernel (k_transport, the round-1 k_wave kept
    as the A/B baseline, k_tile) seals and opens
    bit-exact vs the oracle on a uniform 1420-B batch and on a mixed 0..3000-B batch (with
    and without WG_F_UNIFORM), and rejects a tampered tag (status BADTAG, plaintext
    scrubbed)."""
    W = wg()
    eng = W.Engine(0, key_slots=64)
    try:
        eng.set_kernel(kern, lanes, variant)
        mixed = list(splitmix_np(11, 4 * 777).view("<u4") % 3001)
        for case, (lengths, uniform) in enumerate([([1420] * 777, True), (mixed, False), (mixed, True)]):
            n = len(lengths)
            desc, keys, inp, out_size = make_batch(n, lengths, 64, seed=101 + case)
            sealed, _ = run_device(eng, torch_dev, desc, keys, inp, out_size, uniform=uniform)
            ref = np.zeros(out_size, np.uint8)
            O.seal_batch(desc, inp, ref, keys, threads=8)
            assert np.array_equal(sealed, ref), (kern, lanes, variant, case)
            od = desc.copy()
            od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
            tampered = sealed.copy()
            tampered[int(desc["out_off"][5]) + int(desc["len"][5])] ^= 0x01
            pt, st = run_device(eng, torch_dev, od, keys, tampered, len(inp), open_=True, uniform=uniform)
            exp = np.zeros(n, np.int32)
            exp[5] = 1
            assert np.array_equal(st, exp), (kern, case)
            for i in range(n):
                o, l = int(desc["in_off"][i]), int(desc["len"][i])
                want = np.zeros(l, np.uint8) if i == 5 else inp[o:o + l]
                assert np.array_equal(pt[o:o + l], want), (kern, case, i)
    finally:
        eng.close()


def test_set_kernel_rejects_unknown_names(engine):
    W = wg()
    with pytest.raises(W.WgError):
        engine.set_kernel("nope", 2, 0)
    with pytest.raises(W.WgError):
        engine.set_kernel("lane", 2, 0)  # round-1 experimental kernels are no longer in the library
    engine.set_kernel("default")


@pytest.mark.parametrize("it", range(10))
def test_randomized_batches_vs_oracle(engine, torch_dev, it):
    """Seeded random batches through the product kernel: random counts, lengths (some batches
    all equal), alignments, key slots, the WG_F_UNIFORM hint either way, ~3% descriptors out
    of range (input past the buffer, key slot past the table, len > max_len) and ~2% forged
    tags. Seal output must equal the oracle's for the valid packets and leave the rest
    untouched; open must report exactly the invalid and forged packets and zero-fill only
    the forged packets' plaintexts."""
    _randomized_batch(engine, torch_dev, it)


@pytest.mark.parametrize("it", [1, 2, 4, 5])
def test_randomized_batches_16_lane_slots(torch_dev, it, monkeypatch):
    """The same random mixed-length batches with 16-lane slots (WG_SLOT16=1: rounds of 16 blocks,
    4 slots per wave, 4-step r-power scan, 4-step slot sum)."""
    monkeypatch.setenv("WG_SLOT16", "1")
    eng = wg().Engine(0, key_slots=4096)
    try:
        _randomized_batch(eng, torch_dev, it)
    finally:
        eng.close()


@pytest.mark.parametrize("plan", ["1", "2"])
@pytest.mark.parametrize("it", [1, 2, 4, 5, 7])
def test_randomized_batches_4_lane_slots(torch_dev, it, plan, monkeypatch):
    """The same random mixed-length batches with 4-lane slots (rounds of 4 blocks, 16 slots per wave,
    descriptors as 8-B pairs per lane, 2-step r-power scan, 2-step slot sum). WG_SLOT4=1: every packet
    in a 4-lane slot; 2: packets of more than two 8-block rounds in 16-lane slots, the rest in 4-lane
    slots (k_*_mixed<4>, the size-based plan for large batches of packets up to 2048 B)."""
    monkeypatch.setenv("WG_SLOT4", plan)
    eng = wg().Engine(0, key_slots=4096)
    try:
        _randomized_batch(eng, torch_dev, it)
    finally:
        eng.close()


def _randomized_batch(engine, torch_dev, it):
    rng = np.random.default_rng(1000 + it)
    n = int(rng.integers(1, 2500))
    if it % 3 == 0:
        lengths = np.full(n, int(rng.integers(0, 3000)), np.int64)
    else:
        lengths = rng.integers(0, 3000, n).astype(np.int64)
    nkeys = int(rng.integers(1, 64))
    desc, keys, inp, out_size = make_batch(n, lengths, nkeys, seed=2000 + it,
                                           in_align=int(rng.choice([1, 4, 16])), out_pad=int(rng.choice([0, 3, 16])))
    desc["in_off"] += np.uint64(int(rng.integers(0, 4)))
    max_len = int(lengths.max())
    bad = rng.random(n) < 0.03
    kind = rng.integers(0, 3, n)
    for i in np.nonzero(bad)[0]:
        if kind[i] == 0:
            desc["in_off"][i] = len(inp) + 7
        elif kind[i] == 1:
            desc["key_slot"][i] = engine.key_slots + 3
        else:
            desc["len"][i] = max_len + 1
    uniform = bool(rng.integers(0, 2))
    sealed, _ = run_device(engine, torch_dev, desc, keys, inp, out_size, uniform=uniform, max_len=max_len)
    ref = np.zeros(out_size, np.uint8)
    good = np.nonzero(~bad)[0]
    if len(good):
        O.seal_batch(desc[good], inp, ref, keys, threads=8)
    assert np.array_equal(sealed, ref), it
    # open: ciphertext back to plaintext; forge ~2% of the valid packets' tags
    od = desc.copy()
    od["in_off"], od["out_off"] = desc["out_off"], desc["in_off"]
    forged = (~bad) & (rng.random(n) < 0.02)
    ct = sealed.copy()
    for i in np.nonzero(forged)[0]:
        ct[int(od["in_off"][i]) + int(od["len"][i])] ^= 0x80
    for i in np.nonzero(bad & (kind == 0))[0]:
        od["in_off"][i] = out_size + 7  # still out of range on the open side
    pt, st = run_device(engine, torch_dev, od, keys, ct, len(inp), open_=True, uniform=uniform, max_len=max_len)
    exp = (bad | forged).astype(np.int32)
    assert np.array_equal(st, exp), it
    for i in range(n):
        if bad[i]:
            continue
        o, L_ = int(desc["in_off"][i]), int(desc["len"][i])
        want = np.zeros(L_, np.uint8) if forged[i] else inp[o:o + L_]
        assert np.array_equal(pt[o:o + L_], want), (it, i)
