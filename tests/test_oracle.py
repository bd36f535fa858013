"""The CPU oracle (oracle/) pinned against the reference's own known-answer
vectors, and against OpenSSL for the transport nonce layout. No GPU needed."""
import json
import os
import struct

import numpy as np
import pytest

from wgtest import ROOT, oracle, splitmix_bytes, splitmix_np

O = oracle()
V = json.load(open(os.path.join(ROOT, "tests/golden/reference_vectors.json")))
T = json.load(open(os.path.join(ROOT, "tests/golden/transport_vectors.json")))
h = bytes.fromhex


def test_chacha20_state_layout():
    v = V["chacha20_state"]  # ChaCha20Test.initializeState
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(struct.unpack("<8I", h(v["key"])))
    s += [v["counter"]] + list(struct.unpack("<3I", h(v["nonce"])))
    assert s == v["words"]


def test_quarter_round_vectors():
    v = V["quarter_round"]  # ChaCha20Test.quarterRound (RFC 8439 2.1.1 / 2.2.1)
    a, b, c, d = v["qr_in"]
    M = 0xFFFFFFFF
    rotl = lambda x, n: ((x << n) | (x >> (32 - n))) & M
    a = (a + b) & M; d = rotl(d ^ a, 16); c = (c + d) & M; b = rotl(b ^ c, 12)
    a = (a + b) & M; d = rotl(d ^ a, 8); c = (c + d) & M; b = rotl(b ^ c, 7)
    assert [a, b, c, d] == v["qr_out"]


@pytest.mark.parametrize("impl", ["py", "c"])
def test_chacha20_block_rfc(impl):
    v = V["chacha20_block"]
    f = O.py_chacha20_block if impl == "py" else O.c_chacha20_block
    assert f(h(v["key"]), v["counter"], h(v["nonce"])) == h(v["out"])


@pytest.mark.parametrize("impl", ["py", "c"])
def test_chacha20_rfc(impl):
    v = V["chacha20"]
    f = O.py_chacha20 if impl == "py" else O.c_chacha20
    assert f(h(v["key"]), h(v["nonce"]), v["counter"], h(v["pt"])) == h(v["ct"])


@pytest.mark.parametrize("impl", ["py", "c"])
@pytest.mark.parametrize("name", ["poly1305", "donna_nacl", "donna_wrap"])
def test_poly1305_vectors(impl, name):
    v = V[name]
    f = O.py_poly1305 if impl == "py" else O.c_poly1305
    assert f(h(v["key"]), h(v["msg"])) == h(v["tag"])


@pytest.mark.parametrize("impl", ["py", "c"])
def test_poly1305_donna_total(impl):
    """MAC of the MACs of i-byte messages of value i under key i^32, i = 0..255 (poly1305-donna.c:136-198)."""
    f = O.py_poly1305 if impl == "py" else O.c_poly1305
    macs = b"".join(f(bytes([i]) * 32, bytes([i]) * i) for i in range(256))
    assert f(h(V["donna_total"]["key"]), macs) == h(V["donna_total"]["tag"])


def test_keygen_rfc():
    v = V["poly1305_keygen"]
    assert O.py_poly1305_keygen(h(v["key"]), h(v["nonce"])) == h(v["otk"])


@pytest.mark.parametrize("impl", ["py", "c"])
def test_aead_rfc(impl):
    v = V["aead"]
    seal = O.py_aead_seal if impl == "py" else O.c_aead_seal
    opn = O.py_aead_open if impl == "py" else O.c_aead_open
    ct_tag = seal(h(v["key"]), h(v["nonce"]), h(v["pt"]), h(v["aad"]))
    assert ct_tag == h(v["ct"]) + h(v["tag"])
    assert opn(h(v["key"]), h(v["nonce"]), ct_tag, h(v["aad"])) == h(v["pt"])
    bad = bytearray(ct_tag); bad[-16] ^= 1  # Poly1305Test.poly1305AeadDecrypt: 1-bit tag flip
    assert opn(h(v["key"]), h(v["nonce"]), bytes(bad), h(v["aad"])) is None


def test_transport_nonce_layout():
    # SymmetricKeypair.getNonceBytes: JAVA_LONG little-endian at offset 0, 4 zero bytes after
    assert O.transport_nonce(0x0102030405060708) == bytes([8, 7, 6, 5, 4, 3, 2, 1, 0, 0, 0, 0])
    assert O.transport_nonce((1 << 64) - 1) == b"\xff" * 8 + b"\x00" * 4


def test_transport_golden_vectors():
    import hashlib
    assert T["openssl_checked"]
    for c in T["cases"]:
        key = h(c["key"])
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        ct_tag = O.c_aead_seal(key, O.transport_nonce(c["counter"]), pt)
        assert hashlib.sha256(ct_tag).hexdigest() == c["sha256"], c
        assert ct_tag[-16:].hex() == c["tag"]
        if "ct_tag" in c:
            assert ct_tag.hex() == c["ct_tag"]


def test_openssl_cross_check_random():
    if O.openssl() is None:
        pytest.skip("libcrypto not present")
    for i, L in enumerate([0, 1, 15, 16, 17, 63, 64, 65, 1420, 9000]):
        key = splitmix_bytes(100 + i, 32)
        pt = splitmix_bytes(200 + i, L)
        n = O.transport_nonce(splitmix_np(300 + i, 8).view("<u8")[0])
        assert O.c_aead_seal(key, n, pt) == O.openssl_seal(key, n, pt)


def test_py_and_c_agree_with_aad():
    for L, A in [(0, 0), (0, 5), (1, 16), (33, 17), (200, 300)]:
        key, nonce = splitmix_bytes(L * 3 + A, 32), splitmix_bytes(L + 7 * A, 12)
        pt, aad = splitmix_bytes(L + 1, L), splitmix_bytes(A + 2, A)
        assert O.py_aead_seal(key, nonce, pt, aad or None) == O.c_aead_seal(key, nonce, pt, aad or None)


def _batch(n, L, nkeys, stride_in, stride_out, seed=1):
    desc = np.zeros(n, O.WG_PKT)
    desc["in_off"] = np.arange(n, dtype=np.uint64) * stride_in
    desc["out_off"] = np.arange(n, dtype=np.uint64) * stride_out
    desc["counter"] = np.arange(n, dtype=np.uint64)
    desc["len"] = L
    desc["key_slot"] = np.arange(n) % nkeys
    keys = splitmix_np(seed, 32 * nkeys)
    inp = splitmix_np(seed + 1, n * stride_in)
    return desc, keys, inp


def test_c_batch_roundtrip_and_tamper():
    n, L = 64, 1420
    desc, keys, inp = _batch(n, L, 4, 1440, 1440)
    sealed = np.zeros(n * 1440, np.uint8)
    O.seal_batch(desc, inp, sealed, keys, threads=4)
    for i in (0, 17, 63):  # spot check against the python restatement
        k = keys[32 * (i % 4):32 * (i % 4) + 32].tobytes()
        pt = inp[i * 1440:i * 1440 + L].tobytes()
        assert sealed[i * 1440:i * 1440 + L + 16].tobytes() == O.py_aead_seal(k, O.transport_nonce(i), pt)
    sealed[5 * 1440 + L] ^= 0x80  # tag flip on packet 5
    out = np.zeros(n * 1440, np.uint8)
    st = O.open_batch(desc, sealed, out, keys, threads=3)
    assert st.tolist() == [1 if i == 5 else 0 for i in range(n)]
    for i in range(n):
        got = out[i * 1440:i * 1440 + L]
        if i == 5:
            assert not got.any()  # untouched (zero) on failure
        else:
            assert np.array_equal(got, inp[i * 1440:i * 1440 + L])
