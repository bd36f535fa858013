"""CPU oracle for the transport AEAD — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module; it is the checker, never the product path.

Two restatements of the reference's algorithm live here:

* ``py_*`` — pure-Python, big-integer Poly1305 and a straightforward ChaCha20
  (small cases only). Follows RFC 8439 and the reference composition:
  ChaCha20 block  ax.xz.wireguard.noise/src/main/c/chacha-generic.c:10-78
  Poly1305        poly1305-donna.c:26-69, poly1305-donna-64.h:75-223
  AEAD            ax.xz.wireguard.noise/.../crypto/ChaCha20Poly1305.java:31-97
  nonce layout    ax.xz.wireguard.noise/.../handshake/SymmetricKeypair.java:52-61
* ``lib`` — ctypes binding of ``oracle/liboracle.so`` (wg_oracle.c), the fast C
  restatement used for large parity checks and the CPU baseline.

Parity pinning: the reference's own known-answer vectors (tests/golden/
reference_vectors.json: RFC 8439 vectors from ChaCha20Test.java /
Poly1305Test.java and the donna power-on self-test vectors of
poly1305-donna.c:83-201). Building the reference's C here was refused (see
DESIGN.md §3), so OpenSSL's independent EVP_chacha20_poly1305 is used as an
extra cross-check of the transport layout on random inputs.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
P1305 = (1 << 130) - 5

# ---------------------------------------------------------------------------
# pure Python


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def py_chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    """RFC 8439 2.3 block; state layout as ChaCha20.initializeState (ChaCha20.java:55-74)."""
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    s += list(struct.unpack("<8I", key))
    s += [counter & 0xFFFFFFFF]
    s += list(struct.unpack("<3I", nonce))
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(x[i] + s[i]) & 0xFFFFFFFF for i in range(16)])


def py_chacha20(key: bytes, nonce: bytes, counter: int, data: bytes) -> bytes:
    """chacha_cipher: keystream XOR from block `counter`, 32-bit wrap (chacha-generic.c:77,81-97)."""
    out = bytearray(len(data))
    for off in range(0, len(data), 64):
        ks = py_chacha20_block(key, (counter + off // 64) & 0xFFFFFFFF, nonce)
        chunk = data[off:off + 64]
        out[off:off + len(chunk)] = bytes(a ^ b for a, b in zip(chunk, ks))
    return bytes(out)


def py_poly1305(key: bytes, msg: bytes) -> bytes:
    """Poly1305 with big integers: clamp r (donna-64.h:80-86), 0x01-pad final block, + s mod 2^128."""
    r = int.from_bytes(key[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    s = int.from_bytes(key[16:32], "little")
    h = 0
    for off in range(0, len(msg), 16):
        blk = msg[off:off + 16]
        h = ((h + int.from_bytes(blk + b"\x01", "little")) * r) % P1305
    return ((h + s) % (1 << 128)).to_bytes(16, "little")


def py_poly1305_keygen(key: bytes, nonce: bytes) -> bytes:
    """ChaCha20Poly1305.poly1305ChaChaKeyGen: first 32 bytes of block 0 (ChaCha20Poly1305.java:11-29)."""
    return py_chacha20_block(key, 0, nonce)[:32]


def _pad16(n: int) -> bytes:
    return b"\x00" * ((16 - n % 16) % 16)


def py_aead_tag(key: bytes, nonce: bytes, aad: bytes | None, ct: bytes) -> bytes:
    """chacha20Poly1305Tag (ChaCha20Poly1305.java:63-93): a null AAD still contributes aadLen = 0."""
    otk = py_poly1305_keygen(key, nonce)
    a = aad or b""
    mac_data = a + _pad16(len(a)) + ct + _pad16(len(ct)) + struct.pack("<QQ", len(a), len(ct))
    return py_poly1305(otk, mac_data)


def py_aead_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes | None = None) -> bytes:
    """poly1305AeadEncrypt: ct = ChaCha20(counter 1) ^ pt; returns ct || tag (ChaCha20Poly1305.java:35-38)."""
    ct = py_chacha20(key, nonce, 1, pt)
    return ct + py_aead_tag(key, nonce, aad, ct)


def py_aead_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes | None = None) -> bytes | None:
    """poly1305AeadDecrypt: verify, then decrypt; None models AEADBadTagException (ChaCha20Poly1305.java:40-56)."""
    ct, tag = ct_tag[:-16], ct_tag[-16:]
    if py_aead_tag(key, nonce, aad, ct) != tag:
        return None
    return py_chacha20(key, nonce, 1, ct)


def transport_nonce(counter: int) -> bytes:
    """SymmetricKeypair.getNonceBytes: LE64(counter) at offset 0 of 12 zero bytes (SymmetricKeypair.java:52-61)."""
    return struct.pack("<Q", counter & 0xFFFFFFFFFFFFFFFF) + b"\x00" * 4


# ---------------------------------------------------------------------------
# C restatement

WG_PKT = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("counter", "<u8"), ("len", "<u4"), ("key_slot", "<u4")])


def _load_lib():
    path = os.path.join(HERE, "liboracle.so")
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
    lib = ctypes.CDLL(path)
    u8p = ctypes.c_void_p
    lib.oracle_chacha20_block.argtypes = [u8p, ctypes.c_uint32, u8p, u8p]
    lib.oracle_chacha20_xor.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_size_t]
    lib.oracle_poly1305.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
    lib.oracle_aead_seal.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p]
    lib.oracle_aead_open.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p]
    lib.oracle_aead_open.restype = ctypes.c_int
    lib.oracle_seal_batch.argtypes = [u8p, ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_int]
    lib.oracle_open_batch.argtypes = [u8p, ctypes.c_size_t, u8p, u8p, u8p, u8p, ctypes.c_int]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _load_lib()
    return _LIB


def _ptr(buf) -> int:
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    if isinstance(buf, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(buf)), ctypes.c_void_p).value
    raise TypeError(type(buf))


def c_chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    out = np.zeros(64, np.uint8)
    k = np.frombuffer(key, np.uint8).copy(); n = np.frombuffer(nonce, np.uint8).copy()
    lib().oracle_chacha20_block(k.ctypes.data, counter & 0xFFFFFFFF, n.ctypes.data, out.ctypes.data)
    return out.tobytes()


def c_chacha20(key: bytes, nonce: bytes, counter: int, data: bytes) -> bytes:
    k = np.frombuffer(key, np.uint8).copy(); n = np.frombuffer(nonce, np.uint8).copy()
    src = np.frombuffer(data, np.uint8).copy() if data else np.zeros(1, np.uint8)
    out = np.zeros(max(len(data), 1), np.uint8)
    lib().oracle_chacha20_xor(k.ctypes.data, n.ctypes.data, counter & 0xFFFFFFFF, src.ctypes.data, out.ctypes.data, len(data))
    return out[: len(data)].tobytes()


def c_poly1305(key: bytes, msg: bytes) -> bytes:
    k = np.frombuffer(key, np.uint8).copy()
    m = np.frombuffer(msg, np.uint8).copy() if msg else np.zeros(1, np.uint8)
    out = np.zeros(16, np.uint8)
    lib().oracle_poly1305(k.ctypes.data, m.ctypes.data, len(msg), out.ctypes.data)
    return out.tobytes()


def c_aead_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes | None = None) -> bytes:
    k = np.frombuffer(key, np.uint8).copy(); n = np.frombuffer(nonce, np.uint8).copy()
    a = np.frombuffer(aad, np.uint8).copy() if aad else np.zeros(1, np.uint8)
    p = np.frombuffer(pt, np.uint8).copy() if pt else np.zeros(1, np.uint8)
    out = np.zeros(len(pt) + 16, np.uint8)
    lib().oracle_aead_seal(k.ctypes.data, n.ctypes.data, a.ctypes.data, len(aad or b""), p.ctypes.data, len(pt),
                           out.ctypes.data, out.ctypes.data + len(pt))
    return out.tobytes()


def c_aead_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes | None = None) -> bytes | None:
    L = len(ct_tag) - 16
    k = np.frombuffer(key, np.uint8).copy(); n = np.frombuffer(nonce, np.uint8).copy()
    a = np.frombuffer(aad, np.uint8).copy() if aad else np.zeros(1, np.uint8)
    c = np.frombuffer(ct_tag, np.uint8).copy()
    out = np.zeros(max(L, 1), np.uint8)
    rc = lib().oracle_aead_open(k.ctypes.data, n.ctypes.data, a.ctypes.data, len(aad or b""), c.ctypes.data, L,
                                c.ctypes.data + L, out.ctypes.data)
    return None if rc else out[:L].tobytes()


def seal_batch(desc: np.ndarray, inp: np.ndarray, out: np.ndarray, keys: np.ndarray, threads: int = 1) -> None:
    """Seal every wg_pkt of `desc` (structured WG_PKT array) — the oracle for wg_seal_batch."""
    assert desc.dtype == WG_PKT and inp.dtype == np.uint8 and out.dtype == np.uint8 and keys.dtype == np.uint8
    rc = lib().oracle_seal_batch(desc.ctypes.data, len(desc), inp.ctypes.data, out.ctypes.data, keys.ctypes.data, threads)
    assert rc == 0


def open_batch(desc: np.ndarray, inp: np.ndarray, out: np.ndarray, keys: np.ndarray, threads: int = 1) -> np.ndarray:
    """Open every wg_pkt; returns the per-packet status (0 ok, 1 bad tag) — the oracle for wg_open_batch."""
    status = np.zeros(len(desc), np.uint32)
    rc = lib().oracle_open_batch(desc.ctypes.data, len(desc), inp.ctypes.data, out.ctypes.data, keys.ctypes.data,
                                 status.ctypes.data, threads)
    assert rc == 0
    return status


# ---------------------------------------------------------------------------
# Transport wire framing (oracle for wg_frame_seal / wg_parse_open)

TRANSPORT_TYPE = 4  # TransportPacket.java:28
HEADER_SIZE = 16    # HEADER_LAYOUT: u8 type, pad 3, u32 receiver_index, u64 counter (TransportPacket.java:30-35)


def transport_header(receiver_index: int, counter: int) -> bytes:
    """The header UnencryptedOutgoingTransport.java:14-18 (type + receiver index) and
    EncryptedOutgoingTransport.java:11-14 (counter) leave in front of ct||tag; the
    JAVA_INT / JAVA_LONG layouts are native order, little-endian on x86-64."""
    return struct.pack("<BxxxIQ", TRANSPORT_TYPE, receiver_index & 0xFFFFFFFF, counter & 0xFFFFFFFFFFFFFFFF)


def frame_headers(desc: np.ndarray, receivers: np.ndarray, out: np.ndarray, key_slots: int,
                  in_size: int | None = None, max_len: int = 65535) -> None:
    """Oracle for wg_frame_seal: header at out_off - 16 of every packet the seal accepts
    (len <= max_len, key slot in the table, input and ct||tag inside their buffers) whose
    out_off >= 16 (UnencryptedOutgoingTransport.java:14-18, EncryptedOutgoingTransport.java:11-14)."""
    for p in desc:
        o, slot, L, io = int(p["out_off"]), int(p["key_slot"]), int(p["len"]), int(p["in_off"])
        if o < HEADER_SIZE or slot >= key_slots or L > max_len:
            continue
        if in_size is not None and (io > in_size or L > in_size - io):
            continue
        if o > len(out) or L + 16 > len(out) - o:
            continue
        out[o - HEADER_SIZE:o] = np.frombuffer(transport_header(int(receivers[slot]), int(p["counter"])), np.uint8)


def parse_wire(wire: np.ndarray, pkt_off: np.ndarray, pkt_len: np.ndarray, key_slot: np.ndarray):
    """Oracle for wg_parse_open (UndecryptedIncomingTransport.java:20-33): ciphertext
    length = packet length - 16, plaintext at +16+ctLen (:30), counter from the header
    (TransportPacket.java:53-55); a wrong type byte is rejected (:24-26). Returns
    (desc, parse_status) with len = 0xFFFFFFFF and status 2 for rejected packets."""
    n = len(pkt_off)
    desc = np.zeros(n, WG_PKT)
    st = np.zeros(n, np.uint32)
    for i in range(n):
        o, wl = int(pkt_off[i]), int(pkt_len[i])
        desc[i]["in_off"], desc[i]["out_off"], desc[i]["key_slot"] = o + 16, o + wl, int(key_slot[i])
        desc[i]["len"], desc[i]["counter"] = 0xFFFFFFFF, 0
        ok = wl >= 32 and o + wl + (wl - 32) <= len(wire) and int(wire[o]) == TRANSPORT_TYPE
        if ok:
            desc[i]["counter"] = struct.unpack_from("<Q", wire[o + 8:o + 16].tobytes())[0]
            desc[i]["len"] = wl - 32
        else:
            st[i] = 2
    return desc, st


# ---------------------------------------------------------------------------
# OpenSSL cross-check (independent implementation; not the reference)

_SSL = None


def openssl():
    global _SSL
    if _SSL is None:
        name = ctypes.util.find_library("crypto")
        if not name:
            return None
        c = ctypes.CDLL(name)
        c.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        c.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        c.EVP_chacha20_poly1305.restype = ctypes.c_void_p
        c.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
        c.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        c.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        c.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _SSL = c
    return _SSL


def openssl_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes | None = None) -> bytes | None:
    c = openssl()
    if c is None:
        return None
    EVP_CTRL_AEAD_GET_TAG = 0x10
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, c.EVP_chacha20_poly1305(), None, key, nonce) == 1
        n = ctypes.c_int(0)
        if aad:
            assert c.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 16)
        if pt:
            assert c.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
        assert c.EVP_EncryptFinal_ex(ctx, None, ctypes.byref(n)) == 1
        tag = ctypes.create_string_buffer(16)
        assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
        return out.raw[: len(pt)] + tag.raw
    finally:
        c.EVP_CIPHER_CTX_free(ctx)
