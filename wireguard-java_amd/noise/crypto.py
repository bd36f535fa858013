"""ax.xz.wireguard.noise.crypto mirror: ChaCha20, Poly1305, ChaCha20Poly1305, Crypto.

Every arithmetic call goes to the device (libwgaead); nothing is computed on the
host. "MemorySegment" arguments are Python buffers: bytes for inputs, and
writable buffers (bytearray, memoryview, numpy uint8) for outputs, which are
filled in place exactly like the Java code fills its output segments.
"""
from __future__ import annotations

import struct

import numpy as np

from .. import _lib as L
from ..engine import default_engine


class BadPaddingException(Exception):
    """javax.crypto.BadPaddingException"""


class AEADBadTagException(BadPaddingException):
    """javax.crypto.AEADBadTagException (thrown by ChaCha20Poly1305.java:51-53)"""


class IllegalStateException(Exception):
    """java.lang.IllegalStateException (Poly1305.java:114-119, 138-143)"""


class Crypto:
    """Constants of Crypto.java:8-14."""
    POLY1305_TAG_SIZE = 16
    ChaChaPoly1305NonceSize = 12
    ChaChaPoly1305Overhead = 16


def _bytes(seg) -> bytes:
    if seg is None:
        return b""
    if isinstance(seg, np.ndarray):
        return seg.astype(np.uint8, copy=False).tobytes()
    return bytes(seg)


def _write(dst, data: bytes) -> None:
    """Copy `data` into the leading bytes of the writable buffer `dst`."""
    if isinstance(dst, np.ndarray):
        dst.reshape(-1).view(np.uint8)[: len(data)] = np.frombuffer(data, np.uint8)
        return
    mv = memoryview(dst).cast("B")
    mv[: len(data)] = data


def _size(seg) -> int:
    if isinstance(seg, np.ndarray):
        return seg.nbytes
    return memoryview(seg).nbytes


def _nonce_words(nonce: bytes) -> list[int]:
    return list(struct.unpack("<3I", nonce))


class ChaCha20:
    """ChaCha20.java: state layout helpers + the chacha_cipher downcalls, on the device."""

    @staticmethod
    def initializeState(key, nonce, state, counter: int) -> None:
        """ChaCha20.java:55-74 (state = constants || key || counter || nonce, LE words)."""
        if _size(state) != 64:
            raise ValueError(f"State size must be 64 bytes (is {_size(state)})")
        words = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(struct.unpack("<8I", _bytes(key)))
        words += [counter & 0xFFFFFFFF] + _nonce_words(_bytes(nonce))
        _write(state, struct.pack("<16I", *words))

    @staticmethod
    def _cipher(key: bytes, nonce: bytes, data: bytes, counter: int) -> bytes:
        d = L.WgAeadDesc()
        d.len = len(data)
        d.ctr0 = counter & 0xFFFFFFFF
        d.nonce[:] = _nonce_words(nonce)
        out, _ = default_engine().aead_host(L.WG_MODE_CIPHER, [d], key, data, b"", len(data))
        return out

    @staticmethod
    def chacha20Block(state, output, counter: int) -> None:
        """ChaCha20.java:85-104: sets word 12 = counter and writes one 64-byte keystream block."""
        st = bytearray(_bytes(state))
        st[48:52] = struct.pack("<I", counter & 0xFFFFFFFF)
        _write(state, bytes(st))
        ks = ChaCha20._cipher(bytes(st[16:48]), bytes(st[52:64]), bytes(64), counter)
        _write(output, ks)

    @staticmethod
    def chacha20(key, nonce, input, output, counter: int) -> None:
        """ChaCha20.java:116-131: output = input ^ keystream(counter, counter+1, ...)."""
        data = _bytes(input)
        if _size(output) < len(data):
            raise ValueError("Output buffer must be at least as large as input buffer")
        _write(output, ChaCha20._cipher(_bytes(key), _bytes(nonce), data, counter))


class Poly1305:
    """Poly1305.java: init / update / finish. Updates are buffered and the MAC is
    evaluated on the device at finish (one-shot, same result as donna streaming)."""

    def __init__(self, context=None):
        self._key: bytes | None = None
        self._buf = bytearray()
        self.initialised = False
        self.finished = False

    def init(self, key) -> None:
        self._key = _bytes(key)[:32]
        self._buf = bytearray()
        self.initialised = True
        self.finished = False

    def update(self, message) -> None:
        if self.finished:
            raise IllegalStateException("Poly1305 context has already been finished")
        if not self.initialised:
            raise IllegalStateException("Poly1305 context has not been initialised")
        self._buf += _bytes(message)

    def finish(self, mac=None):
        if self.finished:
            raise IllegalStateException("Poly1305 context has already been finished")
        if not self.initialised:
            raise IllegalStateException("Poly1305 context has not been initialised")
        d = L.WgAeadDesc()
        d.len = len(self._buf)
        tag, _ = default_engine().aead_host(L.WG_MODE_MAC, [d], self._key, bytes(self._buf), b"", 16)
        self.finished = True
        self._key = None
        if mac is None:
            return tag
        _write(mac, tag)
        return None


class ChaCha20Poly1305:
    """ChaCha20Poly1305.java:10-98 (RFC 8439 AEAD) on the device."""

    @staticmethod
    def poly1305ChaChaKeyGen(*args):
        """(key, nonce) -> bytes[32], or (stateBuffer, key, nonce, output) (ChaCha20Poly1305.java:11-29)."""
        if len(args) == 2:
            key, nonce = args
            ks = ChaCha20._cipher(_bytes(key), _bytes(nonce), bytes(64), 0)
            return ks[:32]
        state, key, nonce, output = args
        ChaCha20.initializeState(key, nonce, state, 0)
        ChaCha20.chacha20Block(state, output, 0)
        return None

    @staticmethod
    def poly1305AeadEncrypt(*args) -> None:
        """([aad,] key, nonce, plaintext, ciphertext, tag) (ChaCha20Poly1305.java:31-38)."""
        aad, key, nonce, pt, ct, tag = args if len(args) == 6 else (None, *args)
        p = _bytes(pt)
        d = L.WgAeadDesc()
        d.len = len(p)
        a = _bytes(aad)
        d.aad_len = len(a)
        d.nonce[:] = _nonce_words(_bytes(nonce))
        out, _ = default_engine().aead_host(L.WG_MODE_SEAL, [d], _bytes(key), p, a, len(p) + 16)
        _write(ct, out[: len(p)])
        _write(tag, out[len(p):])

    @staticmethod
    def poly1305AeadDecrypt(*args) -> None:
        """([aad,] key, nonce, ciphertext, plaintext, tag); raises AEADBadTagException and leaves
        plaintext untouched on a mismatch (ChaCha20Poly1305.java:40-60)."""
        aad, key, nonce, ct, pt, tag = args if len(args) == 6 else (None, *args)
        c = _bytes(ct)
        t = _bytes(tag)[:16]
        d = L.WgAeadDesc()
        d.len = len(c)
        a = _bytes(aad)
        d.aad_len = len(a)
        d.nonce[:] = _nonce_words(_bytes(nonce))
        out, status = default_engine().aead_host(L.WG_MODE_OPEN, [d], _bytes(key), c + t, a, len(c))
        if status[0] != L.WG_PKT_OK:
            raise AEADBadTagException(f"Invalid tag (got {list(t)})")
        _write(pt, out)
