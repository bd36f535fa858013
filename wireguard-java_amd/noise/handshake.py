"""ax.xz.wireguard.noise.handshake.SymmetricKeypair mirror — the drop-in boundary.

Keeps the reference API (SymmetricKeypair.java:20-94): cipher(src, dst) -> counter,
decipher(counter, src, dst) raising BadPaddingException (AEADBadTagException),
clean(). Keys live in the device key table of the engine; the nonce is the
reference layout LE64(counter) || 0^4, built on the device. An additive batch
API (cipher_batch / decipher_batch) feeds whole device-resident batches.
"""
from __future__ import annotations

import threading

import numpy as np

from .. import _lib as L
from ..engine import Engine, default_engine, desc_as_int64, pack_desc
from .crypto import AEADBadTagException, IllegalStateException, _bytes, _size, _write


class SymmetricKeypair:
    def __init__(self, sendKey: bytes, receiveKey: bytes, engine: Engine | None = None):
        """SymmetricKeypair(byte[] sendKeyBytes, byte[] receiveKeyBytes) (SymmetricKeypair.java:39-50)."""
        self._engine = engine or default_engine()
        self._send_slot, self._recv_slot = self._engine.alloc_slots(2)
        # one upload per slot: after frees the two claimed slots need not be adjacent
        self._engine.set_keys(self._send_slot, bytes(sendKey))
        self._engine.set_keys(self._recv_slot, bytes(receiveKey))
        self._counter = 0  # volatile long sendCounter = 0 (:37)
        self._lock = threading.Lock()
        self._clean = False

    @property
    def send_slot(self) -> int:
        return self._send_slot

    @property
    def receive_slot(self) -> int:
        return self._recv_slot

    def _next(self, n: int = 1) -> int:
        with self._lock:  # SEND_COUNTER.getAndAdd(this, n) (:64)
            c = self._counter
            self._counter += n
            return c

    def _live(self):
        if self._clean:  # the reference's keys live in a closed Arena after clean() (:85-93)
            raise IllegalStateException("SymmetricKeypair used after clean()")

    def cipher(self, src, dst) -> int:
        """dst = ct || tag (L + 16 bytes); returns the counter used (SymmetricKeypair.java:63-74)."""
        self._live()
        counter = self._next()
        pt = _bytes(src)
        if _size(dst) < len(pt) + 16:
            raise IndexError("dst too small for ciphertext and tag")
        _write(dst, self._engine.seal1(self._send_slot, counter, pt))
        return counter

    def decipher(self, counter: int, src, dst) -> None:
        """src = ct || tag; plaintext of L = |src| - 16 bytes into dst (SymmetricKeypair.java:76-83)."""
        self._live()
        data = _bytes(src)
        if len(data) < 16:
            raise IndexError("ciphertext shorter than the 16-byte tag")  # asSlice(textLength, 16) fails
        pt = self._engine.open1(self._recv_slot, counter, data)
        if pt is None:
            raise AEADBadTagException("Invalid tag")
        _write(dst, pt)

    def clean(self) -> None:
        """Zero both keys (SymmetricKeypair.java:85-93). Runs once: a second clean() is a
        no-op, so the slots cannot be released twice."""
        with self._lock:
            if self._clean:
                return
            self._clean = True
        self._engine.free_slots([self._send_slot, self._recv_slot])

    # ---- additive batch API (device-resident) --------------------------------------
    def cipher_batch(self, inp, in_offsets, lengths, out, out_offsets, uniform: bool = False, stream=None):
        """Seal n packets of the torch uint8 device buffer `inp` into `out` (ct || tag each).
        Consumes n consecutive counters; returns (first_counter, desc_tensor)."""
        import torch
        self._live()
        n = len(lengths)
        c0 = self._next(n)
        d = pack_desc(in_offsets, out_offsets, np.arange(c0, c0 + n, dtype=np.uint64), lengths, self._send_slot)
        dt = torch.from_numpy(desc_as_int64(d)).to(inp.device)
        max_len = int(np.max(lengths)) if n else 0
        self._engine.seal(dt, inp, out, max_len, uniform=uniform, stream=stream)
        return c0, dt

    def decipher_batch(self, inp, in_offsets, counters, lengths, out, out_offsets, uniform: bool = False,
                       stream=None):
        """Open n packets (ct || tag at in_offsets, L = lengths); returns the device status tensor."""
        import torch
        self._live()
        n = len(lengths)
        d = pack_desc(in_offsets, out_offsets, counters, lengths, self._recv_slot)
        dt = torch.from_numpy(desc_as_int64(d)).to(inp.device)
        status = torch.empty(n, dtype=torch.int32, device=inp.device)
        max_len = int(np.max(lengths)) if n else 0
        self._engine.open(dt, inp, out, status, max_len, uniform=uniform, stream=stream)
        return status
