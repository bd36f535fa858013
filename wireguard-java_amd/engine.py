"""Device context and the batched transport API over libwgaead.

``Engine`` owns one ``wg_ctx`` (one HIP device, its stream and device key
table). It is the MI355X-side counterpart of the reference's per-packet
ForkJoinPool dispatch (TransportManager.java:41,70-93,137-158): packets are
sealed/opened in batches that stay resident in HBM.

Descriptors are ``wg_pkt`` records (include/wgaead.h). On the torch side a
batch of them is an int64 tensor of shape [n, 4]: (in_off, out_off, counter,
len | key_slot << 32) — byte-identical to the C struct array.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib as L

WG_PKT_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("counter", "<u8"), ("len", "<u4"),
                         ("key_slot", "<u4")])


def pack_desc(in_off, out_off, counter, length, key_slot) -> np.ndarray:
    """Build a wg_pkt array (numpy structured) from per-packet columns."""
    n = len(np.atleast_1d(in_off))
    d = np.zeros(n, WG_PKT_DTYPE)
    d["in_off"], d["out_off"], d["counter"] = in_off, out_off, counter
    d["len"], d["key_slot"] = length, key_slot
    return d


WG_AEAD_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("aad_off", "<u8"), ("len", "<u4"),
                          ("aad_len", "<u4"), ("key_slot", "<u4"), ("ctr0", "<u4"), ("nonce", "<u4", (3,)),
                          ("_reserved", "<u4", (3,))])


def desc_as_int64(d: np.ndarray) -> np.ndarray:
    """wg_pkt array viewed as int64 [n, 4] (for torch.from_numpy)."""
    d = np.ascontiguousarray(d)
    return d.view(np.int64).reshape(-1, d.dtype.itemsize // 8)


class Engine:
    """One HIP device: stream, key table (``key_slots`` x 32 bytes) and batch entry points."""

    def __init__(self, device: int = 0, key_slots: int = 1024):
        self._lib = L.lib()
        ctx = ctypes.c_void_p()
        L.check(self._lib.wg_ctx_create(device, key_slots, ctypes.byref(ctx)))
        self.ctx = ctx
        self.device = device
        self.key_slots = key_slots
        self._free = set(range(key_slots))
        self._slot_lock = threading.Lock()
        self._pinned = {}

    # ---- lifecycle --------------------------------------------------------------
    def close(self):
        if self.ctx:
            for p in self._pinned.values():
                self._lib.wg_host_free(self.ctx, p)
            self._pinned.clear()
            self._lib.wg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_kernel(self, name: str | None = "default", lanes: int = 0, variant: int = 0) -> None:
        """Transport kernel for this engine's seal/open calls (wg_ctx_set_kernel): "default"
        (k_transport), "wave1" (the round-1 kernel) or "tile"; every kernel computes the
        same bytes, only the speed differs."""
        L.check(self._lib.wg_ctx_set_kernel(self.ctx, None if name is None else name.encode(), lanes, variant))

    @property
    def stream(self) -> int:
        return self._lib.wg_ctx_stream(self.ctx)

    def sync(self, stream: int | None = None):
        L.check(self._lib.wg_sync(self.ctx, stream))

    # ---- keys (SymmetricKeypair.java:39-50, 85-93) ------------------------------
    def alloc_slots(self, n: int) -> list[int]:
        """Claim n free key slots (lowest first). Callers upload each slot's key on its
        own (set_keys(slot, key)): claimed slots need not be adjacent after frees."""
        with self._slot_lock:
            if len(self._free) < n:
                raise L.WgError(L.WG_ERANGE, "key table full")
            got = sorted(self._free)[:n]
            self._free.difference_update(got)
            return got

    def free_slots(self, slots):
        """Zero and release slots claimed with alloc_slots (SymmetricKeypair.clean). A slot
        that is not currently claimed is an error, so a double release cannot hand one
        slot to two keypairs."""
        with self._slot_lock:
            bad = [s for s in slots if s in self._free or not 0 <= s < self.key_slots]
            if bad or len(set(slots)) != len(slots):
                raise L.WgError(L.WG_EINVAL, f"key slots {slots} are not all claimed")
        for s in slots:
            self.zero_keys(s, 1)
        with self._slot_lock:
            self._free.update(slots)

    def set_keys(self, first_slot: int, keys) -> None:
        k = np.ascontiguousarray(np.frombuffer(bytes(keys), np.uint8) if not isinstance(keys, np.ndarray) else keys,
                                 dtype=np.uint8)
        assert k.size % 32 == 0
        L.check(self._lib.wg_keys_set(self.ctx, first_slot, k.size // 32, k.ctypes.data))

    def zero_keys(self, first_slot: int, n: int) -> None:
        L.check(self._lib.wg_keys_zero(self.ctx, first_slot, n))

    # ---- device-resident batches (torch tensors on this device) -------------------
    def seal(self, desc, inp, out, max_len: int, uniform: bool = False, stream: int | None = None,
             frame: bool = False):
        """wg_seal_batch over torch tensors: desc int64 [n,4], inp/out uint8 (device).
        frame=True also writes each packet's transport header (WG_F_FRAME)."""
        n = desc.shape[0]
        flags = (L.WG_F_UNIFORM if uniform else 0) | (L.WG_F_FRAME if frame else 0)
        L.check(self._lib.wg_seal_batch(self.ctx, desc.data_ptr(), n, inp.data_ptr(), inp.numel(), out.data_ptr(),
                                        out.numel(), max_len, flags,
                                        stream if stream is not None else _torch_stream()))

    def open(self, desc, inp, out, status, max_len: int, uniform: bool = False, stream: int | None = None,
             rx_filter: bool = False):
        """wg_open_batch; `status` is an int32/uint32 device tensor of n entries (0 ok, 1 bad tag).
        rx_filter (WG_F_RX_FILTER): the receive-side keepalive / IP / AllowedIPs verdict of
        wg_rx_check(WG_RX_FILTER) written by the open kernel itself."""
        n = desc.shape[0]
        flags = (L.WG_F_UNIFORM if uniform else 0) | (L.WG_F_RX_FILTER if rx_filter else 0)
        L.check(self._lib.wg_open_batch(self.ctx, desc.data_ptr(), n, inp.data_ptr(), inp.numel(), out.data_ptr(),
                                        out.numel(), status.data_ptr(), max_len, flags,
                                        stream if stream is not None else _torch_stream()))

    def duplex(self, seal_desc, seal_in, seal_out, seal_max_len: int, open_desc, open_in, open_out, status,
               open_max_len: int, uniform: bool = False, frame: bool = False, stream: int | None = None,
               after_seal: bool = False):
        """wg_duplex_batch: seal one batch and open another in one launch. Without after_seal the
        open batch must not read what the seal batch writes; with it (WG_F_AFTER_SEAL) open packet i
        is ordered after seal packet i (k_step for uniform batches). Same tensors as seal() / open()."""
        u = L.WG_F_UNIFORM if uniform else 0
        sb = L.WgBatch(seal_desc.data_ptr(), seal_in.data_ptr(), seal_out.data_ptr(), None, seal_in.numel(),
                       seal_out.numel(), seal_desc.shape[0], seal_max_len, u | (L.WG_F_FRAME if frame else 0), 0)
        ob = L.WgBatch(open_desc.data_ptr(), open_in.data_ptr(), open_out.data_ptr(),
                       status.data_ptr() if status is not None else None, open_in.numel(), open_out.numel(),
                       open_desc.shape[0], open_max_len, u | (L.WG_F_AFTER_SEAL if after_seal else 0), 0)
        L.check(self._lib.wg_duplex_batch(self.ctx, ctypes.byref(sb), ctypes.byref(ob),
                                          stream if stream is not None else _torch_stream()))

    def prepare_duplex(self, seal_desc, seal_in, seal_out, seal_max_len: int, open_desc, open_in, open_out, status,
                       open_max_len: int, uniform: bool = False, after_seal: bool = False, stream: int | None = None):
        """The same wg_duplex_batch call as duplex(), with its argument structs built once: returns a
        zero-argument callable that issues the launch on `stream` (default: torch's current stream when
        prepared). A caller that re-launches one batch layout over and over (a pipeline stage, a bench
        step) so pays one foreign call per launch instead of rebuilding the arguments. The tensors must
        stay alive and in place while the callable is used."""
        u = L.WG_F_UNIFORM if uniform else 0
        sb = L.WgBatch(seal_desc.data_ptr(), seal_in.data_ptr(), seal_out.data_ptr(), None, seal_in.numel(),
                       seal_out.numel(), seal_desc.shape[0], seal_max_len, u, 0)
        ob = L.WgBatch(open_desc.data_ptr(), open_in.data_ptr(), open_out.data_ptr(),
                       status.data_ptr() if status is not None else None, open_in.numel(), open_out.numel(),
                       open_desc.shape[0], open_max_len, u | (L.WG_F_AFTER_SEAL if after_seal else 0), 0)
        fn, ctx = self._lib.wg_duplex_batch, self.ctx
        ps, po = ctypes.byref(sb), ctypes.byref(ob)
        st = stream if stream is not None else _torch_stream()
        keep = (sb, ob, seal_desc, seal_in, seal_out, open_desc, open_in, open_out, status)

        def launch():
            rc = fn(ctx, ps, po, st)
            if rc < 0:
                L.check(rc)
            return keep  # (holds the structs and tensors for as long as the callable lives)
        return launch

    # ---- receive side after open (wg_rx_check) -------------------------------------
    def filter_set(self, filter_id: int, prefixes) -> None:
        """wg_filter_set from (address string or ipaddress object, prefix_len) pairs, as
        IPFilter.insert(InetAddress, int) takes them (util/IPFilter.java:30-42)."""
        import ipaddress
        arr = (L.WgPrefix * max(1, len(prefixes)))()
        for k, (addr, plen) in enumerate(prefixes):
            a = ipaddress.ip_address(addr) if isinstance(addr, str) else addr
            arr[k].family = 4 if a.version == 4 else 6
            arr[k].prefix_len = plen
            b = a.packed
            for i, x in enumerate(b):
                arr[k].addr[i] = x
        L.check(self._lib.wg_filter_set(self.ctx, filter_id, ctypes.addressof(arr), len(prefixes)))

    def slot_filters_set(self, first_slot: int, filter_ids) -> None:
        ids = np.ascontiguousarray(np.asarray(filter_ids, dtype=np.uint32))
        L.check(self._lib.wg_slot_filters_set(self.ctx, first_slot, len(ids), ids.ctypes.data))

    def replay_enable(self, window_bits: int = 8192) -> None:
        L.check(self._lib.wg_replay_enable(self.ctx, window_bits))

    def replay_reset(self, first_slot: int, n: int) -> None:
        L.check(self._lib.wg_replay_reset(self.ctx, first_slot, n))

    def replay_state(self, slot: int, window_bits: int):
        """(top, bitmap words as uint64 numpy array) of one key slot's window."""
        top = ctypes.c_uint64()
        bits = np.zeros(window_bits // 64, np.uint64)
        L.check(self._lib.wg_replay_state(self.ctx, slot, ctypes.byref(top), bits.ctypes.data, len(bits)))
        return top.value, bits

    def rx_check(self, desc, pt, status, flags: int = 1, stream: int | None = None) -> None:
        """wg_rx_check after open(desc, ..., out=pt, status) on the same stream."""
        n = desc.shape[0]
        L.check(self._lib.wg_rx_check(self.ctx, desc.data_ptr(), n, pt.data_ptr(), pt.numel(), status.data_ptr(),
                                      flags, stream if stream is not None else _torch_stream()))

    def set_receivers(self, receivers) -> None:
        """wg_ctx_set_receivers: device tensor of receiver_index per key slot for
        seal(..., frame=True) — contiguous, 4-byte integers, on this engine's device, at
        least key_slots entries; the engine keeps it alive while seals use it."""
        if receivers is None:
            L.check(self._lib.wg_ctx_set_receivers(self.ctx, None, 0))
            self._receivers = None
            return
        if receivers.device.type != "cuda" or receivers.device.index not in (None, self.device):
            raise L.WgError(L.WG_EINVAL, f"receiver table on {receivers.device}, engine on cuda:{self.device}")
        if not receivers.is_contiguous() or receivers.element_size() != 4:
            raise L.WgError(L.WG_EINVAL, "receiver table must be a contiguous int32/uint32 tensor")
        if receivers.numel() < self.key_slots:
            raise L.WgError(L.WG_ERANGE, f"receiver table has {receivers.numel()} entries for {self.key_slots} slots")
        L.check(self._lib.wg_ctx_set_receivers(self.ctx, receivers.data_ptr(), receivers.numel()))
        self._receivers = receivers

    def frame_seal(self, desc, receivers, out, in_size: int, max_len: int, stream: int | None = None):
        """wg_frame_seal: write the 16-B transport header {4, 0, 0, 0, receiver_index, counter}
        in front of every packet the seal accepts (UnencryptedOutgoingTransport.java:14-18,
        EncryptedOutgoingTransport.java:11-14). `receivers` is a uint32/int32 device tensor
        indexed by key slot; in_size / max_len are the seal call's."""
        n = desc.shape[0]
        L.check(self._lib.wg_frame_seal(self.ctx, desc.data_ptr(), n, receivers.data_ptr(), out.data_ptr(),
                                        out.numel(), in_size, max_len,
                                        stream if stream is not None else _torch_stream()))

    def parse_open(self, wire, pkt_off, pkt_len, key_slot, desc_out, parse_status=None, stream: int | None = None):
        """wg_parse_open: open descriptors from received wire packets on device
        (UndecryptedIncomingTransport.java:20-33); plaintext lands right after each
        packet's ciphertext in `wire`. pkt_off int64, pkt_len / key_slot int32 device tensors."""
        n = pkt_off.shape[0]
        L.check(self._lib.wg_parse_open(self.ctx, wire.data_ptr(), wire.numel(), pkt_off.data_ptr(),
                                        pkt_len.data_ptr(), key_slot.data_ptr(), n, desc_out.data_ptr(),
                                        parse_status.data_ptr() if parse_status is not None else None,
                                        stream if stream is not None else _torch_stream()))

    def aead(self, mode: int, desc, inp, aad, out, status, max_len: int, stream: int | None = None):
        """wg_aead_batch over torch tensors: desc int64 [n, 8] (wg_aead_desc records)."""
        n = desc.shape[0]
        L.check(self._lib.wg_aead_batch(self.ctx, mode, desc.data_ptr(), n, inp.data_ptr() if inp is not None else None,
                                        inp.numel() if inp is not None else 0,
                                        aad.data_ptr() if aad is not None else None,
                                        aad.numel() if aad is not None else 0, out.data_ptr(), out.numel(),
                                        status.data_ptr() if status is not None else None, max_len,
                                        stream if stream is not None else _torch_stream()))

    # ---- host buffers ---------------------------------------------------------------
    def seal_host(self, desc: np.ndarray, inp, out, max_len: int, uniform: bool = False):
        """wg_seal_host: a batch in host memory. ``inp``/``out`` are numpy arrays (pageable:
        chunked copy pipeline) or pinned buffers from :meth:`host_alloc` (zero-copy)."""
        d = np.ascontiguousarray(desc)
        ip, isz = _host_buf(inp)
        op, osz = _host_buf(out)
        L.check(self._lib.wg_seal_host(self.ctx, d.ctypes.data, len(d), ip, isz, op, osz, max_len,
                                       L.WG_F_UNIFORM if uniform else 0))

    def open_host(self, desc: np.ndarray, inp, out, max_len: int, uniform: bool = False) -> np.ndarray:
        d = np.ascontiguousarray(desc)
        status = np.zeros(len(d), np.uint32)
        ip, isz = _host_buf(inp)
        op, osz = _host_buf(out)
        L.check(self._lib.wg_open_host(self.ctx, d.ctypes.data, len(d), ip, isz, op, osz, status.ctypes.data, max_len,
                                       L.WG_F_UNIFORM if uniform else 0))
        return status

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """A pinned, device-mapped host ring (wg_host_alloc) as a uint8 numpy array; freed
        with :meth:`host_free` (or when the engine closes)."""
        p = ctypes.c_void_p()
        L.check(self._lib.wg_host_alloc(self.ctx, nbytes, ctypes.byref(p)))
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value))[:nbytes]
        self._pinned[arr.ctypes.data] = p
        return arr

    def host_free(self, arr: np.ndarray) -> None:
        p = self._pinned.pop(arr.ctypes.data, None)
        if p is not None:
            L.check(self._lib.wg_host_free(self.ctx, p))

    def aead_host(self, mode: int, descs, keys: bytes, inp: bytes, aad: bytes, out_size: int):
        """General AEAD / primitive batch on host buffers (wg_aead_host). Returns (out, status)."""
        arr = (L.WgAeadDesc * len(descs))(*descs)
        kb = np.frombuffer(keys, np.uint8).copy()
        ib = np.frombuffer(inp, np.uint8).copy() if inp else np.zeros(1, np.uint8)
        ab = np.frombuffer(aad, np.uint8).copy() if aad else np.zeros(1, np.uint8)
        out = np.zeros(max(out_size, 1), np.uint8)
        status = np.zeros(len(descs), np.uint32)
        L.check(self._lib.wg_aead_host(self.ctx, mode, ctypes.addressof(arr), len(descs), kb.ctypes.data,
                                       kb.size // 32, ib.ctypes.data, len(inp), ab.ctypes.data, len(aad),
                                       out.ctypes.data, out_size, status.ctypes.data))
        return out[:out_size].tobytes(), status

    def queue(self, mode: str, capacity: int = 0, max_len: int = 0, max_batch: int = 0) -> "Queue":
        """wg_queue_create: an asynchronous seal ("seal") or open ("open") queue on this context."""
        return Queue(self, mode, capacity, max_len, max_batch)

    def seal1(self, slot: int, counter: int, pt: bytes) -> bytes:
        src = np.frombuffer(pt, np.uint8).copy() if pt else np.zeros(1, np.uint8)
        out = np.zeros(len(pt) + 16, np.uint8)
        L.check(self._lib.wg_seal1(self.ctx, slot, counter, src.ctypes.data, len(pt), out.ctypes.data))
        return out.tobytes()

    def open1(self, slot: int, counter: int, ct_tag: bytes) -> bytes | None:
        n = len(ct_tag) - 16
        src = np.frombuffer(ct_tag, np.uint8).copy()
        out = np.zeros(max(n, 1), np.uint8)
        rc = L.check(self._lib.wg_open1(self.ctx, slot, counter, src.ctypes.data, n, out.ctypes.data))
        return None if rc == 1 else out[:n].tobytes()

    def pp_config(self, waves: int = 16, idle_us: int = 20000) -> None:
        """wg_pp_config: waves of the persistent per-packet server (k_pp) that serves
        seal1/open1 (a power of two), and how long it stays resident without work (microseconds)."""
        L.check(self._lib.wg_pp_config(self.ctx, waves, idle_us))

    batcher_config = pp_config  # round-3 name

    def batcher_stats(self) -> tuple[int, int]:
        """(server launches, packets served) of the per-packet path so far."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        L.check(self._lib.wg_batcher_stats(self.ctx, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    # ---- instrumentation ----------------------------------------------------------
    def timing(self, on: bool):
        L.check(self._lib.wg_timing_enable(self.ctx, 1 if on else 0))

    def timing_read(self) -> tuple[float, int]:
        ms = ctypes.c_double()
        k = ctypes.c_uint64()
        L.check(self._lib.wg_timing_read(self.ctx, ctypes.byref(ms), ctypes.byref(k)))
        return ms.value, k.value


def _torch_stream() -> int:
    import torch
    return torch.cuda.current_stream().cuda_stream


def selftest(device: int = 0) -> bool:
    """wg_aead_selftest: the reference's known-answer vectors, on the device (Poly1305.java:62-76)."""
    return L.lib().wg_aead_selftest(device) == 1


_default: dict[int, Engine] = {}
_default_lock = threading.Lock()


def default_engine(device: int | None = None) -> Engine:
    """Process-wide engine per device, created on first use (like the reference's static initialisers)."""
    import os
    dev = int(os.environ.get("WG_DEVICE", "0")) if device is None else device
    with _default_lock:
        if dev not in _default:
            _default[dev] = Engine(dev, key_slots=int(os.environ.get("WG_KEY_SLOTS", "65536")))
        return _default[dev]


def _host_buf(x):
    """(pointer, nbytes) of a host buffer: numpy array or CPU torch tensor (pinned or not)."""
    if isinstance(x, np.ndarray):
        assert x.flags.c_contiguous
        return x.ctypes.data, x.nbytes
    return x.data_ptr(), x.numel() * x.element_size()


class Queue:
    """wg_queue: producers submit packets without waiting for the crypto (wg_submit_seal /
    wg_submit_open), a consumer reaps the results (wg_reap, wg_reap_done). The batching
    replacement for TransportManager's per-packet ForkJoinPool submission
    (TransportManager.java:41,70-93,137-158)."""

    def __init__(self, engine: Engine, mode: str, capacity: int = 0, max_len: int = 0, max_batch: int = 0):
        self._lib = engine._lib
        self.mode = {"seal": L.WG_MODE_SEAL, "open": L.WG_MODE_OPEN}[mode]
        q = ctypes.c_void_p()
        L.check(self._lib.wg_queue_create(engine.ctx, self.mode, capacity, max_len, max_batch, ctypes.byref(q)))
        self.q = q.value
        self._buf = (L.WgCompletion * 4096)()

    def submit(self, key_slot: int, counter: int, data: bytes, user: int = 0) -> None:
        """seal: data = plaintext; open: data = ct || tag."""
        n = len(data) - (16 if self.mode == L.WG_MODE_OPEN else 0)
        if n < 0:
            raise ValueError("open needs ct || tag (at least 16 bytes)")
        src = np.frombuffer(bytes(data), np.uint8) if data else np.zeros(1, np.uint8)
        fn = self._lib.wg_submit_seal if self.mode == L.WG_MODE_SEAL else self._lib.wg_submit_open
        L.check(fn(self.q, key_slot, counter, src.ctypes.data, n, user))

    def submit_n(self, packets) -> int:
        """wg_submit_seal_n / wg_submit_open_n: packets = [(key_slot, counter, data, user)] queued in
        one call (data as for submit()); returns how many were queued (fewer than len(packets) only
        when the submit timeout ran out partway)."""
        arr = (L.WgSubmit * max(1, len(packets)))()
        keep = []
        for k, (key_slot, counter, data, user) in enumerate(packets):
            n = len(data) - (16 if self.mode == L.WG_MODE_OPEN else 0)
            if n < 0:
                raise ValueError("open needs ct || tag (at least 16 bytes)")
            src = np.frombuffer(bytes(data), np.uint8) if data else np.zeros(1, np.uint8)
            keep.append(src)
            arr[k].user, arr[k].counter, arr[k].data = user, counter, src.ctypes.data
            arr[k].len, arr[k].key_slot = n, key_slot
        fn = self._lib.wg_submit_seal_n if self.mode == L.WG_MODE_SEAL else self._lib.wg_submit_open_n
        return L.check(fn(self.q, arr, len(packets)))

    def reap(self, max_n: int = 4096, timeout_us: int = 100000):
        """[(user, counter, status, result bytes)], the slots handed back at once; the result is
        ct || tag for a seal, the plaintext for an open (None unless status is WG_PKT_OK)."""
        m = min(max_n, len(self._buf))
        n = L.check(self._lib.wg_reap(self.q, self._buf, m, timeout_us))
        out = []
        for k in range(n):
            c = self._buf[k]
            size = c.len + (16 if self.mode == L.WG_MODE_SEAL else 0)
            ok = c.status == L.WG_PKT_OK
            data = ctypes.string_at(c.data, size) if ok and size else (b"" if ok else None)
            out.append((c.user, c.counter, c.status, data))
        L.check(self._lib.wg_reap_done(self.q, self._buf, n))
        return out

    def set_submit_timeout(self, timeout_us: int) -> None:
        """wg_queue_set_submit_timeout: submit() raises WgError(EAGAIN) once no slot has been free for
        timeout_us (0: it waits without bound, the default)."""
        L.check(self._lib.wg_queue_set_submit_timeout(self.q, timeout_us))

    def stats(self) -> tuple[int, int]:
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        L.check(self._lib.wg_queue_stats(self.q, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def close(self) -> None:
        if self.q:
            L.check(self._lib.wg_queue_destroy(self.q))
            self.q = None
