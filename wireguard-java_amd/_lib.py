"""ctypes binding of libwgaead.so — the C-ABI declared in include/wgaead.h.

The product path has no CPU fallback: if the shared library (built in-tree by
``make -C wireguard-java_amd/csrc``) is missing or no HIP device is usable, the
calls below raise ``WgError`` instead of computing anything on the host.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WG_LIB_PATH") or os.path.join(HERE, "libwgaead.so")

WG_OK = 0
WG_EINVAL = -22
WG_ENOMEM = -12
WG_ERANGE = -34
WG_E2BIG = -7
WG_EDEVICE = -5
WG_ESELFTEST = -74
WG_EAGAIN = -11
WG_ENOKEY = -126
WG_PKT_OK = 0
WG_PKT_BADTAG = 1
WG_PKT_BADHDR = 2
WG_PKT_KEEPALIVE = 3
WG_PKT_BADIP = 4
WG_PKT_FILTERED = 5
WG_PKT_REPLAY = 6
WG_PKT_NOKEY = 7
WG_PKT_FAILED = 255
WG_QUEUE_MAX_LEN = 16384
WG_RX_FILTER = 1
WG_RX_REPLAY = 2
WG_MAX_FILTERS = 65536
WG_NO_FILTER = 0xFFFFFFFF
WG_LEN_INVALID = 0xFFFFFFFF
WG_TAG_SIZE = 16
WG_NONCE_SIZE = 12
WG_KEY_SIZE = 32
WG_MAX_PACKET = 65535
WG_F_UNIFORM = 1
WG_F_FRAME = 2
WG_F_AFTER_SEAL = 4
WG_F_RX_FILTER = 8
WG_MODE_SEAL, WG_MODE_OPEN, WG_MODE_CIPHER, WG_MODE_MAC = 0, 1, 2, 3

_ERRNAMES = {WG_EINVAL: "EINVAL", WG_ENOMEM: "ENOMEM", WG_ERANGE: "ERANGE", WG_E2BIG: "E2BIG",
             WG_EDEVICE: "EDEVICE", WG_ESELFTEST: "ESELFTEST", WG_EAGAIN: "EAGAIN", WG_ENOKEY: "ENOKEY"}


class WgError(RuntimeError):
    """A negative return code of libwgaead (mirrors the RuntimeException the reference's
    FFM wrappers raise on a failed downcall, ChaCha20.java:102,110,141)."""

    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"libwgaead {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class WgPkt(ctypes.Structure):
    _fields_ = [("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64), ("counter", ctypes.c_uint64),
                ("len", ctypes.c_uint32), ("key_slot", ctypes.c_uint32)]


class WgAeadDesc(ctypes.Structure):
    _fields_ = [("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64), ("aad_off", ctypes.c_uint64),
                ("len", ctypes.c_uint32), ("aad_len", ctypes.c_uint32), ("key_slot", ctypes.c_uint32),
                ("ctr0", ctypes.c_uint32), ("nonce", ctypes.c_uint32 * 3), ("_reserved", ctypes.c_uint32 * 3)]


class WgPrefix(ctypes.Structure):
    _fields_ = [("family", ctypes.c_uint8), ("prefix_len", ctypes.c_uint8), ("addr", ctypes.c_uint8 * 16)]


class WgBatch(ctypes.Structure):
    """wg_batch: one direction of wg_duplex_batch (device pointers)."""
    _fields_ = [("desc", ctypes.c_void_p), ("in_", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("in_size", ctypes.c_uint64), ("out_size", ctypes.c_uint64),
                ("n", ctypes.c_uint32), ("max_len", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("_reserved", ctypes.c_uint32)]


class WgCompletion(ctypes.Structure):
    """wg_completion: one reaped packet of a wg_queue."""
    _fields_ = [("user", ctypes.c_uint64), ("counter", ctypes.c_uint64), ("data", ctypes.c_void_p),
                ("len", ctypes.c_uint32), ("status", ctypes.c_uint32), ("key_slot", ctypes.c_uint32),
                ("slot", ctypes.c_uint32), ("submit_ns", ctypes.c_uint64)]


class WgSubmit(ctypes.Structure):
    """wg_submit: one packet of wg_submit_seal_n / wg_submit_open_n."""
    _fields_ = [("user", ctypes.c_uint64), ("counter", ctypes.c_uint64), ("data", ctypes.c_void_p),
                ("len", ctypes.c_uint32), ("key_slot", ctypes.c_uint32)]


assert ctypes.sizeof(WgBatch) == 64 and ctypes.sizeof(WgCompletion) == 48 and ctypes.sizeof(WgSubmit) == 32
assert ctypes.sizeof(WgPkt) == 32 and ctypes.sizeof(WgAeadDesc) == 64 and ctypes.sizeof(WgPrefix) == 18

# (name, restype, argtypes) for every symbol include/wgaead.h declares
_VP, _U32, _U64, _I, _D = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
SIGNATURES = [
    ("wg_aead_selftest", _I, [_I]),
    ("wg_ctx_create", _I, [_I, _U32, ctypes.POINTER(_VP)]),
    ("wg_ctx_destroy", _I, [_VP]),
    ("wg_ctx_device", _I, [_VP]),
    ("wg_ctx_key_slots", _U32, [_VP]),
    ("wg_ctx_stream", _VP, [_VP]),
    ("wg_sync", _I, [_VP, _VP]),
    ("wg_last_error", ctypes.c_char_p, []),
    ("wg_version", ctypes.c_char_p, []),
    ("wg_device_numa_node", _I, [_I]),
    ("wg_ctx_set_kernel", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]),
    ("wg_keys_set", _I, [_VP, _U32, _U32, _VP]),
    ("wg_keys_zero", _I, [_VP, _U32, _U32]),
    ("wg_seal_batch", _I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64, _U32, _U32, _VP]),
    ("wg_open_batch", _I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64, _VP, _U32, _U32, _VP]),
    ("wg_duplex_batch", _I, [_VP, ctypes.POINTER(WgBatch), ctypes.POINTER(WgBatch), _VP]),
    ("wg_ctx_set_receivers", _I, [_VP, _VP, _U32]),
    ("wg_frame_seal", _I, [_VP, _VP, _U32, _VP, _VP, _U64, _U64, _U32, _VP]),
    ("wg_parse_open", _I, [_VP, _VP, _U64, _VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    ("wg_aead_batch", _I, [_VP, _I, _VP, _U32, _VP, _U64, _VP, _U64, _VP, _U64, _VP, _U32, _VP]),
    ("wg_filter_set", _I, [_VP, _U32, _VP, _U32]),
    ("wg_slot_filters_set", _I, [_VP, _U32, _U32, _VP]),
    ("wg_replay_enable", _I, [_VP, _U32]),
    ("wg_replay_reset", _I, [_VP, _U32, _U32]),
    ("wg_replay_state", _I, [_VP, _U32, ctypes.POINTER(_U64), _VP, _U32]),
    ("wg_rx_check", _I, [_VP, _VP, _U32, _VP, _U64, _VP, _U32, _VP]),
    ("wg_seal1", _I, [_VP, _U32, _U64, _VP, _U32, _VP]),
    ("wg_open1", _I, [_VP, _U32, _U64, _VP, _U32, _VP]),
    ("wg_pp_config", _I, [_VP, _U32, _U32]),
    ("wg_pp_last_call", _I, [ctypes.POINTER(_U64), _U32]),
    ("wg_batcher_config", _I, [_VP, _U32, _U32]),
    ("wg_batcher_stats", _I, [_VP, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    ("wg_queue_create", _I, [_VP, _I, _U32, _U32, _U32, ctypes.POINTER(_VP)]),
    ("wg_queue_destroy", _I, [_VP]),
    ("wg_submit_seal", _I, [_VP, _U32, _U64, _VP, _U32, _U64]),
    ("wg_submit_open", _I, [_VP, _U32, _U64, _VP, _U32, _U64]),
    ("wg_submit_seal_n", _I, [_VP, ctypes.POINTER(WgSubmit), _U32]),
    ("wg_submit_open_n", _I, [_VP, ctypes.POINTER(WgSubmit), _U32]),
    ("wg_reap", _I, [_VP, ctypes.POINTER(WgCompletion), _U32, _U32]),
    ("wg_reap_done", _I, [_VP, ctypes.POINTER(WgCompletion), _U32]),
    ("wg_queue_stats", _I, [_VP, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    ("wg_queue_set_submit_timeout", _I, [_VP, _U32]),
    ("wg_queue_key_residue", _U32, [_VP]),
    ("wg_seal_host", _I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64, _U32, _U32]),
    ("wg_open_host", _I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64, _VP, _U32, _U32]),
    ("wg_host_alloc", _I, [_VP, _U64, ctypes.POINTER(_VP)]),
    ("wg_host_free", _I, [_VP, _VP]),
    ("wg_host_register", _I, [_VP, _VP, _U64]),
    ("wg_host_unregister", _I, [_VP, _VP]),
    ("wg_aead_host", _I, [_VP, _I, _VP, _U32, _VP, _U32, _VP, _U64, _VP, _U64, _VP, _U64, _VP]),
    ("wg_timing_enable", _I, [_VP, _I]),
    ("wg_timing_read", _I, [_VP, ctypes.POINTER(_D), ctypes.POINTER(_U64)]),
]

_lib = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    """Load libwgaead.so (once). Raises WgError(EDEVICE) when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise WgError(WG_EDEVICE, f"{LIB_PATH} not built (run `make -C wireguard-java_amd/csrc`)")
            L = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def last_error() -> str:
    msg = lib().wg_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> int:
    if rc < 0:
        raise WgError(rc, last_error())
    return rc
