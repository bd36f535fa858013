"""wireguard-java_amd — MI355X-native transport-data AEAD for chop0/wireguard-java.

Layout:
  csrc/        gfx950 HIP kernels + the C-ABI (libwgaead.so, include/wgaead.h)
  _lib.py      ctypes binding of the C-ABI (fails loudly if the library is missing)
  engine.py    per-device context, key table, device-resident batch API
  noise/       mirror of ax.xz.wireguard.noise (ChaCha20, Poly1305, ChaCha20Poly1305,
               SymmetricKeypair) on top of the device path
  java/        the Java drop-in sources that bind libwgaead through Panama

Import with importlib (the directory name carries a hyphen):
  wg = importlib.import_module("wireguard-java_amd")
"""
from ._lib import WgError, lib  # noqa: F401
from .engine import Engine, default_engine, desc_as_int64, pack_desc, selftest, WG_PKT_DTYPE  # noqa: F401
