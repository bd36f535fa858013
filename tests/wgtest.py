"""Shared test helpers: deterministic inputs and the package import."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MASK64 = (1 << 64) - 1


def splitmix_bytes(seed: int, n: int) -> bytes:
    """splitmix64 byte stream (the BASELINE.md input generator)."""
    out = bytearray()
    x = seed & MASK64
    while len(out) < n:
        x = (x + 0x9E3779B97F4A7C15) & MASK64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


def splitmix_np(seed: int, n: int) -> np.ndarray:
    """Vectorised splitmix64 stream of n bytes (same bytes as splitmix_bytes)."""
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) + np.arange(1, words + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def wg():
    return importlib.import_module("wireguard-java_amd")


def noise():
    return importlib.import_module("wireguard-java_amd.noise")


def oracle():
    return importlib.import_module("oracle.oracle")
