"""Generate transport_vectors.json: SymmetricKeypair.cipher outputs for the
reference's nonce layout (LE64(counter) || 0^4, SymmetricKeypair.java:52-61).

Each case is sealed by the pure-Python oracle (oracle/oracle.py py_aead_seal) and
cross-checked against OpenSSL's independent EVP_chacha20_poly1305 with the same
12-byte nonce before it is written; generation aborts on any disagreement.
Payloads and keys are derived from a splitmix64 stream (tests/wgtest.py
splitmix_bytes) so the fixture stores only seeds, lengths and results.
Usage: python tests/golden/make_transport_vectors.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))
from oracle import oracle as O  # noqa: E402
from wgtest import splitmix_bytes  # noqa: E402

LENGTHS = [0, 1, 2, 3, 4, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 127, 128, 129, 255, 256, 576, 1280, 1420,
           1500, 2032, 4080, 4096, 9000]


def main():
    cases = []
    seed = 0x5EED2026
    counters = [0, 1, 2, 255, 256, 65535, 1 << 32, (1 << 32) - 1, (1 << 63) + 12345, (1 << 64) - 1]
    i = 0
    for L in LENGTHS + [int.from_bytes(splitmix_bytes(seed + 1000 + k, 2), "little") % 9001 for k in range(40)]:
        for ctr in (counters[i % len(counters)], counters[(i * 7 + 3) % len(counters)]):
            key = splitmix_bytes(seed + 2 * i, 32)
            pt = splitmix_bytes(seed + 2 * i + 1, L)
            nonce = O.transport_nonce(ctr)
            ct_tag = O.py_aead_seal(key, nonce, pt)
            ssl = O.openssl_seal(key, nonce, pt)
            if ssl is not None and ssl != ct_tag:
                raise SystemExit(f"OpenSSL disagrees for len={L} counter={ctr}")
            case = {"key": key.hex(), "counter": ctr, "len": L, "pt_seed": seed + 2 * i + 1,
                    "tag": ct_tag[-16:].hex(), "sha256": hashlib.sha256(ct_tag).hexdigest()}
            if L <= 128:
                case["ct_tag"] = ct_tag.hex()
            cases.append(case)
            i += 1
    with open(os.path.join(HERE, "transport_vectors.json"), "w") as f:
        json.dump({"_source": "oracle/oracle.py py_aead_seal, cross-checked with OpenSSL EVP_chacha20_poly1305; "
                              "nonce = LE64(counter)||0^4 (SymmetricKeypair.java:52-61)",
                   "openssl_checked": O.openssl() is not None, "cases": cases}, f, indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
