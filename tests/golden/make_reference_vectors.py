"""Extract the reference's own known-answer vectors into reference_vectors.json.

Reads the reference test sources and the donna self-test AS TEXT (no reference
code is run) and transcribes their byte arrays:
  ax.xz.wireguard.noise/src/test/java/ax/xz/wireguard/noise/crypto/ChaCha20Test.java
  ax.xz.wireguard.noise/src/test/java/ax/xz/wireguard/noise/crypto/Poly1305Test.java
  ax.xz.wireguard.noise/src/main/c/poly1305-donna.c  (poly1305_power_on_self_test)
Run once in the build container (where /root/reference exists); the JSON it
writes is the committed fixture. Usage: python tests/golden/make_reference_vectors.py
"""
import json
import os
import re

REF = os.environ.get("WG_REFERENCE", "/root/reference")
NOISE = os.path.join(REF, "ax.xz.wireguard.noise/src")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")


def java_bytes(src: str, name: str) -> bytes:
    """byte[] NAME = { ... } (with or without (byte) casts)."""
    m = re.search(r"byte\[\]\s+" + re.escape(name) + r"\s*=\s*\{(.*?)\};", src, re.S)
    assert m, name
    vals = re.findall(r"0x([0-9a-fA-F]{1,2})", m.group(1))
    return bytes(int(v, 16) for v in vals)


def java_bytes_in(block: str, name: str) -> bytes:
    return java_bytes(block, name)


def method_body(src: str, method: str) -> str:
    i = src.index("void " + method + "(")
    j = src.index("\t@Test", i + 1) if "\t@Test" in src[i + 1:] else len(src)
    return src[i:j]


def c_bytes(src: str, name: str) -> bytes:
    m = re.search(r"static const unsigned char " + re.escape(name) + r"\[(\d+)\]\s*=\s*\{(.*?)\};", src, re.S)
    assert m, name
    vals = bytes(int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]{2})", m.group(2)))
    return vals + b"\x00" * (int(m.group(1)) - len(vals))  # C zero-fills the rest of the array


def main():
    cc = open(os.path.join(NOISE, "test/java/ax/xz/wireguard/noise/crypto/ChaCha20Test.java")).read()
    pc = open(os.path.join(NOISE, "test/java/ax/xz/wireguard/noise/crypto/Poly1305Test.java")).read()
    dc = open(os.path.join(NOISE, "main/c/poly1305-donna.c")).read()
    sunscreen = re.search(r'var plaintext = "(Ladies[^"]*)"', cc).group(1)
    v = {"_source": "transcribed from the reference's own tests by tests/golden/make_reference_vectors.py"}

    key = java_bytes(cc, "TEST_KEY")
    n0 = java_bytes(cc, "TEST_NONCE_0")
    n1 = java_bytes(cc, "TEST_NONCE_1")
    init_words = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{8})", method_body(cc, "initializeState"))]
    v["chacha20_state"] = {"ref": "ChaCha20Test.java:111-125", "key": key.hex(), "nonce": n0.hex(), "counter": 1,
                           "words": init_words}
    v["chacha20_block"] = {"ref": "ChaCha20Test.java:127-145 (RFC 8439 2.3.2)", "key": key.hex(), "nonce": n0.hex(),
                           "counter": 1, "out": java_bytes(method_body(cc, "chacha20Block"), "expectedOutputByte").hex()}
    v["chacha20"] = {"ref": "ChaCha20Test.java:147-168 (RFC 8439 2.4.2)", "key": key.hex(), "nonce": n1.hex(),
                     "counter": 1, "pt": sunscreen.encode().hex(),
                     "ct": java_bytes(method_body(cc, "chacha20"), "expectedCiphertext").hex()}
    qr = method_body(cc, "quarterRound")
    words = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{8})", qr)]
    v["quarter_round"] = {"ref": "ChaCha20Test.java:28-87 (RFC 8439 2.1.1, 2.2.1)",
                          "qr_in": words[0:4], "qr_out": words[4:8], "state_in": words[8:24],
                          "state_out": words[24:40], "indices": [2, 7, 8, 13]}

    v["poly1305"] = {"ref": "Poly1305Test.java:49-61 (RFC 8439 2.5.2)", "key": java_bytes(pc, "TEST_KEY").hex(),
                     "msg": b"Cryptographic Forum Research Group".hex(),
                     "tag": java_bytes(method_body(pc, "testPoly1305"), "expectedTag").hex()}
    kg = method_body(pc, "poly1305ChaChaKeyGen")
    v["poly1305_keygen"] = {"ref": "Poly1305Test.java:117-149 (RFC 8439 2.6.2)", "key": java_bytes(kg, "key").hex(),
                            "nonce": java_bytes(kg, "nonce").hex(), "otk": java_bytes(kg, "expectedOutput").hex()}
    ae = method_body(pc, "poly1305AeadEncrypt")
    v["aead"] = {"ref": "Poly1305Test.java:151-199 (RFC 8439 2.8.2)", "aad": java_bytes(ae, "aad").hex(),
                 "key": java_bytes(ae, "key").hex(), "nonce": java_bytes(ae, "nonce").hex(),
                 "pt": sunscreen.encode().hex(), "ct": java_bytes(ae, "expectedCiphertext").hex(),
                 "tag": java_bytes(ae, "expectedTag").hex()}

    v["donna_nacl"] = {"ref": "poly1305-donna.c:85-116", "key": c_bytes(dc, "nacl_key").hex(),
                       "msg": c_bytes(dc, "nacl_msg").hex(), "tag": c_bytes(dc, "nacl_mac").hex()}
    v["donna_wrap"] = {"ref": "poly1305-donna.c:118-134", "key": c_bytes(dc, "wrap_key").hex(),
                       "msg": c_bytes(dc, "wrap_msg").hex(), "tag": c_bytes(dc, "wrap_mac").hex()}
    v["donna_total"] = {"ref": "poly1305-donna.c:136-198 (MAC of the MACs of messages i^i, i = 0..255)",
                        "key": c_bytes(dc, "total_key").hex(), "tag": c_bytes(dc, "total_mac").hex()}
    with open(OUT, "w") as f:
        json.dump(v, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
