"""CPU model of the k_lane-family arithmetic (wireguard-java_amd/csrc/wg_lane.h), checked
against the oracle: the radix-2^32 Poly1305 step on the clamped r (p32_block) with every
intermediate kept inside the machine word the kernel uses, and the K-lane split of a
packet into contiguous block ranges recombined with r^e_h, e_h = nc + 5 - 4 (h+1) Q.
The GPU parity tests check the kernels themselves; this pins the algebra they rely on."""
import numpy as np
import pytest

from wgtest import oracle, splitmix_bytes

O = oracle()
P130 = (1 << 130) - 5
M32, M64 = (1 << 32) - 1, (1 << 64) - 1


def addc(a, b, c):
    t = a + b + c
    assert a <= M32 and b <= M32
    return t & M32, t >> 32


def p32_block(h, m, r):
    """wg_lane.h p32_block: h = (h + m + 2^128) r mod 2^130-5, partially reduced."""
    r0, r1, r2, r3 = r
    s1, s2, s3 = r1 + (r1 >> 2), r2 + (r2 >> 2), r3 + (r3 >> 2)
    h0, c = addc(h[0], m[0], 0)
    h1, c = addc(h[1], m[1], c)
    h2, c = addc(h[2], m[2], c)
    h3, c = addc(h[3], m[3], c)
    h4 = h[4] + c + 1
    assert h4 <= 6
    d0 = h0 * r0 + h1 * s3 + h2 * s2 + h3 * s1
    d1 = h0 * r1 + h1 * r0 + h2 * s3 + h3 * s2 + h4 * s1
    d2 = h0 * r2 + h1 * r1 + h2 * r0 + h3 * s3 + h4 * s2
    d3 = h0 * r3 + h1 * r2 + h2 * r1 + h3 * r0 + h4 * s3
    assert max(d0, d1, d2, d3) <= M64  # every column fits one v_mad_u64_u32 chain
    t4 = h4 * r0
    assert t4 <= M32
    e0 = d0 & M32
    e1, c = addc(d1 & M32, d0 >> 32, 0)
    f1 = (d1 >> 32) + c
    e2, c = addc(d2 & M32, f1, 0)
    f2 = (d2 >> 32) + c
    e3, c = addc(d3 & M32, f2, 0)
    f3 = (d3 >> 32) + c
    e4 = t4 + f3
    assert e4 <= M32
    q = e4 >> 2
    k = q + (q << 2)
    assert k <= M32
    e4 &= 3
    n0, c = addc(e0, k, 0)
    n1, c = addc(e1, 0, c)
    n2, c = addc(e2, 0, c)
    n3, c = addc(e3, 0, c)
    out = [n0, n1, n2, n3, e4 + c]
    assert out[4] <= 4
    return out


def val(h):
    return h[0] | h[1] << 32 | h[2] << 64 | h[3] << 96 | h[4] << 128


def words(b16):
    return list(np.frombuffer(b16, "<u4").astype(object))


def lane_tag(otk: bytes, ct: bytes, K: int) -> bytes:
    """The tag as K lanes of k_lane compute it (ChaCha20Poly1305.java:63-93 MAC input)."""
    L = len(ct)
    r = [w & m for w, m in zip(words(otk[:16]), [0x0FFFFFFF, 0x0FFFFFFC, 0x0FFFFFFC, 0x0FFFFFFC])]
    rr = val(r + [0])
    s = int.from_bytes(otk[16:32], "little")
    nb = (L + 63) // 64 + 1
    Q = (nb + K - 1) // K
    nc = (L + 15) // 16
    h_last = (nb - 1) // Q
    pad = ct + bytes(-L % 16)
    total = 0
    for h in range(K):
        acc = [0, 0, 0, 0, 0]
        for b in range(h * Q, min(nb, (h + 1) * Q)):
            if b == 0:
                continue  # the one-time-key block
            for c in range(4):
                off = 64 * (b - 1) + 16 * c
                if off < L:
                    acc = p32_block(acc, words(pad[off:off + 16]), r)
        if h == h_last:
            acc = p32_block(acc, [0, 0, L & M32, L >> 32], r)
        e = nc + 5 - 4 * (h + 1) * Q if h < h_last else 0
        total += val(acc) * pow(rr, e, P130)
    return ((total % P130 + s) & ((1 << 128) - 1)).to_bytes(16, "little")


@pytest.mark.parametrize("K", [1, 2, 4, 8])
@pytest.mark.parametrize("L", [0, 1, 15, 16, 63, 64, 65, 127, 704, 1420, 4080, 9000])
def test_k_lane_tag_matches_oracle(K, L):
    key = splitmix_bytes(7 + L, 32)
    nonce = O.transport_nonce(1000 + L)
    pt = splitmix_bytes(11 + L, L)
    ct_tag = O.c_aead_seal(key, nonce, pt)
    otk = O.py_poly1305_keygen(key, nonce)
    assert lane_tag(otk, ct_tag[:L], K) == ct_tag[L:]


def test_p32_block_extreme_limbs():
    """Largest clamped r and a saturated accumulator stay inside the word bounds."""
    r = [0x0FFFFFFF, 0x0FFFFFFC, 0x0FFFFFFC, 0x0FFFFFFC]
    h = [M32, M32, M32, M32, 4]
    out = p32_block(h, [M32] * 4, r)
    want = (val(h) + ((1 << 128) | val([M32] * 4 + [0]))) * val(r + [0]) % P130
    assert val(out) % P130 == want
