"""The stitched Horner schedule of wg_transport.hip (ST) restated lane by lane in Python: a slot of G lanes, its
rounds' LDS image as the XOR phase leaves it, the previous round's four steps per lane run in the next round
(window [4 G kp - 4, 4 G kp + 4 G - 4), the zeroed key-block lane supplying round 0's chunks -4..-1 without
the 2^128 bit) and the packet's last round sequential after its XOR phase, with the same index formulas as the
kernel. Every lane's accumulator must equal the plain Horner evaluation of its residue class of MAC chunks
(the sequential kernel's per-lane invariant; poly1305-donna-64.h:101-151 restated with multiplier R = r^G),
over lengths 0..3000, 9000 and 65535, for G = 4, 8 and 16. CPU only."""
import random

import pytest

from test_stitch_asm import P, chunk_limbs, poly_mul, val


def lane_accumulators(G, L, R, rng):
    JM, SH = G - 1, G.bit_length() - 1
    nc = (L + 15) // 16
    M = nc + 1
    D = G * ((M + JM) >> SH) - M
    chunks = [[rng.getrandbits(32) for _ in range(4)] for _ in range(nc)] + [[0, 0, L, 0]]
    nb = ((L + 63) >> 6) + 1
    acc = [[0] * 5 for _ in range(G)]

    def image(rnd):  # (row, lane) -> chunk words, as the XOR phase (and the length-block lane) leave them
        im = {}
        for j in range(G):
            b = G * rnd + j
            for q in range(4):
                ci = 4 * (b - 1) + q
                im[(q, j)] = [0, 0, 0, 0] if b == 0 else (chunks[ci] if ci <= nc else None)
        return im

    rnd = 0
    while True:
        last = G * (rnd + 1) >= nb
        im = image(rnd)
        for j in range(G):
            if not last:  # these four steps run stitched into round rnd + 1's ChaCha20 rounds
                kp = rnd
                u = 4 * G * kp + ((j - ((4 * G * kp - 4 + D) & JM)) & JM)
                lanepart = ((u >> 2) - G * kp) & (G // 4 - 1)
                for t in range(4):
                    m = chunk_limbs(im[(u & 3, lanepart + (G // 4) * t)])
                    if kp == 0 and u < 4 and t == 0:
                        m[4] -= 1 << 24  # hib0 = 0
                    acc[j] = [a + b for a, b in zip(poly_mul(acc[j], R), m)]
            else:  # the packet's last round: its own steps after its XOR phase (unchanged sequential code)
                c_lo = 4 * G * rnd - 4 if rnd else 0
                c_end = min(nc + 1, 4 * G * rnd + 4 * G - 4)
                c0 = c_lo + ((j - ((c_lo + D) & JM)) & JM)
                for t in range(4):
                    ci = c0 + G * t
                    if ci < c_end:
                        if rnd or t:
                            acc[j] = poly_mul(acc[j], R)
                        acc[j] = [a + b for a, b in zip(acc[j], chunk_limbs(im[(ci & 3, (ci >> 2) + 1 - G * rnd)]))]
        if last:
            if nc >= 4 * G * rnd + 4 * G - 4:  # the length block after the last round: lane JM at the finish
                acc[JM] = [a + b for a, b in zip(poly_mul(acc[JM], R), chunk_limbs([0, 0, L, 0]))]
            break
        rnd += 1
    want = []
    for j in range(G):
        a = 0
        for c in range(nc + 1):
            if (c + D) % G == j:
                a = (a * val(R) + val(chunk_limbs(chunks[c]))) % P
        want.append(a)
    return [val(a) % P for a in acc], want


@pytest.mark.parametrize("G", [4, 8, 16])
def test_stitched_schedule_keeps_every_lane_accumulator(G):
    rng = random.Random(G)
    R = [rng.getrandbits(26) for _ in range(5)]
    for L in list(range(0, 3000, 13)) + [1420, 9000, 65535]:
        got, want = lane_accumulators(G, L, R, rng)
        assert got == want, (G, L)
