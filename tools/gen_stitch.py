#!/usr/bin/env python3
"""Generates wireguard-java_amd/csrc/wg_stitch.h: the first half of a ChaCha20 block's rounds with the
four Poly1305 Horner steps of a slot lane's previous round interleaved into it (one asm statement).

Why: inside a wave the transport kernel ran each round's phases in sequence
(DMA, ChaCha20, XOR/store, Horner), so the Horner steps' dependent v_mad_u64_u32 chains could only hide
behind other waves, which reach them at the same point of their packets. The MAC input of round k - 1
(the ciphertext in the wave's LDS image) is independent of round k's keystream (ChaCha20Poly1305.java:40-56
for open, :31-38 for seal), so round k - 1's Horner steps can run between round k's ARX instructions.

Layout of the statement (operands):
  %0..%15   x0..x15   ChaCha20 state (in/out)
  %16..%20  H0..H4    the lane's Horner accumulator (in/out; radix 2^26)
  %21..%25  N0..N4    the other accumulator set (scratch: steps alternate H -> N -> H, four steps end in H)
  %26..%29  W0..W3    the step's 16-B chunk (scratch, four ds_read_b32)
  %30       sgpr pair: the v_mad_u64_u32 carry-out (unused)
  %31..%35  R0..R4    R = r^G limbs (inputs from here on)
  %36..%39  S1..S4    5 R1..5 R4
  %40       the LDS byte address of the lane's first chunk of the window
  %41       sgpr: 0x3ffffff
  %42       sgpr: 1 << 24 (the chunk's 2^128 bit in limb 4)
  %43       vgpr: the 2^128 bit of step 0's chunk (0 for a lane whose first step of a packet's round 0 is a
            virtual chunk before the data: it reads the zeroed key-block lane, and without the bit it adds 0)
  v[62:63]  the 64-bit accumulator of one limb's product chain (clobbered: a register pair's halves
            cannot be named through an asm operand)
Every instruction is an 8-byte encoding (VOP3 / DS), so the placed stream keeps the ChaCha20 rounds'
issue rate; each s_waitcnt is paired with an s_nop 0 (two 4-byte instructions).
Step t reads its chunk at %39 + 4 G t (chunks c0 + G t of the slot, one row of the image).
Horner step (poly_mul of wg_device.h, then the chunk's limbs added): acc' = acc R + m, carry-seeded chains.
"""
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "wireguard-java_amd", "csrc", "wg_stitch.h")

X = [f"%{i}" for i in range(16)]
HSET = [f"%{16 + i}" for i in range(5)]
NSET = [f"%{21 + i}" for i in range(5)]
W = [f"%{26 + i}" for i in range(4)]
CC = "%30"
R = [f"%{31 + i}" for i in range(5)]
S = [None] + [f"%{36 + i}" for i in range(4)]
ADDR, M26, HIB, HIB0 = "%40", "%41", "%42", "%43"
D, DLO, DHI = "v[62:63]", "v62", "v63"


def chacha_instrs(first_dr, n_dr):
    """ChaCha20 rounds (hoisted form: the first double round starts from column 0's quarter round
    only, columns 1..3 of the first column round are done per packet) as a list of instructions."""
    def A(a, b):
        return f"v_add_u32_e64 {X[a]}, {X[a]}, {X[b]}"

    def Xo(d, a):
        return f"v_xor_b32_e64 {X[d]}, {X[d]}, {X[a]}"

    def Ro(d, s):
        return f"v_alignbit_b32 {X[d]}, {X[d]}, {X[d]}, {s}"

    def step4(q, s):
        out = [A(p, r) for p, r, _ in q] + [Xo(t, p) for p, _, t in q] + [Ro(t, s) for _, _, t in q]
        return out

    def qr4(cols):
        a = [(c[0], c[1], c[3]) for c in cols]
        c_ = [(c[2], c[3], c[1]) for c in cols]
        return step4(a, 16) + step4(c_, 20) + step4(a, 24) + step4(c_, 25)

    def qr1(a, b, c, d):
        return [A(a, b), Xo(d, a), Ro(d, 16), A(c, d), Xo(b, c), Ro(b, 20), A(a, b), Xo(d, a), Ro(d, 24),
                A(c, d), Xo(b, c), Ro(b, 25)]

    cols = [(0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15)]
    diags = [(0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)]
    out = []
    for dr in range(first_dr, first_dr + n_dr):
        if dr == 0:
            out += qr1(0, 4, 8, 12) + qr4(diags)
        else:
            out += qr4(cols) + qr4(diags)
    return out


def horner_step(t, G, H, N, last):
    """One Horner step: N = H * R + chunk t (limbs), the chunk read by this step's ds_read_b32 x4 (issued
    at the end of the previous step, or before the first ChaCha20 instruction for step 0)."""
    mads = {
        0: [(4, S[1]), (3, S[2]), (2, S[3]), (1, S[4]), (0, R[0])],
        1: [(0, R[1]), (1, R[0]), (2, S[4]), (3, S[3]), (4, S[2])],
        2: [(0, R[2]), (1, R[1]), (2, R[0]), (3, S[4]), (4, S[3])],
        3: [(0, R[3]), (1, R[2]), (2, R[1]), (3, R[0]), (4, S[4])],
        4: [(0, R[4]), (1, R[3]), (2, R[2]), (3, R[1]), (4, R[0])],
    }
    out = []
    for limb in range(5):
        for k, (h, r) in enumerate(mads[limb]):
            c = "0" if (limb == 0 and k == 0) else D
            out.append(f"v_mad_u64_u32 {D}, {CC}, {H[h]}, {r}, {c}")
        out.append(f"v_and_b32_e64 {N[limb]}, {DLO}, {M26}")
        if limb < 4:
            out.append(f"v_lshrrev_b64 {D}, 26, {D}")
    # 2^130 wrap: N0 += 5 (d4 >> 26); carry N0's bit 26 into N1
    out.append(f"v_alignbit_b32 {DLO}, {DHI}, {DLO}, 26")
    out.append(f"v_lshl_add_u32 {DLO}, {DLO}, 2, {DLO}")
    out.append(f"v_add_u32_e64 {N[0]}, {N[0]}, {DLO}")
    out.append(f"v_lshrrev_b32_e64 {DLO}, 26, {N[0]}")
    out.append(f"v_and_b32_e64 {N[0]}, {N[0]}, {M26}")
    out.append(f"v_add_u32_e64 {N[1]}, {N[1]}, {DLO}")
    # the chunk: wait for its four dwords, add its limbs
    out.append("WAIT")
    out.append(f"v_and_b32_e64 {DLO}, {W[0]}, {M26}")
    out.append(f"v_add_u32_e64 {N[0]}, {N[0]}, {DLO}")
    for k, sh in ((1, 26), (2, 20), (3, 14)):
        out.append(f"v_alignbit_b32 {DLO}, {W[k]}, {W[k - 1]}, {sh}")
        out.append(f"v_and_b32_e64 {DLO}, {DLO}, {M26}")
        out.append(f"v_add_u32_e64 {N[k]}, {N[k]}, {DLO}")
    out.append(f"v_lshrrev_b32_e64 {DLO}, 8, {W[3]}")
    out.append(f"v_add3_u32 {N[4]}, {N[4]}, {DLO}, {HIB0 if t == 0 else HIB}")
    if not last:
        out += loads(t + 1, G)
    return out


def loads(t, G):
    base = 4 * G * t  # step t: G/4 lanes of 16 B further along the image row
    return [f"ds_read_b32 {W[k]}, {ADDR} offset:{base + 4 * k}" for k in range(4)]


def merge(arx, hor):
    """Spread the Horner instructions evenly between the ARX instructions (ARX first)."""
    out = []
    n, m = len(arx), len(hor)
    j = 0
    for i, a in enumerate(arx):
        out.append(a)
        want = (i + 1) * m // n
        while j < want:
            out.append(hor[j])
            j += 1
    out += hor[j:]
    return out


def emit(lines):
    res = []
    for ln in lines:
        if ln == "WAIT":
            res.append("s_waitcnt lgkmcnt(0)")
            res.append("s_nop 0")
        else:
            res.append(ln)
    return "\\n\"\n    \"".join(res)


def gen(G, n_dr_a):
    arx = chacha_instrs(0, n_dr_a)
    hor = []
    sets = [(HSET, NSET), (NSET, HSET), (HSET, NSET), (NSET, HSET)]
    for t in range(4):
        hor += horner_step(t, G, sets[t][0], sets[t][1], t == 3)
    body = loads(0, G) + merge(arx, hor)
    return body


HEADER = '''// wg_stitch.h — GENERATED by tools/gen_stitch.py; do not edit by hand.
//
// ChaCha20 rounds with a slot lane's four Poly1305 Horner steps of the previous round interleaved
// (VERDICT r05 item 1; design in tools/gen_stitch.py and DESIGN.md §4.1 "Stitched Horner"). Reference
// semantics: chacha_permute (chacha-generic.c:10-55) and poly1305_blocks (poly1305-donna-64.h:101-151)
// in radix 2^26, as wg_device.h's chacha20_rounds_hoisted_asm and poly_mul.
#pragma once
#include <stdint.h>

namespace wgd {

constexpr int kStitchDR = {NDR};  // double rounds in the stitched first part (the rest: chacha20_rounds_tail_asm)

#define WG_STITCH_OPS(x, h, n, r, s, w, addr, m26, cc, hib, hib0)                                          \\
  : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),       \\
    "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]), \\
    "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]),                                           \\
    "=&v"(n[0]), "=&v"(n[1]), "=&v"(n[2]), "=&v"(n[3]), "=&v"(n[4]),                                      \\
    "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&s"(cc)                                         \\
  : "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]),                                                \\
    "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]),                                                           \\
    "v"(addr), "s"(m26), "s"(hib), "v"(hib0)                                                              \\
  : "v62", "v63", "memory"
'''

FUNC = '''
// G = {G}: the first {NDR} double rounds (hoisted form) of x with four Horner steps on acc:
// acc = ((((acc R + m0) R + m1) R + m2) R + m3), m_t the 16-B chunk at LDS byte address addr + {STEP} t.
template <>
__device__ __forceinline__ void chacha20_rounds_stitch_asm<{G}>(uint32_t x[16], uint32_t acc[5], const uint32_t R[5],
                                                                const uint32_t Rs[4], uint32_t addr, uint32_t hib0) {
  uint32_t n[5], w[4];
  const uint32_t m26 = 0x3ffffffu, hib = 1u << 24;
  uint64_t cc;
  asm volatile(
    ".p2align 3\\n\\ts_nop 0\\n\\t"
    "{BODY}\\n"
    WG_STITCH_OPS(x, acc, n, R, Rs, w, addr, m26, cc, hib, hib0));
  (void)n; (void)w; (void)cc;
}
'''

TAIL = '''
// the remaining double rounds of a block whose first kStitchDR ran in chacha20_rounds_stitch_asm or
// chacha20_rounds_head_asm
__device__ __forceinline__ void chacha20_rounds_tail_asm(uint32_t x[16]) {
  asm volatile(WG_PLACE {TAILDR} : WG_X16(x));
}
// the first kStitchDR double rounds without Horner steps (no slot of the wave has a pending round)
__device__ __forceinline__ void chacha20_rounds_head_asm(uint32_t x[16]) {
  asm volatile(WG_PLACE WG_QR1(0, 4, 8, 12) WG_DIAGS {HEADDR} : WG_X16(x));
}

}  // namespace wgd
'''


def main():
    ndr = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    s = HEADER.replace("{NDR}", str(ndr))
    s += '''
template <int G>
__device__ __forceinline__ void chacha20_rounds_stitch_asm(uint32_t x[16], uint32_t acc[5], const uint32_t R[5],
                                                           const uint32_t Rs[4], uint32_t addr, uint32_t hib0);
'''
    for G in (4, 8, 16):
        body = emit(gen(G, ndr))
        s += FUNC.replace("{G}", str(G)).replace("{NDR}", str(ndr)).replace("{STEP}", str(4 * G)).replace(
            "{BODY}", body)
    s += TAIL.replace("{TAILDR}", " ".join(["WG_DR"] * (10 - ndr))).replace(
        "{HEADDR}", " ".join(["WG_DR"] * (ndr - 1)))
    open(OUT, "w").write(s)
    print(f"wrote {OUT}: {ndr} stitched double rounds")


if __name__ == "__main__":
    main()
