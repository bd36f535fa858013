// wg_device.h — gfx950 device arithmetic for the transport AEAD.
//
// ChaCha20 block (RFC 8439 2.3) restated for 64-wide CDNA4 waves: one lane owns
// one 64-byte counter block in 16 VGPRs. Reference semantics:
//   chacha_permute / chacha_block_generic  ax.xz.wireguard.noise/src/main/c/chacha-generic.c:10-78
//   state layout (constants, key, ctr, nonce) ChaCha20.java:55-74
// Poly1305 (RFC 8439 2.5) in radix 2^26 (5 limbs in VGPRs) with v_mad_u64_u32
// products; canonical final reduction as poly1305-donna-64.h:154-223.
//
// Measured on MI355X (tools/microbench2.hip): v_add/v_xor issue at
// ~60 T lane-op/s, every shift/rotate/perm/3-operand op at ~35 T, v_mad_u64_u32 at
// ~30 T. The rotates therefore set the ChaCha20 cost; 16/8-bit rotates use
// v_perm_b32 (measured 1-3% ahead of v_alignbit_b32).
#pragma once

#ifndef WG_CHACHA_UNROLL
#define WG_CHACHA_UNROLL 3  // double rounds per loop trip of chacha20_block_hoisted (9 in all)
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wgd {

constexpr uint32_t M26 = 0x3ffffffu;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }

#define WG_QR(a, b, c, d)                \
  a += b; d ^= a; d = rotl16(d);         \
  c += d; b ^= c; b = rotl(b, 12);       \
  a += b; d ^= a; d = rotl8(d);          \
  c += d; b ^= c; b = rotl(b, 7);

// Keystream block for (key, 32-bit block counter, nonce words n0..n2).
// out[i] = permute(state)[i] + state[i], i.e. little-endian keystream words.
__device__ __forceinline__ void chacha20_block(const uint32_t k[8], uint32_t ctr, uint32_t n0, uint32_t n1,
                                               uint32_t n2, uint32_t out[16]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll 2
  for (int r = 0; r < 10; ++r) {
    WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
    WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
  }
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
  out[4] = x4 + k[0]; out[5] = x5 + k[1]; out[6] = x6 + k[2]; out[7] = x7 + k[3];
  out[8] = x8 + k[4]; out[9] = x9 + k[5]; out[10] = x10 + k[6]; out[11] = x11 + k[7];
  out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}
// rotl16(d ^ a) as two SDWA xors, one per 16-bit half (the halves swap places):
// VOP2-SDWA issue instead of v_xor_b32 + v_perm_b32 (tools/microbench6.hip).
__device__ __forceinline__ uint32_t xor_rotl16_sdwa(uint32_t d, uint32_t a) {
  uint32_t t;
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(t) : "v"(d), "v"(a));
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
      : "+v"(t) : "v"(d), "v"(a));
  return t;
}

#define WG_QR_SDWA(a, b, c, d)             \
  a += b; d = xor_rotl16_sdwa(d, a);       \
  c += d; b ^= c; b = rotl(b, 12);         \
  a += b; d ^= a; d = rotl8(d);            \
  c += d; b ^= c; b = rotl(b, 7);

// Same block, key read from LDS twice (before the rounds and again for the
// feed-forward) so the 8 key words are not live across the 20 rounds; the
// "memory" clobber keeps the compiler from merging the two reads.
// SDWA: rotl16 as two SDWA xors instead of v_xor + v_perm.
template <bool SDWA = false>
__device__ __forceinline__ void chacha20_block_lds(const uint4* key_lds, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                   uint32_t n2, uint32_t out[16]) {
  uint4 ka = key_lds[0], kb = key_lds[1];
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = ka.x, x5 = ka.y, x6 = ka.z, x7 = ka.w, x8 = kb.x, x9 = kb.y, x10 = kb.z, x11 = kb.w;
  uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll 2
  for (int r = 0; r < 10; ++r) {
    if constexpr (SDWA) {
      WG_QR_SDWA(x0, x4, x8, x12) WG_QR_SDWA(x1, x5, x9, x13) WG_QR_SDWA(x2, x6, x10, x14) WG_QR_SDWA(x3, x7, x11, x15)
      WG_QR_SDWA(x0, x5, x10, x15) WG_QR_SDWA(x1, x6, x11, x12) WG_QR_SDWA(x2, x7, x8, x13) WG_QR_SDWA(x3, x4, x9, x14)
    } else {
      WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
      WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
    }
  }
  asm volatile("" ::: "memory");
  ka = key_lds[0];
  kb = key_lds[1];
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
  out[4] = x4 + ka.x; out[5] = x5 + ka.y; out[6] = x6 + ka.z; out[7] = x7 + ka.w;
  out[8] = x8 + kb.x; out[9] = x9 + kb.y; out[10] = x10 + kb.z; out[11] = x11 + kb.w;
  out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}
// One ChaCha20 column quarter round on its own (the per-packet part of the first round).
__device__ __forceinline__ void chacha20_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) { WG_QR(a, b, c, d) }

// ---- ChaCha20 rounds as placed VOP3 code (gfx950 issue rate) ---------------------------
// Measured on MI355X (tools/microbench16-18): a ChaCha20 double round issues
// at 3.9-4.1 cycles per wave-instruction (8 waves per SIMD) as the compiler emits it (4-byte
// VOP2 v_add/v_xor mixed with 8-byte v_alignbit), and at 3.35-3.48 when EVERY instruction is
// an 8-byte VOP3 encoding placed at an address = 4 mod 8 (the same stream at 0 mod 8: 4.0).
// So the rounds are one asm block of _e64 encodings, started by `.p2align 3; s_nop 0` (the
// nop executes once per block). Operands %0..%15 are state words x0..x15; the order inside a
// step is grouped (the four columns' adds, then xors, then rotates), rotl(x, n) =
// v_alignbit(x, x, 32 - n).
#define WG_A(a, b) "v_add_u32_e64 %" #a ", %" #a ", %" #b "\n"
#define WG_X(d, a) "v_xor_b32_e64 %" #d ", %" #d ", %" #a "\n"
#define WG_R(d, s) "v_alignbit_b32 %" #d ", %" #d ", %" #d ", " #s "\n"
#define WG_STEP4(p0, q0, t0, p1, q1, t1, p2, q2, t2, p3, q3, t3, s)                         \
  WG_A(p0, q0) WG_A(p1, q1) WG_A(p2, q2) WG_A(p3, q3) WG_X(t0, p0) WG_X(t1, p1) WG_X(t2, p2) \
  WG_X(t3, p3) WG_R(t0, s) WG_R(t1, s) WG_R(t2, s) WG_R(t3, s)
// four quarter rounds (a_i, b_i, c_i, d_i), i = 0..3, interleaved step by step
#define WG_QR4(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3)     \
  WG_STEP4(a0, b0, d0, a1, b1, d1, a2, b2, d2, a3, b3, d3, 16)                     \
  WG_STEP4(c0, d0, b0, c1, d1, b1, c2, d2, b2, c3, d3, b3, 20)                     \
  WG_STEP4(a0, b0, d0, a1, b1, d1, a2, b2, d2, a3, b3, d3, 24)                     \
  WG_STEP4(c0, d0, b0, c1, d1, b1, c2, d2, b2, c3, d3, b3, 25)
#define WG_QR1(a, b, c, d)                                                                  \
  WG_A(a, b) WG_X(d, a) WG_R(d, 16) WG_A(c, d) WG_X(b, c) WG_R(b, 20) WG_A(a, b) WG_X(d, a) \
  WG_R(d, 24) WG_A(c, d) WG_X(b, c) WG_R(b, 25)
#define WG_COLS WG_QR4(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
#define WG_DIAGS WG_QR4(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14)
#define WG_DR WG_COLS WG_DIAGS
#define WG_PLACE ".p2align 3\ns_nop 0\n"
#define WG_X16(x)                                                                                       \
  "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),       \
      "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])

// the 20 rounds of chacha_permute (chacha-generic.c:10-55) on x[0..15]
__device__ __forceinline__ void chacha20_rounds_asm(uint32_t x[16]) {
  asm volatile(WG_PLACE WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR : WG_X16(x));
}
// the same with columns 1..3 of the first column round already applied (chacha20_block_hoisted)
__device__ __forceinline__ void chacha20_rounds_hoisted_asm(uint32_t x[16]) {
  asm volatile(WG_PLACE WG_QR1(0, 4, 8, 12) WG_DIAGS WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR WG_DR
               : WG_X16(x));
}

#ifndef WG_CHACHA_ASM
#define WG_CHACHA_ASM 1
#endif

// Same block with the first column round of columns 1..3 already done: they depend only on
// the key and the nonce (state words 13..15), not on the block counter, so a packet computes
// them once (H = {x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15} after that round)
// and every block of the packet starts from column 0's quarter round.
__device__ __forceinline__ void chacha20_block_hoisted(const uint4* key_lds, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                       uint32_t n2, const uint32_t H[12], uint32_t out[16]) {
  uint4 ka = key_lds[0], kb = key_lds[1];
#if WG_CHACHA_ASM
  uint32_t y[16] = {0x61707865u, H[0], H[4], H[8], ka.x, H[1], H[5], H[9],
                    kb.x,        H[2], H[6], H[10], ctr, H[3], H[7], H[11]};
  chacha20_rounds_hoisted_asm(y);
  asm volatile("" ::: "memory");
  ka = key_lds[0];
  kb = key_lds[1];
  out[0] = y[0] + 0x61707865u; out[1] = y[1] + 0x3320646eu; out[2] = y[2] + 0x79622d32u; out[3] = y[3] + 0x6b206574u;
  out[4] = y[4] + ka.x; out[5] = y[5] + ka.y; out[6] = y[6] + ka.z; out[7] = y[7] + ka.w;
  out[8] = y[8] + kb.x; out[9] = y[9] + kb.y; out[10] = y[10] + kb.z; out[11] = y[11] + kb.w;
  out[12] = y[12] + ctr; out[13] = y[13] + n0; out[14] = y[14] + n1; out[15] = y[15] + n2;
  return;
#endif
  uint32_t x0 = 0x61707865u, x4 = ka.x, x8 = kb.x, x12 = ctr;
  uint32_t x1 = H[0], x5 = H[1], x9 = H[2], x13 = H[3];
  uint32_t x2 = H[4], x6 = H[5], x10 = H[6], x14 = H[7];
  uint32_t x3 = H[8], x7 = H[9], x11 = H[10], x15 = H[11];
  WG_QR(x0, x4, x8, x12)
  WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
#pragma unroll WG_CHACHA_UNROLL
  for (int r = 1; r < 10; ++r) {
    WG_QR(x0, x4, x8, x12) WG_QR(x1, x5, x9, x13) WG_QR(x2, x6, x10, x14) WG_QR(x3, x7, x11, x15)
    WG_QR(x0, x5, x10, x15) WG_QR(x1, x6, x11, x12) WG_QR(x2, x7, x8, x13) WG_QR(x3, x4, x9, x14)
  }
  asm volatile("" ::: "memory");
  ka = key_lds[0];
  kb = key_lds[1];
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
  out[4] = x4 + ka.x; out[5] = x5 + ka.y; out[6] = x6 + ka.z; out[7] = x7 + ka.w;
  out[8] = x8 + kb.x; out[9] = x9 + kb.y; out[10] = x10 + kb.z; out[11] = x11 + kb.w;
  out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}
// A whole block without the hoisted first column round (2-lane slots, which have no lanes to compute it on
// for the others): the same placed asm over all 20 rounds, then the feed-forward.
__device__ __forceinline__ void chacha20_block_full(const uint4* key_lds, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                    uint32_t n2, uint32_t out[16]) {
  uint4 ka = key_lds[0], kb = key_lds[1];
  uint32_t y[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, ka.x, ka.y, ka.z, ka.w,
                    kb.x,        kb.y,        kb.z,        kb.w,        ctr,  n0,   n1,   n2};
  chacha20_rounds_asm(y);
  asm volatile("" ::: "memory");
  ka = key_lds[0];
  kb = key_lds[1];
  out[0] = y[0] + 0x61707865u; out[1] = y[1] + 0x3320646eu; out[2] = y[2] + 0x79622d32u; out[3] = y[3] + 0x6b206574u;
  out[4] = y[4] + ka.x; out[5] = y[5] + ka.y; out[6] = y[6] + ka.z; out[7] = y[7] + ka.w;
  out[8] = y[8] + kb.x; out[9] = y[9] + kb.y; out[10] = y[10] + kb.z; out[11] = y[11] + kb.w;
  out[12] = y[12] + ctr; out[13] = y[13] + n0; out[14] = y[14] + n1; out[15] = y[15] + n2;
}
#undef WG_QR
#undef WG_QR_SDWA

// ---- Poly1305, radix 2^26 -------------------------------------------------
// An element of Z/(2^130-5) as 5 limbs h[i] (value = sum h[i] 2^(26 i)), kept
// partially reduced (limbs < 2^26 + 2^8 after poly_mul; < 2^27 after adding one
// message block).

// 16 message bytes (four LE words) -> limbs; hibit = 1<<24 adds 2^128 (full block).
__device__ __forceinline__ void poly_block_limbs(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t hibit,
                                                 uint32_t c[5]) {
  c[0] = w0 & M26;
  c[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
  c[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
  c[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
  c[4] = (w3 >> 8) | hibit;
}

// r from the first 16 bytes of the one-time key, clamped as in
// poly1305-donna-64.h:80-86 (r &= 0x0ffffffc0ffffffc0ffffffc0fffffff).
__device__ __forceinline__ void poly_r_limbs(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t r[5]) {
  poly_block_limbs(k0 & 0x0fffffffu, k1 & 0x0ffffffcu, k2 & 0x0ffffffcu, k3 & 0x0ffffffcu, 0u, r);
}

// h = h * r mod 2^130-5 (partial reduction). s[i] = 5 * r[i] for i = 1..4.
// Bounds: h limbs < 2^27, r limbs < 2^26 => each d_i < 2^58 (so the 26-bit
// carries fit 32 bits) and the wrap carry from d4 is < 2^29.3 (so 5c < 2^32).
// Each limb's carry seeds the next limb's v_mad_u64_u32 accumulator chain, so a
// step costs 25 mads + 5 alignbits + 5 ands (+ the 2^130 wrap) and no 64-bit adds.
// one v_mad_u64_u32 (d = a * b + c) as an asm statement: a chain of them keeps each limb's carry in
// the accumulator instead of a separate 64-bit add
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return d;
}
// The same product visible to the compiler. Between two dependent asm statements the hazard
// recognizer inserts an s_nop 0 (it cannot see into them); other waves on the SIMD hide those in the
// transport kernels, a wave on its own pays them (the per-packet server's Poly1305 wave, wg_pp.hip).
__device__ __forceinline__ uint64_t mad64c(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
#ifdef WG_POLY_C  // the plain-C product (the compiler adds each limb's carry with a separate 64-bit add)
template <bool ASM = true>
__device__ __forceinline__ void poly_mul(uint32_t h[5], const uint32_t r[5], const uint32_t s[5]) {
  const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
  uint64_t d = (uint64_t)h0 * r[0] + (uint64_t)h1 * s[4] + (uint64_t)h2 * s[3] + (uint64_t)h3 * s[2] +
               (uint64_t)h4 * s[1];
  h[0] = (uint32_t)d & M26;
  d = (uint64_t)(uint32_t)(d >> 26) + (uint64_t)h0 * r[1] + (uint64_t)h1 * r[0] + (uint64_t)h2 * s[4] +
      (uint64_t)h3 * s[3] + (uint64_t)h4 * s[2];
  h[1] = (uint32_t)d & M26;
  d = (uint64_t)(uint32_t)(d >> 26) + (uint64_t)h0 * r[2] + (uint64_t)h1 * r[1] + (uint64_t)h2 * r[0] +
      (uint64_t)h3 * s[4] + (uint64_t)h4 * s[3];
  h[2] = (uint32_t)d & M26;
  d = (uint64_t)(uint32_t)(d >> 26) + (uint64_t)h0 * r[3] + (uint64_t)h1 * r[2] + (uint64_t)h2 * r[1] +
      (uint64_t)h3 * r[0] + (uint64_t)h4 * s[4];
  h[3] = (uint32_t)d & M26;
  d = (uint64_t)(uint32_t)(d >> 26) + (uint64_t)h0 * r[4] + (uint64_t)h1 * r[3] + (uint64_t)h2 * r[2] +
      (uint64_t)h3 * r[1] + (uint64_t)h4 * r[0];
  h[4] = (uint32_t)d & M26;
  uint32_t c = (uint32_t)(d >> 26);
  h[0] += c * 5u;
  c = h[0] >> 26; h[0] &= M26;
  h[1] += c;
}
#else
// Default: each v_mad_u64_u32 as an asm statement, so every limb's chain starts from the
// previous limb's carry instead of the compiler adding the carry to a separately formed
// chain: -1.4% VALU instructions per k_transport launch (SQ_INSTS_VALU 37.70 M -> 37.18 M on
// C1), bit-exact. ASM = false: the same chains with compiler-visible products (mad64c).
// One limb's five products as ONE asm statement: d = a0 b0 + a1 b1 + ... + a4 b4 + c, a chain of dependent
// v_mad_u64_u32 with no pads inside (the compiler pads only at an asm statement's boundary, so five chains
// per product cost 5 s_nop 0 instead of the 25 of one asm statement per v_mad_u64_u32).
__device__ __forceinline__ uint64_t mad5(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                                         uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint64_t c) {
  uint64_t d, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %12\n\t"
      "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %7, %0\n\t"
      "v_mad_u64_u32 %0, %1, %8, %9, %0\n\t"
      "v_mad_u64_u32 %0, %1, %10, %11, %0"
      : "=&v"(d), "=&s"(cc)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(c));
  return d;
}
__device__ __forceinline__ uint64_t mad5z(uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                                          uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4) {  // mad5 with c = 0
  uint64_t d, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0\n\t"
      "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %7, %0\n\t"
      "v_mad_u64_u32 %0, %1, %8, %9, %0\n\t"
      "v_mad_u64_u32 %0, %1, %10, %11, %0"
      : "=&v"(d), "=&s"(cc)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4));
  return d;
}
template <bool ASM = true>
__device__ __forceinline__ void poly_mul(uint32_t h[5], const uint32_t r[5], const uint32_t s[5]) {
#ifdef WG_POLY_CHAIN5
  if constexpr (ASM) {
    const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
    uint64_t d = mad5z(h4, s[1], h3, s[2], h2, s[3], h1, s[4], h0, r[0]);
    h[0] = (uint32_t)d & M26;
    d = mad5(h0, r[1], h1, r[0], h2, s[4], h3, s[3], h4, s[2], d >> 26);
    h[1] = (uint32_t)d & M26;
    d = mad5(h0, r[2], h1, r[1], h2, r[0], h3, s[4], h4, s[3], d >> 26);
    h[2] = (uint32_t)d & M26;
    d = mad5(h0, r[3], h1, r[2], h2, r[1], h3, r[0], h4, s[4], d >> 26);
    h[3] = (uint32_t)d & M26;
    d = mad5(h0, r[4], h1, r[3], h2, r[2], h3, r[1], h4, r[0], d >> 26);
    h[4] = (uint32_t)d & M26;
    uint32_t c = (uint32_t)(d >> 26);
    h[0] += c * 5u;
    c = h[0] >> 26; h[0] &= M26;
    h[1] += c;
    return;
  }
#endif
  auto mad = [](uint32_t a, uint32_t b, uint64_t c) { return ASM ? mad64(a, b, c) : mad64c(a, b, c); };
  const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
  uint64_t d = mad(h0, r[0], mad(h1, s[4], mad(h2, s[3], mad(h3, s[2], (uint64_t)h4 * s[1]))));
  h[0] = (uint32_t)d & M26;
  d = mad(h4, s[2], mad(h3, s[3], mad(h2, s[4], mad(h1, r[0], mad(h0, r[1], d >> 26)))));
  h[1] = (uint32_t)d & M26;
  d = mad(h4, s[3], mad(h3, s[4], mad(h2, r[0], mad(h1, r[1], mad(h0, r[2], d >> 26)))));
  h[2] = (uint32_t)d & M26;
  d = mad(h4, s[4], mad(h3, r[0], mad(h2, r[1], mad(h1, r[2], mad(h0, r[3], d >> 26)))));
  h[3] = (uint32_t)d & M26;
  d = mad(h4, r[0], mad(h3, r[1], mad(h2, r[2], mad(h1, r[3], mad(h0, r[4], d >> 26)))));
  h[4] = (uint32_t)d & M26;
  uint32_t c = (uint32_t)(d >> 26);
  h[0] += c * 5u;
  c = h[0] >> 26; h[0] &= M26;
  h[1] += c;
}
#endif

// Two Horner steps in one reduction: h = h * q + m * r (q = r^2; the caller adds the next
// chunk), both products in one carry-seeded v_mad_u64_u32 chain per limb (tools/microbench20.hip
// variant C: 239.9 cycles per chunk and wave against 281.9 for two poly_mul steps). Bounds: h < 2^27,
// m < 2^26, q and r limbs < 2^26 + 2^8 => each limb sum < 2^60; limb 4 holds no 5x terms, so its
// sum is < 2^56 and the wrap carry c < 2^30, whose 5c is added in 64 bits.
__device__ __forceinline__ void poly_mul2(uint32_t h[5], const uint32_t q[5], const uint32_t qs[5], const uint32_t m[5],
                                          const uint32_t r[5], const uint32_t s[5]) {
  const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
  uint64_t d = mad64(h0, q[0], mad64(h1, qs[4], mad64(h2, qs[3], mad64(h3, qs[2], (uint64_t)h4 * qs[1]))));
  d = mad64(m[0], r[0], mad64(m[1], s[4], mad64(m[2], s[3], mad64(m[3], s[2], mad64(m[4], s[1], d)))));
  h[0] = (uint32_t)d & M26;
  d = mad64(h4, qs[2], mad64(h3, qs[3], mad64(h2, qs[4], mad64(h1, q[0], mad64(h0, q[1], d >> 26)))));
  d = mad64(m[4], s[2], mad64(m[3], s[3], mad64(m[2], s[4], mad64(m[1], r[0], mad64(m[0], r[1], d)))));
  h[1] = (uint32_t)d & M26;
  d = mad64(h4, qs[3], mad64(h3, qs[4], mad64(h2, q[0], mad64(h1, q[1], mad64(h0, q[2], d >> 26)))));
  d = mad64(m[4], s[3], mad64(m[3], s[4], mad64(m[2], r[0], mad64(m[1], r[1], mad64(m[0], r[2], d)))));
  h[2] = (uint32_t)d & M26;
  d = mad64(h4, qs[4], mad64(h3, q[0], mad64(h2, q[1], mad64(h1, q[2], mad64(h0, q[3], d >> 26)))));
  d = mad64(m[4], s[4], mad64(m[3], r[0], mad64(m[2], r[1], mad64(m[1], r[2], mad64(m[0], r[3], d)))));
  h[3] = (uint32_t)d & M26;
  d = mad64(h4, q[0], mad64(h3, q[1], mad64(h2, q[2], mad64(h1, q[3], mad64(h0, q[4], d >> 26)))));
  d = mad64(m[4], r[0], mad64(m[3], r[1], mad64(m[2], r[2], mad64(m[1], r[3], mad64(m[0], r[4], d)))));
  h[4] = (uint32_t)d & M26;
  const uint64_t t = (uint64_t)(uint32_t)(d >> 26) * 5u + h[0];
  h[0] = (uint32_t)t & M26;
  h[1] += (uint32_t)(t >> 26);
}

__device__ __forceinline__ void poly_scale5(const uint32_t r[5], uint32_t s[5]) {
  s[0] = 0;
  s[1] = r[1] * 5u; s[2] = r[2] * 5u; s[3] = r[3] * 5u; s[4] = r[4] * 5u;
}

// Full carry, canonical reduction (h < p), + s mod 2^128 -> tag words.
// Input limbs may be as large as 2^32 - 1 (sum of up to 63 partial products).
__device__ __forceinline__ void poly_finish(uint32_t h[5], uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                            uint32_t tag[4]) {
  uint32_t c;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    c = h[0] >> 26; h[0] &= M26; h[1] += c;
    c = h[1] >> 26; h[1] &= M26; h[2] += c;
    c = h[2] >> 26; h[2] &= M26; h[3] += c;
    c = h[3] >> 26; h[3] &= M26; h[4] += c;
    c = h[4] >> 26; h[4] &= M26; h[0] += c * 5u;
  }
  // non-wrapping normalisation: limbs 0..3 canonical, h4 <= 2^26, so h < 2p
  c = h[0] >> 26; h[0] &= M26; h[1] += c;
  c = h[1] >> 26; h[1] &= M26; h[2] += c;
  c = h[2] >> 26; h[2] &= M26; h[3] += c;
  c = h[3] >> 26; h[3] &= M26; h[4] += c;
  // g = h + 5 - 2^130; take g when it does not borrow (h >= p)
  uint32_t g0 = h[0] + 5u; c = g0 >> 26; g0 &= M26;
  uint32_t g1 = h[1] + c; c = g1 >> 26; g1 &= M26;
  uint32_t g2 = h[2] + c; c = g2 >> 26; g2 &= M26;
  uint32_t g3 = h[3] + c; c = g3 >> 26; g3 &= M26;
  uint32_t g4 = h[4] + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1u;  // all ones if h >= p
  h[0] = (h[0] & ~mask) | (g0 & mask);
  h[1] = (h[1] & ~mask) | (g1 & mask);
  h[2] = (h[2] & ~mask) | (g2 & mask);
  h[3] = (h[3] & ~mask) | (g3 & mask);
  h[4] = (h[4] & ~mask) | (g4 & mask);
  // h mod 2^128 as four words, then + s
  uint32_t w0 = h[0] | (h[1] << 26);
  uint32_t w1 = (h[1] >> 6) | (h[2] << 20);
  uint32_t w2 = (h[2] >> 12) | (h[3] << 14);
  uint32_t w3 = (h[3] >> 18) | (h[4] << 8);
  uint64_t f = (uint64_t)w0 + s0; tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + s1 + (f >> 32); tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + s2 + (f >> 32); tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + s3 + (f >> 32); tag[3] = (uint32_t)f;
}

}  // namespace wgd
