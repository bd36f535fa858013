// wg_lane.h — k_lane: the transport seal/open kernel laid out as K lanes per packet.
//
// Each packet is split into K contiguous ranges of ChaCha20 counter blocks, one per
// lane; lane h owns blocks [hQ, min(nb, (h+1)Q)) with nb = ceil(len/64) + 1 and
// Q = ceil(nb/K) (block 0 is the Poly1305 one-time key, ChaCha20Poly1305.java:11-14;
// data block b uses counter b, :36,55). A lane streams its range block by block:
// keystream in registers, 64 payload bytes in (prefetched one block ahead), XOR,
// 64 bytes out, and the block's ciphertext chunks go straight into the lane's own
// Poly1305 Horner accumulator. No LDS, no barriers, no block-to-lane transposes.
//
// Poly1305 per lane (the MAC input of a range is contiguous, so a lane multiplies by
// r itself): radix 2^32, four 32-bit limbs + a small top limb, the clamped r making
// every column of the product fit 64 bits (r_i < 2^28, 4 | r_1..r_3 so that
// s_i = r_i + r_i/4 = 5 r_i / 4 folds the 2^130 = 5 wrap exactly) — 20 v_mad_u64_u32
// per 16-byte chunk and no shifts. This is the same polynomial as
// poly1305-donna-64.h:75-152 (h = (h + m) r mod 2^130-5), evaluated in another radix.
//
// Combining the K partial Horner sums: lane h's sum A_h covers positions ending at its
// range's last chunk, so tag = sum_h A_h r^(e_h) + s with e_h = chunks after the range
// (+1 for the length block); e_h is raised per lane by square-and-multiply in radix
// 2^26 (wg_device.h poly_mul), the K products are added with lane shuffles, and the
// group's first lane runs the canonical finish (poly1305-donna-64.h:154-223).
//
// Reference path: ChaCha20Poly1305.java:31-60 (seal/open), SymmetricKeypair.java:52-83
// (nonce = LE64(counter) || 0^4), chacha-generic.c:81-108.
#pragma once

namespace wgk {

// h = (h + m + 2^128) * r  mod 2^130 - 5, partially reduced (h4 <= 4 on exit).
// r0 < 2^28, r1..r3 < 2^28 and divisible by 4 (clamped), s_i = r_i + (r_i >> 2).
__device__ __forceinline__ void p32_block(uint32_t h[5], uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                          uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s1,
                                          uint32_t s2, uint32_t s3) {
  uint64_t d0 = (uint64_t)h[0] + m0;
  uint64_t d1 = (uint64_t)h[1] + m1 + (d0 >> 32);
  uint64_t d2 = (uint64_t)h[2] + m2 + (d1 >> 32);
  uint64_t d3 = (uint64_t)h[3] + m3 + (d2 >> 32);
  const uint32_t h0 = (uint32_t)d0, h1 = (uint32_t)d1, h2 = (uint32_t)d2, h3 = (uint32_t)d3;
  uint32_t h4 = h[4] + (uint32_t)(d3 >> 32) + 1u;  // <= 6
  d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s3 + (uint64_t)h2 * s2 + (uint64_t)h3 * s1;
  d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)(h4 * s1);
  d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s3 + (uint64_t)(h4 * s2);
  d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)(h4 * s3);
  h4 *= r0;
  d1 += d0 >> 32;
  d2 += d1 >> 32;
  d3 += d2 >> 32;
  h4 += (uint32_t)(d3 >> 32);
  // fold bits >= 2^130: (h4 >> 2) * 5
  const uint32_t c = (h4 >> 2) + (h4 & ~3u);
  h4 &= 3u;
  uint64_t t = (uint64_t)(uint32_t)d0 + c;
  h[0] = (uint32_t)t;
  t = (uint64_t)(uint32_t)d1 + (t >> 32);
  h[1] = (uint32_t)t;
  t = (uint64_t)(uint32_t)d2 + (t >> 32);
  h[2] = (uint32_t)t;
  t = (uint64_t)(uint32_t)d3 + (t >> 32);
  h[3] = (uint32_t)t;
  h[4] = h4 + (uint32_t)(t >> 32);
}

__device__ __forceinline__ void mul26(uint32_t x[5], const uint32_t y[5]) {
  uint32_t ys[5];
  poly_scale5(y, ys);
  poly_mul(x, y, ys);
}

// Variant bits V: 1 prefetch the next block's payload one round ahead,
// 2 s_setprio by progress (earlier rounds first).
template <int MODE, int K, int V>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K >= 8 ? 8 : (K >= 4 ? 4 : 2))))
k_lane(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  static_assert(K == 1 || K == 2 || K == 4 || K == 8, "lanes per packet");
  const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t pkt = (uint32_t)(gid / K), h = (uint32_t)(gid % K);
  const bool in_grid = gid < (uint64_t)P.n * K;

  uint4 lo = make_uint4(0, 0, 0, 0), hi = make_uint4(0, 0, 0, 0);
  if (in_grid) {
    const uint4* dp = (const uint4*)(P.desc + pkt);
    lo = dp[0];
    hi = dp[1];
  }
  const uint64_t in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
  const uint64_t out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
  const uint32_t ctr_lo = hi.x, ctr_hi = hi.y, len = hi.z, kslot = hi.w;
  bool valid = in_grid && len <= P.max_len && kslot < P.key_slots;
  {
    const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
    valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
  }
  const uint32_t nb = ((len + 63u) >> 6) + 1u;  // block 0 + data blocks
  const uint32_t Q = (nb + K - 1u) / K;         // blocks per lane
  const uint32_t b0 = h * Q;
  const uint32_t nr = (valid && b0 < nb) ? min(Q, nb - b0) : 0u;  // this lane's rounds
  const uint8_t* src = P.in + in_off;
  uint8_t* dst = P.out + out_off;

  uint4 ka = make_uint4(0, 0, 0, 0), kb = make_uint4(0, 0, 0, 0);
  if (valid) {
    const uint4* kp = (const uint4*)(P.keys + 8u * kslot);
    ka = kp[0];
    kb = kp[1];
  }
  const uint32_t key[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};

  uint32_t acc[5] = {0, 0, 0, 0, 0};
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, sv0 = 0, sv1 = 0, sv2 = 0, sv3 = 0;
  uint32_t wn[16];
  if constexpr ((V & 1) != 0) {
    if (nr > 0 && b0 > 0) {
      const uint32_t off = 64u * (b0 - 1u);
      load_block(src + off, min(64u, len - off), wn);
    }
  }

  for (uint32_t t = 0; __any(t < nr); ++t) {
    if constexpr ((V & 2) != 0) {
      if (t == 0) __builtin_amdgcn_s_setprio(2);
      else if (t == 2) __builtin_amdgcn_s_setprio(1);
      else if (t == 4) __builtin_amdgcn_s_setprio(0);
    }
    const bool act = t < nr;
    const uint32_t b = b0 + t;
    const bool data = act && b > 0;
    const uint32_t off = 64u * (b - 1u);
    const uint32_t nbytes = data ? min(64u, len - off) : 0u;
    uint32_t w[16];
    if constexpr ((V & 1) != 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = wn[i];
      if (t + 1u < nr) {  // next round's block of this lane (always a data block)
        const uint32_t noff = off + 64u;
        load_block(src + noff, min(64u, len - noff), wn);
      }
    } else {
      if (data) load_block(src + off, nbytes, w);
    }
    uint32_t nch = 0;
    if (act) {
      uint32_t ks[16];
      chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
      if (!data) {  // block 0: the Poly1305 one-time key r || s
        r0 = ks[0] & 0x0fffffffu;
        r1 = ks[1] & 0x0ffffffcu;
        r2 = ks[2] & 0x0ffffffcu;
        r3 = ks[3] & 0x0ffffffcu;
        sv0 = ks[4]; sv1 = ks[5]; sv2 = ks[6]; sv3 = ks[7];
      } else {
        if constexpr (MODE == WG_MODE_OPEN) {
          if (nbytes < 64u) mask_block(nbytes, w);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t c = w[i];
            w[i] ^= ks[i];
            ks[i] = c;  // ks now holds the MAC input (the ciphertext)
          }
          store_block(dst + off, nbytes, w);
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] = ks[i];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
          store_block(dst + off, nbytes, w);
          if (nbytes < 64u) mask_block(nbytes, w);
        }
        nch = (nbytes + 15u) >> 4;
      }
    }
    if (K > 1 && t == 0) {  // the group's r from its first lane (which ran block 0)
      const int src_lane = (int)((threadIdx.x & 63u) & ~(uint32_t)(K - 1));
      r0 = __shfl(r0, src_lane, 64);
      r1 = __shfl(r1, src_lane, 64);
      r2 = __shfl(r2, src_lane, 64);
      r3 = __shfl(r3, src_lane, 64);
    }
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
#pragma unroll
    for (uint32_t c = 0; c < 4u; ++c)
      if (c < nch) p32_block(acc, w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3], r0, r1, r2, r3, s1, s2, s3);
  }

  // the length block le64(0) || le64(len) closes the last data range (or block 0's)
  const uint32_t h_last = (nb - 1u) / Q;
  if (valid && h == h_last) {
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    p32_block(acc, 0u, 0u, len, 0u, r0, r1, r2, r3, s1, s2, s3);
  }
  uint32_t A[5];
  poly_block_limbs(acc[0], acc[1], acc[2], acc[3], acc[4] << 24, A);  // radix 2^26, limbs < 2^27
  if constexpr (K > 1) {
    // A_h * r^e, e = chunks after this lane's range, the length block included
    const uint32_t nc = (len + 15u) >> 4;
    uint32_t e = (valid && h < h_last) ? nc + 5u - 4u * (h + 1u) * Q : 0u;
    if (__any(e != 0u)) {
      uint32_t base[5], pw[5];
      poly_r_limbs(r0, r1, r2, r3, base);
#pragma unroll
      for (int i = 0; i < 5; ++i) pw[i] = 0;
      bool have = false;
      const bool need = e != 0u;
      while (__any(e != 0u)) {
        if (e & 1u) {
          if (have) {
            mul26(pw, base);
          } else {
#pragma unroll
            for (int i = 0; i < 5; ++i) pw[i] = base[i];
            have = true;
          }
        }
        e >>= 1;
        if (e != 0u) {
          uint32_t tmp[5];
#pragma unroll
          for (int i = 0; i < 5; ++i) tmp[i] = base[i];
          mul26(base, tmp);
        }
      }
      if (need) mul26(A, pw);
    }
#pragma unroll
    for (int off = 1; off < K; off <<= 1) {
#pragma unroll
      for (int i = 0; i < 5; ++i) A[i] += __shfl_xor(A[i], off, 64);
    }
  }

  uint32_t bad = valid ? 0u : 1u;
  if (h == 0 && valid) {
    uint32_t tag[4];
    poly_finish(A, sv0, sv1, sv2, sv3, tag);
    if constexpr (MODE == WG_MODE_SEAL) {
      uint8_t* tp = dst + len;
      if ((((uintptr_t)tp) & 15u) == 0) {
        *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
      }
    } else {  // all 16 bytes compared, no early exit
      const uint8_t* tp = src + len;
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
      bad = diff ? 1u : 0u;
    }
  }
  if constexpr (MODE == WG_MODE_OPEN) {
    if constexpr (K > 1) bad = __shfl(bad, (int)((threadIdx.x & 63u) & ~(uint32_t)(K - 1)), 64);
    if (in_grid && h == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
    if (bad && valid) {  // scrub the unauthenticated plaintext this lane wrote
      uint32_t z[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) z[i] = 0;
      for (uint32_t t = 0; t < nr; ++t) {
        const uint32_t b = b0 + t;
        if (b == 0) continue;
        const uint32_t off = 64u * (b - 1u);
        store_block(dst + off, min(64u, len - off), z);
      }
    }
  }
}

}  // namespace wgk
