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
// Carry chains are written with __builtin_addc so they lower to v_add_co_u32 /
// v_addc_co_u32 pairs; the 20 products are v_mad_u64_u32 accumulation chains.
__device__ __forceinline__ void p32_block(uint32_t h[5], uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                          uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s1,
                                          uint32_t s2, uint32_t s3) {
  unsigned c;
  const uint32_t h0 = __builtin_addc(h[0], m0, 0u, &c);
  const uint32_t h1 = __builtin_addc(h[1], m1, c, &c);
  const uint32_t h2 = __builtin_addc(h[2], m2, c, &c);
  const uint32_t h3 = __builtin_addc(h[3], m3, c, &c);
  const uint32_t h4 = h[4] + c + 1u;  // <= 6
  const uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s3 + (uint64_t)h2 * s2 + (uint64_t)h3 * s1;
  const uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
  const uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
  const uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s3;
  const uint32_t t4 = (uint32_t)((uint64_t)h4 * r0);  // < 2^31: one v_mad_u64_u32, not a quarter-rate v_mul_lo
  // h4:h0 = t4 << 128 + d3 << 96 + d2 << 64 + d1 << 32 + d0
  const uint32_t e0 = (uint32_t)d0;
  const uint32_t e1 = __builtin_addc((uint32_t)d1, (uint32_t)(d0 >> 32), 0u, &c);
  const uint32_t f1 = (uint32_t)(d1 >> 32) + c;
  const uint32_t e2 = __builtin_addc((uint32_t)d2, f1, 0u, &c);
  const uint32_t f2 = (uint32_t)(d2 >> 32) + c;
  const uint32_t e3 = __builtin_addc((uint32_t)d3, f2, 0u, &c);
  const uint32_t f3 = (uint32_t)(d3 >> 32) + c;
  uint32_t e4 = t4 + f3;
  // fold bits >= 2^130: (e4 >> 2) * 5
  const uint32_t q = e4 >> 2;
  const uint32_t k = q + (q << 2);
  e4 &= 3u;
  h[0] = __builtin_addc(e0, k, 0u, &c);
  h[1] = __builtin_addc(e1, 0u, c, &c);
  h[2] = __builtin_addc(e2, 0u, c, &c);
  h[3] = __builtin_addc(e3, 0u, c, &c);
  h[4] = e4 + c;
}

__device__ __forceinline__ void mul26(uint32_t x[5], const uint32_t y[5]) {
  uint32_t ys[5];
  poly_scale5(y, ys);
  poly_mul(x, y, ys);
}

// Variant bits V: 1 prefetch the next block's payload one round ahead,
// 2 s_setprio by progress (earlier rounds first), 4 one-wave workgroups (64 threads;
// otherwise 256) so the dispatcher spreads a small grid evenly over the SIMDs.
// Timing ablations (results are wrong; tools/ablate.py only): 8 no payload loads or
// stores, 16 no Poly1305 chunk steps, 32 no ChaCha20 keystream.
template <int V>
constexpr int lane_wg_threads() { return (V & 4) ? 64 : 256; }

template <int MODE, int K, int V>
__global__ void __launch_bounds__(lane_wg_threads<V>()) __attribute__((amdgpu_waves_per_eu(K >= 8 ? 8 : (K >= 4 ? 4 : 2))))
k_lane(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  static_assert(K == 1 || K == 2 || K == 4 || K == 8, "lanes per packet");
  const uint64_t gid = (uint64_t)blockIdx.x * lane_wg_threads<V>() + threadIdx.x;
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
  if constexpr ((V & 9) == 1) {
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
    if constexpr ((V & 8) != 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = t * 0x9e3779b9u + (uint32_t)i;
    } else if constexpr ((V & 1) != 0) {
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
      if constexpr ((V & 32) != 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] = key[i & 7] + b * (uint32_t)i;
      } else {
        chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
      }
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
          if constexpr ((V & 8) == 0) store_block(dst + off, nbytes, w);
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] = ks[i];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
          if constexpr ((V & 8) == 0) store_block(dst + off, nbytes, w);
          if (nbytes < 64u) mask_block(nbytes, w);
        }
        nch = (V & 16) ? 0u : (nbytes + 15u) >> 4;
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


// ---------------------------------------------------------------------------
// k_quad — k_lane with K = 4 (a quad of lanes per packet) and quad-cooperative
// payload IO. In k_lane every lane streams its own 64-byte block, so one
// global_load/store_dwordx4 of a wave touches 64 different cache lines (64 x 16 B),
// and the memory pipeline, not the VALU, set the pace (timing ablation).
// Here the four lanes of a packet move one 64-byte block together: in access i,
// lane h loads chunk h of quad-mate i's block, so a wave instruction reads 16
// contiguous 64-byte blocks. A per-wave LDS exchange (rows of 80 B) hands every lane
// its own block before the rounds, and gathers the output blocks back for the
// cooperative stores. Arithmetic, ranges and the Poly1305 combine are k_lane's.
__device__ __forceinline__ void store_chunk16(uint8_t* p, uint32_t n, const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const bool a4 = (((uintptr_t)p) & 3u) == 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = (int)n - 4 * k;
    if (r >= 4 && a4) *(uint32_t*)(p + 4 * k) = w[k];
    else if (r > 0) st_bytes(p + 4 * k, w[k], r < 4 ? r : 4);
  }
}

// orders this wave's LDS accesses around lane-crossing exchanges (LDS is in order per
// wave; the clobber keeps the compiler from moving accesses across)
__device__ __forceinline__ void quad_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// V: 2 s_setprio by progress; timing ablations: 16 no Poly1305 chunk steps, 32 no keystream
template <int MODE, int V>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) k_quad(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  constexpr uint32_t K = 4, ROW = 5;  // row stride in uint4 (64 B of payload + 16 B pad)
  __shared__ uint4 xch[64 * ROW];
  const uint32_t lane = threadIdx.x;
  const uint64_t gid = (uint64_t)blockIdx.x * 64u + lane;
  const uint32_t pkt = (uint32_t)(gid / K), h = (uint32_t)(gid % K);
  const uint32_t qb = lane & ~(K - 1u);
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
  const uint32_t nb = ((len + 63u) >> 6) + 1u;
  const uint32_t Q = (nb + K - 1u) / K;
  const uint32_t b0 = h * Q;
  const uint32_t nr = (valid && b0 < nb) ? min(Q, nb - b0) : 0u;
  const uint8_t* src = P.in + in_off;
  uint8_t* dst = P.out + out_off;

  uint4 ka = make_uint4(0, 0, 0, 0), kb = make_uint4(0, 0, 0, 0);
  if (valid) {
    const uint4* kp = (const uint4*)(P.keys + 8u * kslot);
    ka = kp[0];
    kb = kp[1];
  }
  const uint32_t key[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};

  // byte offset of chunk h of quad-mate i's block at round t, or ~0u when that chunk
  // holds no payload (block 0, past the mate's range, or past the packet)
  auto chunk_off = [&](uint32_t i, uint32_t t) -> uint32_t {
    const uint32_t bi = i * Q + t;
    const bool in_range = valid && i * Q < nb && t < Q && bi < nb && bi > 0;
    const uint32_t off = 64u * (bi - 1u) + 16u * h;
    return (in_range && off < len) ? off : ~0u;
  };
  auto load_chunk = [&](uint32_t i, uint32_t t) -> uint4 {
    const uint32_t off = chunk_off(i, t);
    if (off == ~0u) return make_uint4(0, 0, 0, 0);
    const uint8_t* q = src + off;
    if (len - off >= 16u && (((uintptr_t)q) & 15u) == 0) return *(const uint4*)q;
    uint32_t w4[4];
    load_chunk16(q, min(16u, len - off), w4);
    return make_uint4(w4[0], w4[1], w4[2], w4[3]);
  };

  uint32_t acc[5] = {0, 0, 0, 0, 0};
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, sv0 = 0, sv1 = 0, sv2 = 0, sv3 = 0;
  uint4 pre[4];
#pragma unroll
  for (uint32_t i = 0; i < K; ++i) pre[i] = load_chunk(i, 0);

  for (uint32_t t = 0; __any(t < nr); ++t) {
    if constexpr ((V & 2) != 0) {
      if (t == 0) __builtin_amdgcn_s_setprio(2);
      else if (t == 2) __builtin_amdgcn_s_setprio(1);
      else if (t == 4) __builtin_amdgcn_s_setprio(0);
    }
    // hand each lane its own block: chunk h of mate i goes to row qb + i
    quad_lds_sync();
#pragma unroll
    for (uint32_t i = 0; i < K; ++i) xch[(qb + i) * ROW + h] = pre[i];
    quad_lds_sync();
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = xch[lane * ROW + j];
      w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
    // next round's chunks are in flight during this round's keystream
#pragma unroll
    for (uint32_t i = 0; i < K; ++i) pre[i] = load_chunk(i, t + 1u);

    const bool act = t < nr;
    const uint32_t b = b0 + t;
    const bool data = act && b > 0;
    const uint32_t off = 64u * (b - 1u);
    const uint32_t nbytes = data ? min(64u, len - off) : 0u;
    uint32_t nch = 0;
    uint32_t o[16];
    if (act) {
      uint32_t ks[16];
      if constexpr ((V & 32) != 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] = key[i & 7] + b * (uint32_t)i;
      } else {
        chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
      }
      if (!data) {
        r0 = ks[0] & 0x0fffffffu;
        r1 = ks[1] & 0x0ffffffcu;
        r2 = ks[2] & 0x0ffffffcu;
        r3 = ks[3] & 0x0ffffffcu;
        sv0 = ks[4]; sv1 = ks[5]; sv2 = ks[6]; sv3 = ks[7];
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] = w[i] ^ ks[i];
        if constexpr (MODE == WG_MODE_SEAL) {
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] = o[i];  // MAC input: the ciphertext
        }
        if (nbytes < 64u) mask_block(nbytes, w);
        nch = (V & 16) ? 0u : (nbytes + 15u) >> 4;
      }
    }
    // gather the output blocks back and store them cooperatively
    quad_lds_sync();
    if (data) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xch[lane * ROW + j] = make_uint4(o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]);
    }
    quad_lds_sync();
#pragma unroll
    for (uint32_t i = 0; i < K; ++i) {
      const uint32_t co = chunk_off(i, t);
      if (co != ~0u) {
        const uint4 v = xch[(qb + i) * ROW + h];
        uint8_t* q = dst + co;
        if (len - co >= 16u && (((uintptr_t)q) & 15u) == 0) *(uint4*)q = v;
        else store_chunk16(q, min(16u, len - co), v);
      }
    }

    if (t == 0) {  // the group's r from its first lane (which ran block 0)
      r0 = __shfl(r0, (int)qb, 64);
      r1 = __shfl(r1, (int)qb, 64);
      r2 = __shfl(r2, (int)qb, 64);
      r3 = __shfl(r3, (int)qb, 64);
    }
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
#pragma unroll
    for (uint32_t c = 0; c < 4u; ++c)
      if (c < nch) p32_block(acc, w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3], r0, r1, r2, r3, s1, s2, s3);
  }

  const uint32_t h_last = (nb - 1u) / Q;
  if (valid && h == h_last) {
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    p32_block(acc, 0u, 0u, len, 0u, r0, r1, r2, r3, s1, s2, s3);
  }
  uint32_t A[5];
  poly_block_limbs(acc[0], acc[1], acc[2], acc[3], acc[4] << 24, A);
  {
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
    for (int sh = 1; sh < (int)K; sh <<= 1) {
#pragma unroll
      for (int i = 0; i < 5; ++i) A[i] += __shfl_xor(A[i], sh, 64);
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
    } else {
      const uint8_t* tp = src + len;
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
      bad = diff ? 1u : 0u;
    }
  }
  if constexpr (MODE == WG_MODE_OPEN) {
    bad = __shfl(bad, (int)qb, 64);
    if (in_grid && h == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
    if (bad && valid) {
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


// ---------------------------------------------------------------------------
// k_coop — k_lane's contiguous block ranges with cooperative, coalesced payload IO.
// tools/microbench8 measured the chip moving N x 1424-B packets at 1.8 TB/s when
// each lane streams its own 64-B block (k_lane's pattern), 3.6-4.5 TB/s when 8 lanes
// move 128-512 contiguous bytes of one packet per instruction, 4.6-5.0 TB/s for a
// flat stream; the transport kernels were bound by that access pattern, not by VALU.
// Here the 8 lanes of a group (8/K packets) move each of their 8 rows together: a
// row is the next two 64-B blocks (128 contiguous bytes) of one lane's range, so in
// access k the group's lane l moves one 16-B chunk of row 8g+k, and a wave
// instruction covers eight 128-B spans. A per-wave 8 KB LDS exchange (1 KB slice per
// access k, chunks rotated by (k + g) so a lane's own row spreads over the banks)
// turns rows into lanes and back. Stage s = rounds 2s, 2s+1; the next stage's
// chunks are loaded into registers while the current stage computes.
//  * Every global access goes through address-space-1 pointers (global_load/store,
//    never FLAT, whose lgkmcnt coupling would stall each LDS exchange on HBM).
//  * The cooperative loads and stores are unconditional: a chunk that carries no
//    whole-block payload is redirected to P.sink, so the vmcnt wait for the next
//    stage's chunks counts a fixed number of stores and does not drain them.
//  * Partial blocks (packet tails) and packets whose offsets are not 16-B aligned
//    are moved by their own lane (g_load_block / g_store_block).
constexpr uint32_t kCoopSinkBytes = 1u << 20;
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint4 gu4;
#else  // the host pass only parses kernel bodies
typedef uint8_t gu8;
typedef uint32_t gu32;
typedef uint4 gu4;
#endif

__device__ __forceinline__ uint32_t g_ld_bytes(const gu8* p, int n) {
  uint32_t v = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (b < n) v |= (uint32_t)p[b] << (8 * b);
  return v;
}
__device__ __forceinline__ void g_load_block(const gu8* src, uint32_t n, uint32_t w[16]) {
  const bool a4 = (((uintptr_t)src) & 3u) == 0, a16 = (((uintptr_t)src) & 15u) == 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int rem = (int)n - 16 * c;
    if (rem >= 16 && a16) {
      const uint4 x = ((const gu4*)src)[c];
      w[4 * c] = x.x; w[4 * c + 1] = x.y; w[4 * c + 2] = x.z; w[4 * c + 3] = x.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = rem - 4 * k;
        const gu8* q = src + 16 * c + 4 * k;
        w[4 * c + k] = r <= 0 ? 0u : (r >= 4 && a4) ? *(const gu32*)q : g_ld_bytes(q, r);
      }
    }
  }
}
__device__ __forceinline__ void g_store_block(gu8* dst, uint32_t n, const uint32_t w[16]) {
  const bool a4 = (((uintptr_t)dst) & 3u) == 0, a16 = (((uintptr_t)dst) & 15u) == 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int rem = (int)n - 16 * c;
    if (rem >= 16 && a16) {
      ((gu4*)dst)[c] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = rem - 4 * k;
        gu8* q = dst + 16 * c + 4 * k;
        if (r >= 4 && a4) {
          *(gu32*)q = w[4 * c + k];
        } else {
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if (b < r) q[b] = (uint8_t)(w[4 * c + k] >> (8 * b));
        }
      }
    }
  }
}

// V (timing ablations, results wrong): 8 no cooperative global loads/stores, 16 no
// Poly1305 chunk steps, 32 no keystream.
template <int MODE, int K, int V>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_coop(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  static_assert(K == 1 || K == 2 || K == 4, "lanes per packet");
  constexpr uint32_t NP = 8 / K;  // packets per 8-lane group
  __shared__ uint4 xs[8 * 64];
  const uint32_t lane = threadIdx.x, g = lane >> 3, l = lane & 7u;
  const uint64_t gid = (uint64_t)blockIdx.x * 64u + lane;
  const uint32_t pkt = (uint32_t)(gid / K), h = (uint32_t)(gid % K);
  const bool in_grid = gid < (uint64_t)P.n * K;

  uint4 lo = make_uint4(0, 0, 0, 0), hi = make_uint4(0, 0, 0, 0);
  if (in_grid) {
    const gu4* dp = (const gu4*)(P.desc + pkt);
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
  const uint32_t nb = ((len + 63u) >> 6) + 1u;
  const uint32_t Q = (nb + K - 1u) / K;
  const uint32_t b0 = h * Q;
  const uint32_t nr = (valid && b0 < nb) ? min(Q, nb - b0) : 0u;
  const gu8* src = (const gu8*)(P.in + in_off);
  gu8* dst = (gu8*)(P.out + out_off);
  const bool coop = valid && (((uintptr_t)src | (uintptr_t)dst) & 15u) == 0;
  gu8* const sink = (gu8*)P.sink + 16u * ((blockIdx.x & 1023u) * 64u + lane);

  uint4 ka = make_uint4(0, 0, 0, 0), kb = make_uint4(0, 0, 0, 0);
  if (valid) {
    const gu4* kp = (const gu4*)(P.keys + 8u * kslot);
    ka = kp[0];
    kb = kp[1];
  }
  const uint32_t key[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};

  // the group's packets (from their first lanes) and rows (row 8g+k = lane 8g+k)
  uint64_t psrc[NP], pdst[NP];
  uint32_t plen[NP];
  bool pco[NP];
#pragma unroll
  for (uint32_t j = 0; j < NP; ++j) {
    const int sl = (int)(8u * g + j * K);
    psrc[j] = __shfl((uint64_t)(uintptr_t)src, sl, 64);
    pdst[j] = __shfl((uint64_t)(uintptr_t)dst, sl, 64);
    plen[j] = __shfl(len, sl, 64);
    pco[j] = __shfl(coop ? 1u : 0u, sl, 64) != 0u;
  }
  uint32_t rb0[8], rnr[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    rb0[k] = __shfl(b0, (int)(8u * g + k), 64);
    rnr[k] = __shfl(nr, (int)(8u * g + k), 64);
  }
  // byte offset of this lane's chunk of row 8g+k in stage st, or ~0u (not a whole
  // block of a cooperative packet)
  auto coop_off = [&](uint32_t k, uint32_t st) -> uint32_t {
    const uint32_t j = k / K, c = (l - k - g) & 7u;
    const uint32_t trel = 2u * st + (c >> 2);
    const uint32_t blk = rb0[k] + trel;
    const bool ok = pco[j] && trel < rnr[k] && blk >= 1u && 64u * blk <= plen[j];
    return ok ? 64u * (blk - 1u) + 16u * (c & 3u) : ~0u;
  };
  auto coop_load = [&](uint32_t k, uint32_t st) -> uint4 {
    const uint32_t o = coop_off(k, st);
    const gu4* p = (const gu4*)(o != ~0u ? (const gu8*)(uintptr_t)psrc[k / K] + o : (const gu8*)sink);
    uint4 v = *p;  // unconditional: a masked-off chunk reads the sink
    if constexpr ((V & 8) != 0) v = make_uint4(o, k, st, 0);
    return v;
  };

  uint4 pf[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) pf[k] = coop_load(k, 0);

  uint32_t acc[5] = {0, 0, 0, 0, 0};
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, sv0 = 0, sv1 = 0, sv2 = 0, sv3 = 0;
  const uint32_t rot = l + g;

  for (uint32_t st = 0; __any(2u * st < nr); ++st) {
    quad_lds_sync();
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) xs[k * 64u + lane] = pf[k];
    quad_lds_sync();
    uint32_t io[2][16];
#pragma unroll
    for (uint32_t c = 0; c < 8; ++c) {
      const uint4 v = xs[l * 64u + 8u * g + ((c + rot) & 7u)];
      io[c >> 2][4 * (c & 3)] = v.x; io[c >> 2][4 * (c & 3) + 1] = v.y;
      io[c >> 2][4 * (c & 3) + 2] = v.z; io[c >> 2][4 * (c & 3) + 3] = v.w;
    }
    // the next stage's chunks are in flight during this stage's rounds
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) pf[k] = coop_load(k, st + 1u);

#pragma unroll
    for (uint32_t u = 0; u < 2; ++u) {
      const uint32_t t = 2u * st + u;
      const bool act = t < nr;
      const uint32_t b = b0 + t;
      const bool data = act && b > 0;
      const uint32_t off = 64u * (b - 1u);
      const uint32_t nbytes = data ? min(64u, len - off) : 0u;
      const bool cblk = coop && data && nbytes == 64u;
      uint32_t* w = io[u];
      if (data && !cblk) g_load_block(src + off, nbytes, w);
      uint32_t m[16];
      uint32_t nch = 0;
      if (act) {
        uint32_t ks[16];
        if constexpr ((V & 32) != 0) {
#pragma unroll
          for (int i = 0; i < 16; ++i) ks[i] = key[i & 7] + b * (uint32_t)i;
        } else {
          chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
        }
        if (!data) {
          r0 = ks[0] & 0x0fffffffu;
          r1 = ks[1] & 0x0ffffffcu;
          r2 = ks[2] & 0x0ffffffcu;
          r3 = ks[3] & 0x0ffffffcu;
          sv0 = ks[4]; sv1 = ks[5]; sv2 = ks[6]; sv3 = ks[7];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t x = w[i] ^ ks[i];
            m[i] = MODE == WG_MODE_SEAL ? x : w[i];  // MAC input: the ciphertext
            w[i] = x;
          }
          if (!cblk) g_store_block(dst + off, nbytes, w);
          if (nbytes < 64u) mask_block(nbytes, m);
          nch = (V & 16) ? 0u : (nbytes + 15u) >> 4;
        }
      }
      if (t == 0) {  // the packet's r from its first lane (which ran block 0)
        const int sl = (int)(lane - h);
        r0 = __shfl(r0, sl, 64);
        r1 = __shfl(r1, sl, 64);
        r2 = __shfl(r2, sl, 64);
        r3 = __shfl(r3, sl, 64);
      }
      const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
#pragma unroll
      for (uint32_t c = 0; c < 4u; ++c)
        if (c < nch) p32_block(acc, m[4 * c], m[4 * c + 1], m[4 * c + 2], m[4 * c + 3], r0, r1, r2, r3, s1, s2, s3);
    }

    // rows back to chunks: the cooperative stores of this stage's whole blocks
    quad_lds_sync();
#pragma unroll
    for (uint32_t c = 0; c < 8; ++c)
      xs[l * 64u + 8u * g + ((c + rot) & 7u)] =
          make_uint4(io[c >> 2][4 * (c & 3)], io[c >> 2][4 * (c & 3) + 1], io[c >> 2][4 * (c & 3) + 2],
                     io[c >> 2][4 * (c & 3) + 3]);
    quad_lds_sync();
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t o = (V & 8) ? ~0u : coop_off(k, st);
      gu4* p = (gu4*)(o != ~0u ? (gu8*)(uintptr_t)pdst[k / K] + o : sink);
      *p = xs[k * 64u + lane];  // unconditional: a masked-off chunk writes the sink
    }
  }

  const uint32_t h_last = (nb - 1u) / Q;
  if (valid && h == h_last) {
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    p32_block(acc, 0u, 0u, len, 0u, r0, r1, r2, r3, s1, s2, s3);
  }
  uint32_t A[5];
  poly_block_limbs(acc[0], acc[1], acc[2], acc[3], acc[4] << 24, A);
  if constexpr (K > 1) {
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
    for (int sh = 1; sh < K; sh <<= 1) {
#pragma unroll
      for (int i = 0; i < 5; ++i) A[i] += __shfl_xor(A[i], sh, 64);
    }
  }

  uint32_t bad = valid ? 0u : 1u;
  if (h == 0 && valid) {
    uint32_t tag[4];
    poly_finish(A, sv0, sv1, sv2, sv3, tag);
    if constexpr (MODE == WG_MODE_SEAL) {
      g_store_block(dst + len, 16u, tag);
    } else {
      uint32_t got[16];
      g_load_block(src + len, 16u, got);
      const uint32_t diff = (got[0] ^ tag[0]) | (got[1] ^ tag[1]) | (got[2] ^ tag[2]) | (got[3] ^ tag[3]);
      bad = diff ? 1u : 0u;  // all 16 bytes compared, no early exit
    }
  }
  if constexpr (MODE == WG_MODE_OPEN) {
    if constexpr (K > 1) bad = __shfl(bad, (int)(lane - h), 64);
    if (in_grid && h == 0 && P.status) ((gu32*)P.status)[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
    if (bad && valid) {
      uint32_t z[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) z[i] = 0;
      for (uint32_t t = 0; t < nr; ++t) {
        const uint32_t b = b0 + t;
        if (b == 0) continue;
        const uint32_t off = 64u * (b - 1u);
        g_store_block(dst + off, min(64u, len - off), z);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_ws — warp-specialised transport kernel (three LDS rounds in flight): k_lane's contiguous block ranges computed
// by 8 consumer waves out of LDS while 2 producer waves move the payload between HBM
// and LDS, so the ARX rounds and the payload stream run at the same time instead of
// taking turns inside every wave. One workgroup = 10 waves; the
// 512 consumer lanes own 512/K packets (K lanes each). Round t of every consumer lane
// lives in LDS row `lane` of buffer t % 2 (64 B; chunk c at 16 * ((c + row/4) & 3) so
// a wave's row reads spread over the banks). Stage t, between two workgroup barriers:
//   consumers: read their row, keystream + XOR, write the output block back into it,
//              Poly1305 from registers;
//   producers: store stage t-1's output rows (ds_read -> global_store), then load
//              stage t+1's rows into the same buffer with global_load_lds_dwordx4
//              (16 rows of 64 contiguous bytes per wave instruction), then wait.
// Partial chunks (packet tails) and unaligned packets take byte-wise paths in the
// producer. The round count T is uniform over the launch (from max_len), so every
// wave passes the same barriers; this kernel serves uniform batches.
struct WsPkt {  // per-packet record in LDS, written by the packet's first consumer lane
  uint32_t in_lo, in_hi, out_lo, out_hi;
  uint32_t len, flags, q, nb;  // flags: 1 valid, 2 in/out 16-B aligned
};

template <int MODE, int K>
__global__ void __launch_bounds__(640) k_ws(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  static_assert(K == 1 || K == 2 || K == 4, "lanes per packet");
  constexpr uint32_t NC = 512, NPK = NC / K;  // consumer lanes, packets per workgroup
  __shared__ uint4 rows[3][NC * 4];           // 3 x 32 KB: rounds t (consumers), t+1 (landed), t+2 (in flight)
  __shared__ WsPkt tab[NPK];
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wave < 8u;
  const uint32_t nbmax = ((P.max_len + 63u) >> 6) + 1u;
  const uint32_t T = (nbmax + K - 1u) / K;  // rounds, uniform over the launch
  auto rowpos = [](uint32_t row, uint32_t c) -> uint32_t { return 4u * row + ((c + (row >> 2)) & 3u); };

  // ---- consumer state ----
  const uint32_t lane = tid;  // consumer lane = row
  const uint64_t gid = (uint64_t)blockIdx.x * NC + lane;
  const uint32_t pkt = (uint32_t)(gid / K), h = (uint32_t)(gid % K);
  bool valid = false;
  uint32_t len = 0, ctr_lo = 0, ctr_hi = 0, nb = 1, Q = 1, b0 = 0, nr = 0;
  uint64_t in_off = 0, out_off = 0;
  uint32_t key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (consumer) {
    const bool in_grid = gid < (uint64_t)P.n * K;
    uint4 lo = make_uint4(0, 0, 0, 0), hi = make_uint4(0, 0, 0, 0);
    if (in_grid) {
      const uint4* dp = (const uint4*)(P.desc + pkt);
      lo = dp[0];
      hi = dp[1];
    }
    in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
    out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
    ctr_lo = hi.x; ctr_hi = hi.y; len = hi.z;
    const uint32_t kslot = hi.w;
    valid = in_grid && len <= P.max_len && kslot < P.key_slots;
    const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
    valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
    nb = ((len + 63u) >> 6) + 1u;
    Q = (nb + K - 1u) / K;
    b0 = h * Q;
    nr = (valid && b0 < nb) ? min(Q, nb - b0) : 0u;
    if (valid) {
      const uint4* kp = (const uint4*)(P.keys + 8u * kslot);
      const uint4 ka = kp[0], kb = kp[1];
      key[0] = ka.x; key[1] = ka.y; key[2] = ka.z; key[3] = ka.w;
      key[4] = kb.x; key[5] = kb.y; key[6] = kb.z; key[7] = kb.w;
    }
    if (h == 0) {
      const uint64_t ia = (uint64_t)(uintptr_t)(P.in + in_off), oa = (uint64_t)(uintptr_t)(P.out + out_off);
      WsPkt r;
      r.in_lo = (uint32_t)ia; r.in_hi = (uint32_t)(ia >> 32);
      r.out_lo = (uint32_t)oa; r.out_hi = (uint32_t)(oa >> 32);
      r.len = len;
      r.flags = (valid ? 1u : 0u) | ((((ia | oa) & 15u) == 0) ? 2u : 0u);
      r.q = Q; r.nb = nb;
      tab[lane / K] = r;
    }
  }
  __syncthreads();

  // ---- producer helpers: wave w (0, 1) owns rows [256 w, 256 w + 256), 16 rows per access
  const uint32_t pw = wave - 8u, pl = tid & 63u;
  // global byte address of chunk (row, c) of round t, or 0 when the chunk carries no payload;
  // `full` = the whole 16 B lie inside the packet's buffer range and are 16-B aligned
  auto chunk_addr = [&](uint32_t row, uint32_t c, uint32_t t, bool out, uint32_t& nbytes) -> uint64_t {
    const WsPkt r = tab[row / K];
    nbytes = 0;
    if (!(r.flags & 1u)) return 0;
    const uint32_t hh = row % K, rb0 = hh * r.q;
    if (rb0 >= r.nb) return 0;
    const uint32_t rnr = min(r.q, r.nb - rb0);
    const uint32_t b = rb0 + t;
    if (t >= rnr || b == 0) return 0;
    const uint32_t coff = 64u * (b - 1u) + 16u * c;
    if (coff >= r.len) return 0;
    nbytes = min(16u, r.len - coff);
    const uint64_t base = out ? ((uint64_t)r.out_lo | ((uint64_t)r.out_hi << 32))
                              : ((uint64_t)r.in_lo | ((uint64_t)r.in_hi << 32));
    if (!(r.flags & 2u)) nbytes |= 0x100u;  // unaligned packet: byte-wise path
    return base + coff;
  };
  // every producer lane issues exactly 16 LDS-DMA loads per round (a chunk without
  // payload reads the sink), so "round t+1 has landed" is s_waitcnt vmcnt(16) while
  // round t+2 is in flight; chunks the DMA cannot take (unaligned packet, or a tail
  // chunk whose 16-B over-read would leave the input buffer) are patched afterwards
  const uint64_t in_end = (uint64_t)(uintptr_t)P.in + P.in_size;
  const uint8_t* sinkp = P.sink + 16u * pl;
  auto dma_ok = [&](uint64_t a, uint32_t nbytes) { return a != 0 && !(nbytes & 0x100u) && a + 16u <= in_end; };
  auto produce_loads = [&](uint32_t t) {
    uint4* buf = rows[t % 3u];
#pragma unroll 4
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t R = 256u * pw + 16u * i, row = R + (pl >> 2), sl = pl & 3u;
      const uint32_t c = (sl - (row >> 2)) & 3u;
      uint32_t nbytes;
      const uint64_t a = chunk_addr(row, c, t, false, nbytes);
      const void* g = dma_ok(a, nbytes) ? (const void*)(uintptr_t)a : (const void*)sinkp;
      __builtin_amdgcn_global_load_lds(g, (void*)&buf[4u * R], 16, 0, 0);
    }
  };
  auto produce_fixups = [&](uint32_t t) {
    uint4* buf = rows[t % 3u];
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t R = 256u * pw + 16u * i, row = R + (pl >> 2), sl = pl & 3u;
      const uint32_t c = (sl - (row >> 2)) & 3u;
      uint32_t nbytes;
      const uint64_t a = chunk_addr(row, c, t, false, nbytes);
      if (a != 0 && !dma_ok(a, nbytes)) {  // bytes, zero padded
        const gu8* q = (const gu8*)(uintptr_t)a;
        const uint32_t n = nbytes & 0xffu;
        uint32_t w4[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          uint32_t v = 0;
#pragma unroll
          for (uint32_t bb = 0; bb < 4; ++bb)
            if (4u * k + bb < n) v |= (uint32_t)q[4u * k + bb] << (8u * bb);
          w4[k] = v;
        }
        buf[4u * R + pl] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
  };
  auto produce_stores = [&](uint32_t t) {
    const uint4* buf = rows[t % 3u];
#pragma unroll 4
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t R = 256u * pw + 16u * i, row = R + (pl >> 2), sl = pl & 3u;
      const uint32_t c = (sl - (row >> 2)) & 3u;
      uint32_t nbytes;
      const uint64_t a = chunk_addr(row, c, t, true, nbytes);
      if (a != 0) {
        const uint4 v = buf[4u * R + pl];
        if (nbytes == 16u) {
          *(gu4*)(uintptr_t)a = v;
        } else {
          gu8* q = (gu8*)(uintptr_t)a;
          const uint32_t n = nbytes & 0xffu, w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t k = 0; k < 16; ++k)
            if (k < n) q[k] = (uint8_t)(w4[k >> 2] >> (8u * (k & 3u)));
        }
      }
    }
  };

  if (!consumer) {
    produce_loads(0);
    if (T > 1u) {
      produce_loads(1);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // round 0 has landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    produce_fixups(0);
  }
  __syncthreads();

  uint32_t acc[5] = {0, 0, 0, 0, 0};
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, sv0 = 0, sv1 = 0, sv2 = 0, sv3 = 0;
  for (uint32_t t = 0; t < T; ++t) {
    if (consumer) {
      uint4* buf = rows[t % 3u];
      const bool act = t < nr;
      const uint32_t b = b0 + t;
      const bool data = act && b > 0;
      const uint32_t off = 64u * (b - 1u);
      const uint32_t nbytes = data ? min(64u, len - off) : 0u;
      uint32_t w[16];
#pragma unroll
      for (uint32_t c = 0; c < 4; ++c) {
        const uint4 v = buf[rowpos(lane, c)];
        w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
      }
      uint32_t m[16];
      uint32_t nch = 0;
      if (act) {
        uint32_t ks[16];
        chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
        if (!data) {
          r0 = ks[0] & 0x0fffffffu;
          r1 = ks[1] & 0x0ffffffcu;
          r2 = ks[2] & 0x0ffffffcu;
          r3 = ks[3] & 0x0ffffffcu;
          sv0 = ks[4]; sv1 = ks[5]; sv2 = ks[6]; sv3 = ks[7];
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t x = w[i] ^ ks[i];
            m[i] = MODE == WG_MODE_SEAL ? x : w[i];  // MAC input: the ciphertext
            w[i] = x;
          }
#pragma unroll
          for (uint32_t c = 0; c < 4; ++c)
            buf[rowpos(lane, c)] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
          if (nbytes < 64u) mask_block(nbytes, m);
          nch = (nbytes + 15u) >> 4;
        }
      }
      if (K > 1 && t == 0) {
        const int sl = (int)((lane & 63u) - h);
        r0 = __shfl(r0, sl, 64);
        r1 = __shfl(r1, sl, 64);
        r2 = __shfl(r2, sl, 64);
        r3 = __shfl(r3, sl, 64);
      }
      const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
#pragma unroll
      for (uint32_t c = 0; c < 4u; ++c)
        if (c < nch) p32_block(acc, m[4 * c], m[4 * c + 1], m[4 * c + 2], m[4 * c + 3], r0, r1, r2, r3, s1, s2, s3);
    } else {
      if (t >= 1u) produce_stores(t - 1u);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // rows t-1 are read before t+2 refills them
      if (t + 2u < T) {
        produce_loads(t + 2u);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // round t+1 has landed, t+2 in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (t + 1u < T) produce_fixups(t + 1u);
    }
    __syncthreads();
  }
  if (!consumer) {
    if (T >= 1u) produce_stores(T - 1u);
    return;
  }

  // ---- consumers: the length block, the K-lane combine and the tag ----
  const uint32_t h_last = (nb - 1u) / Q;
  if (valid && h == h_last) {
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    p32_block(acc, 0u, 0u, len, 0u, r0, r1, r2, r3, s1, s2, s3);
  }
  uint32_t A[5];
  poly_block_limbs(acc[0], acc[1], acc[2], acc[3], acc[4] << 24, A);
  if constexpr (K > 1) {
    const uint32_t nc = (len + 15u) >> 4;
    uint32_t e = (valid && h < h_last) ? nc + 5u - 4u * (h + 1u) * Q : 0u;
    if (__any(e != 0u)) {
      uint32_t base[5], pwr[5];
      poly_r_limbs(r0, r1, r2, r3, base);
#pragma unroll
      for (int i = 0; i < 5; ++i) pwr[i] = 0;
      bool have = false;
      const bool need = e != 0u;
      while (__any(e != 0u)) {
        if (e & 1u) {
          if (have) {
            mul26(pwr, base);
          } else {
#pragma unroll
            for (int i = 0; i < 5; ++i) pwr[i] = base[i];
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
      if (need) mul26(A, pwr);
    }
#pragma unroll
    for (int sh = 1; sh < K; sh <<= 1) {
#pragma unroll
      for (int i = 0; i < 5; ++i) A[i] += __shfl_xor(A[i], sh, 64);
    }
  }
  const uint8_t* src = P.in + in_off;
  uint8_t* dst = P.out + out_off;
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
    } else {
      const uint8_t* tp = src + len;
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
      bad = diff ? 1u : 0u;
    }
  }
  if constexpr (MODE == WG_MODE_OPEN) {
    if constexpr (K > 1) bad = __shfl(bad, (int)((lane & 63u) - h), 64);
    const bool in_grid = gid < (uint64_t)P.n * K;
    if (in_grid && h == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
  }
  // OPEN with a bad tag: the producers' stores of this lane's rows may still be in
  // flight, so the scrub runs in a second launch (k_ws_scrub) ordered after this one
}

// Zero the plaintext of every packet whose status is BADTAG (k_ws's open leaves it
// to this launch, which the stream orders after the producers' stores).
__global__ void __launch_bounds__(256) k_ws_scrub(StreamParams P) {
  const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t pkt = (uint32_t)(gid >> 4), part = (uint32_t)(gid & 15u);
  if (pkt >= P.n || !P.status || P.status[pkt] != WG_PKT_BADTAG) return;
  const uint4 lo = ((const uint4*)(P.desc + pkt))[0], hi = ((const uint4*)(P.desc + pkt))[1];
  const uint64_t in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32), out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
  const uint32_t len = hi.z;
  const bool valid = len <= P.max_len && hi.w < P.key_slots && in_off <= P.in_size &&
                     (uint64_t)len + 16u <= P.in_size - in_off && out_off <= P.out_size &&
                     (uint64_t)len <= P.out_size - out_off;
  if (!valid) return;
  uint8_t* o = P.out + out_off;
  for (uint32_t i = part; i < len; i += 16u) o[i] = 0;
}

}  // namespace wgk
