// wg_tile.hip — general AEAD / primitive kernel (k_tile) for gfx950: the reference's static
// ChaCha20, Poly1305 and ChaCha20Poly1305 API with explicit nonces, counters and AAD.
//
// One workgroup owns a TILE: a run of whole packets. Two phases per tile:
//
//  1. ChaCha phase — lane <-> 64-byte counter block of some packet (block 0 of
//     each packet is the Poly1305 key block, RFC 8439 2.6 / ChaCha20Poly1305.java:11-14;
//     data block j uses counter j, ChaCha20Poly1305.java:36,55). The lane computes
//     the keystream in registers, XORs its 64 payload bytes, stores them to HBM and
//     leaves the MAC input (the ciphertext) in an LDS image of the tile.
//  2. Poly1305 phase — G lanes per packet evaluate the MAC polynomial over the
//     LDS image with a G-strided Horner rule (multiplier r^G), scale lane j's
//     partial by r^(G-j) and sum over the group with wave shuffles
//     (tag = sum c_i r^(M-i) + s; ChaCha20Poly1305.java:63-93, poly1305-donna-64.h).
//
// Open verifies in the same pass: the plaintext is written in phase 1 and
// zero-filled again after phase 2 when the tag does not match, so the caller
// never observes unauthenticated plaintext (ChaCha20Poly1305.java:40-56
// leaves dst untouched; the host wrappers copy back only on success).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wg_device.h"
#include "wg_kernels.h"

namespace wgk {

using namespace wgd;

// ---------------------------------------------------------------------------
// descriptors
struct Pkt {
  uint64_t in_off, out_off, aad_off;
  uint32_t len, aad_len, key_slot, ctr0, n0, n1, n2;
};

template <bool GENERAL>
__device__ __forceinline__ Pkt load_pkt(const void* d, uint32_t i) {
  Pkt p;
  if constexpr (GENERAL) {
    const wg_aead_desc* a = (const wg_aead_desc*)d + i;
    p.in_off = a->in_off; p.out_off = a->out_off; p.aad_off = a->aad_off;
    p.len = a->len; p.aad_len = a->aad_len; p.key_slot = a->key_slot; p.ctr0 = a->ctr0;
    p.n0 = a->nonce[0]; p.n1 = a->nonce[1]; p.n2 = a->nonce[2];
  } else {
    // transport: nonce = LE64(counter) || 0^4 (SymmetricKeypair.java:52-61)
    const wg_pkt* t = (const wg_pkt*)d + i;
    uint4 lo = *(const uint4*)t;        // in_off, out_off
    uint4 hi = *((const uint4*)t + 1);  // counter, len, key_slot
    p.in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
    p.out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
    p.aad_off = 0; p.aad_len = 0; p.ctr0 = 0;
    p.n0 = hi.x; p.n1 = hi.y; p.n2 = 0;
    p.len = hi.z; p.key_slot = hi.w;
  }
  return p;
}

// blocks a packet occupies in the ChaCha phase
template <int MODE>
__device__ __forceinline__ uint32_t pkt_blocks(uint32_t len) {
  uint32_t nb = (len + 63u) >> 6;
  return (MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN) ? nb + 1u : nb;
}

// ---------------------------------------------------------------------------
// 64-byte block IO. Fast path: whole, 16-byte aligned block -> 4 x dwordx4.
// Partial blocks (packet tails) and unaligned packets go chunk by chunk:
// whole 16-byte chunks still use dwordx4 when aligned, the remainder uses
// dword accesses when 4-byte aligned and byte accesses otherwise.
__device__ __forceinline__ uint32_t ld_bytes(const uint8_t* p, int n) {
  uint32_t v = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (b < n) v |= (uint32_t)p[b] << (8 * b);
  return v;
}

__device__ __forceinline__ void load_block(const uint8_t* src, uint32_t n, uint32_t w[16]) {
  const uintptr_t a = (uintptr_t)src;
  if (n == 64u && (a & 15u) == 0) {
    const uint4* p = (const uint4*)src;
    uint4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
    w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w; w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
    w[8] = x2.x; w[9] = x2.y; w[10] = x2.z; w[11] = x2.w; w[12] = x3.x; w[13] = x3.y; w[14] = x3.z; w[15] = x3.w;
    return;
  }
  const bool a4 = (a & 3u) == 0, a16 = (a & 15u) == 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int rem = (int)n - 16 * c;
    if (rem >= 16 && a16) {
      uint4 x = ((const uint4*)src)[c];
      w[4 * c] = x.x; w[4 * c + 1] = x.y; w[4 * c + 2] = x.z; w[4 * c + 3] = x.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = rem - 4 * k;
        const uint8_t* q = src + 16 * c + 4 * k;
        w[4 * c + k] = r <= 0 ? 0u : (r >= 4 && a4) ? *(const uint32_t*)q : ld_bytes(q, r);
      }
    }
  }
}

__device__ __forceinline__ void st_bytes(uint8_t* p, uint32_t v, int n) {
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (b < n) p[b] = (uint8_t)(v >> (8 * b));
}

__device__ __forceinline__ void store_block(uint8_t* dst, uint32_t n, const uint32_t w[16]) {
  const uintptr_t a = (uintptr_t)dst;
  if (n == 64u && (a & 15u) == 0) {
    uint4* p = (uint4*)dst;
    p[0] = make_uint4(w[0], w[1], w[2], w[3]);
    p[1] = make_uint4(w[4], w[5], w[6], w[7]);
    p[2] = make_uint4(w[8], w[9], w[10], w[11]);
    p[3] = make_uint4(w[12], w[13], w[14], w[15]);
    return;
  }
  const bool a4 = (a & 3u) == 0, a16 = (a & 15u) == 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int rem = (int)n - 16 * c;
    if (rem >= 16 && a16) {
      ((uint4*)dst)[c] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = rem - 4 * k;
        uint8_t* q = dst + 16 * c + 4 * k;
        if (r >= 4 && a4) *(uint32_t*)q = w[4 * c + k];
        else if (r > 0) st_bytes(q, w[4 * c + k], r);
      }
    }
  }
}

// zero bytes >= n of a 64-byte register block (MAC input must be zero padded: pad16)
__device__ __forceinline__ void mask_block(uint32_t n, uint32_t w[16]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int rem = (int)n - 4 * k;
    uint32_t m = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (0xffffffffu >> (32 - 8 * rem)));
    w[k] &= m;
  }
}

__device__ __forceinline__ void lds_store_block(uint8_t* lds, const uint32_t w[16]) {
  uint4* p = (uint4*)lds;
  p[0] = make_uint4(w[0], w[1], w[2], w[3]);
  p[1] = make_uint4(w[4], w[5], w[6], w[7]);
  p[2] = make_uint4(w[8], w[9], w[10], w[11]);
  p[3] = make_uint4(w[12], w[13], w[14], w[15]);
}

__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* p) {
  if ((((uintptr_t)p) & 3u) == 0) return *(const uint32_t*)p;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ void store_u32_any(uint8_t* p, uint32_t v) {
  if ((((uintptr_t)p) & 3u) == 0) { *(uint32_t*)p = v; return; }
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// 16-byte chunk of global memory with the bytes >= n zeroed (AAD blocks)
__device__ __forceinline__ void load_chunk16(const uint8_t* src, uint32_t n, uint32_t w[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if ((uint32_t)(4 * k + b) < n) v |= (uint32_t)src[4 * k + b] << (8 * b);
    w[k] = v;
  }
}

// ---------------------------------------------------------------------------
// LDS tile: per-packet records (128 bytes each, read as 16-byte vectors) then the
// payload image (MAC input, 64-byte granules, zero padded to 16 per packet).
//   rec[q * 8 + 0] = {in_off lo, in_off hi, out_off lo, out_off hi}
//   rec[q * 8 + 1] = {len, valid, first tile block, aad_len}
//   rec[q * 8 + 2] = {aad_off lo, aad_off hi, verdict, image byte offset}
//   rec[q * 8 + 3] = {n0, n1, n2, ctr0}          nonce words, CIPHER start counter
//   rec[q * 8 + 4..5] = key (ChaCha key, or the MAC one-time key)
//   rec[q * 8 + 6..7] = Poly1305 one-time key from block 0 (AEAD)
// blk[q] (u32, mp + 1 entries) duplicates the first-block column for the search.
__device__ __forceinline__ uint4* tile_rec(uint8_t* base) { return (uint4*)base; }
__device__ __forceinline__ uint32_t* tile_blk(uint8_t* base, uint32_t mp) { return (uint32_t*)(base + 128u * mp); }
__device__ __forceinline__ uint8_t* tile_img(uint8_t* base, uint32_t mp) { return base + tile_header_bytes(mp); }

__device__ __forceinline__ void shfl5(const uint32_t v[5], int src, uint32_t o[5]) {
#pragma unroll
  for (int i = 0; i < 5; ++i) o[i] = __shfl(v[i], src, 64);
}

__device__ __forceinline__ void lds_load_chunk(const uint8_t* p, uint32_t w[4]) {
  uint4 v = *(const uint4*)p;
  w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
}

// ---------------------------------------------------------------------------
template <int MODE, bool GENERAL>
__global__ void __launch_bounds__(WG_TPB) k_tile(TileParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  constexpr bool AEAD = (MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN);
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = blockIdx.x;
  uint32_t p0, p1;
  if (P.uniform) {
    p0 = tile * P.ppt;
    if (p0 >= P.n) return;
    p1 = min(P.n, p0 + P.ppt);
  } else {
    if (tile >= *P.ntiles_dev) return;
    p0 = P.tile_start[tile];
    p1 = P.tile_start[tile + 1];
  }
  const uint32_t np = p1 - p0;
  const uint32_t mp = P.max_tile_pkts;
  uint4* rec = tile_rec(lds_raw);
  uint32_t* blk = tile_blk(lds_raw, mp);
  uint8_t* img_base = tile_img(lds_raw, mp);

  // ---- packet records --------------------------------------------------------
  for (uint32_t q = tid; q < np; q += WG_TPB) {
    Pkt pk = load_pkt<GENERAL>(P.desc, p0 + q);
    const uint32_t len = pk.len;
    bool ok = len <= P.max_len && pk.key_slot < P.key_slots;
    if (P.uniform) ok = ok && len == P.max_len;
    const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    const uint64_t out_need = MODE == WG_MODE_MAC ? 16u : (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    ok = ok && pk.in_off <= P.in_size && in_need <= P.in_size - pk.in_off;
    ok = ok && pk.out_off <= P.out_size && out_need <= P.out_size - pk.out_off;
    if (GENERAL && AEAD && pk.aad_len)
      ok = ok && pk.aad_off <= P.aad_size && (uint64_t)pk.aad_len <= P.aad_size - pk.aad_off;
    const uint32_t b0 = P.uniform ? q * P.nb_uniform : P.blk_prefix[p0 + q] - P.blk_prefix[p0];
    blk[q] = b0;
    const uint32_t img_off = 64u * (b0 - (AEAD ? q : 0u));
    uint4* r = rec + 8u * q;
    r[0] = make_uint4((uint32_t)pk.in_off, (uint32_t)(pk.in_off >> 32), (uint32_t)pk.out_off,
                      (uint32_t)(pk.out_off >> 32));
    r[1] = make_uint4(len, ok ? 1u : 0u, b0, pk.aad_len);
    r[2] = make_uint4((uint32_t)pk.aad_off, (uint32_t)(pk.aad_off >> 32), 0u, img_off);
    r[3] = make_uint4(pk.n0, pk.n1, pk.n2, pk.ctr0);
    const uint4* kp = (const uint4*)(P.keys + 8u * (ok ? pk.key_slot : 0u));
    r[4] = kp[0];
    r[5] = kp[1];
  }
  if (tid == 0) blk[np] = P.uniform ? np * P.nb_uniform : P.blk_prefix[p1] - P.blk_prefix[p0];
  __syncthreads();

  // ---- phase 1: ChaCha20 over every counter block of the tile ---------------
  const uint32_t nblk = blk[np];
  for (uint32_t b = tid; b < nblk; b += WG_TPB) {
    uint32_t q;
    if (P.uniform) {
      q = P.nb_uniform == 1u ? b : __umulhi(b, P.nb_magic);
    } else {  // last q with blk[q] <= b
      uint32_t lo = 0, hi = np;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (blk[mid] <= b) lo = mid; else hi = mid;
      }
      q = lo;
    }
    const uint4* r = rec + 8u * q;
    const uint4 r1 = r[1];
    if (!r1.y) continue;
    const uint32_t len = r1.x, j = b - r1.z;
    const uint32_t d = AEAD ? j - 1u : j;  // data block index (AEAD block 0 = Poly1305 key)
    const bool data = !(AEAD && j == 0);
    const uint4 r0 = r[0];
    const uint64_t in_off = (uint64_t)r0.x | ((uint64_t)r0.y << 32);
    const uint64_t out_off = (uint64_t)r0.z | ((uint64_t)r0.w << 32);
    const uint32_t off = 64u * d;
    const uint32_t n = data ? min(64u, len - off) : 0u;
    uint8_t* img = img_base + r[2].w + off;
    uint32_t w[16];
    if (data) load_block(P.in + in_off + off, n, w);  // in flight during the rounds below

    if constexpr (MODE == WG_MODE_MAC) {
      if (n < 64u) mask_block(n, w);
      lds_store_block(img, w);
    } else {
      const uint4 ka = r[4], kb = r[5], nn = r[3];
      const uint32_t key[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
      const uint32_t ctr = (MODE == WG_MODE_CIPHER) ? nn.w + j : j;
      uint32_t ks[16];
      chacha20_block(key, ctr, nn.x, nn.y, nn.z, ks);
      if (!data) {
        uint4* o = (uint4*)(rec + 8u * q + 6);
        o[0] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
        o[1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
        continue;
      }
      if constexpr (MODE == WG_MODE_OPEN) {
        if (n < 64u) mask_block(n, w);
        lds_store_block(img, w);  // MAC over the received ciphertext
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
      store_block(P.out + out_off + off, n, w);
      if constexpr (MODE == WG_MODE_SEAL) {
        if (n < 64u) mask_block(n, w);
        lds_store_block(img, w);  // MAC over the ciphertext just produced
      }
    }
  }
  if constexpr (MODE == WG_MODE_CIPHER) {
    return;
  }
  __syncthreads();

  // ---- phase 2: Poly1305, G lanes per packet --------------------------------
  {
    const uint32_t G = P.poly_g;
    const uint32_t ppw = 64u / G;  // packets per wave
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const uint32_t gq = lane / G, j = lane - gq * G;
    const uint32_t base = gq * G;  // first lane of the group
    const bool lane_used = gq < ppw;
    for (uint32_t qb = wave * ppw; qb < np; qb += (WG_TPB / 64u) * ppw) {
      const uint32_t q = qb + gq;
      const uint32_t qq = (lane_used && q < np) ? q : 0u;
      const uint4* r = rec + 8u * qq;
      const uint4 r1 = r[1];
      const bool act = lane_used && q < np && r1.y;
      const uint4 ka = AEAD ? r[6] : r[4];  // r || s
      const uint4 kb = AEAD ? r[7] : r[5];
      uint32_t rl[5];
      poly_r_limbs(ka.x, ka.y, ka.z, ka.w, rl);
      // powers: lane j of the group ends with r^(j+1) (Hillis-Steele product scan)
      uint32_t x[5] = {rl[0], rl[1], rl[2], rl[3], rl[4]};
      for (uint32_t st = 1; st < G; st <<= 1) {
        uint32_t y[5], ys[5];
        shfl5(x, (int)(lane >= st ? lane - st : lane), y);
        poly_scale5(y, ys);
        if (j >= st) poly_mul(x, y, ys);
      }
      uint32_t R[5], Rs[5];
      shfl5(x, (int)min(base + G - 1u, 63u), R);  // r^G
      poly_scale5(R, Rs);

      uint32_t acc[5] = {0, 0, 0, 0, 0};
      if (act) {
        const uint32_t len = r1.x, alen = r1.w;
        const uint4 r2 = r[2];
        const uint8_t* img = img_base + r2.w;
        const uint32_t na = (alen + 15u) >> 4, nc = (len + 15u) >> 4;
        const uint32_t M = (MODE == WG_MODE_MAC) ? nc : na + nc + 1u;
        const uint32_t K = (M + G - 1u) / G;
        const int D = (int)(K * G - M);
        for (uint32_t k = 0; k < K; ++k) {
          if (k) poly_mul(acc, R, Rs);
          const int t = (int)(j + k * G) - D;
          if (t < 0) continue;
          const uint32_t tt = (uint32_t)t;
          uint32_t w[4];
          uint32_t hib = 1u << 24;
          if constexpr (MODE == WG_MODE_MAC) {
            lds_load_chunk(img + 16u * tt, w);
            const uint32_t rem = len - 16u * tt;
            if (rem < 16u) {  // final partial block: 0x01 pad, no 2^128 bit (poly1305-donna-64.h:162-168)
              hib = 0;
              const uint32_t sh = 8u * (rem & 3u), wi = rem >> 2;
              w[0] |= (wi == 0) ? (1u << sh) : 0u;
              w[1] |= (wi == 1) ? (1u << sh) : 0u;
              w[2] |= (wi == 2) ? (1u << sh) : 0u;
              w[3] |= (wi == 3) ? (1u << sh) : 0u;
            }
          } else if (GENERAL && tt < na) {
            const uint32_t o = 16u * tt;
            const uint64_t aad_off = (uint64_t)r2.x | ((uint64_t)r2.y << 32);
            load_chunk16(P.aad + aad_off + o, min(16u, alen - o), w);
          } else if (tt < na + nc) {
            lds_load_chunk(img + 16u * (tt - na), w);
          } else {  // le64(aad_len) || le64(ct_len) (ChaCha20Poly1305.java:88-90)
            w[0] = alen; w[1] = 0; w[2] = len; w[3] = 0;
          }
          uint32_t c[5];
          poly_block_limbs(w[0], w[1], w[2], w[3], hib, c);
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[i] += c[i];
        }
      }
      // scale lane j's partial by r^(G-j) (lane G-1-j holds it after the scan)
      {
        uint32_t W[5], Ws[5];
        shfl5(x, (int)min(base + G - 1u - j, 63u), W);
        poly_scale5(W, Ws);
        if (act) poly_mul(acc, W, Ws);
      }
      // group sum into lane j == 0
      for (uint32_t st = 1; st < G; st <<= 1) {
        uint32_t y[5];
        shfl5(acc, (int)(lane + st < 64u ? lane + st : lane), y);
        if (j + st < G) {
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[i] += y[i];
        }
      }
      if (act && j == 0) {
        uint32_t tag[4];
        poly_finish(acc, kb.x, kb.y, kb.z, kb.w, tag);
        const uint4 r0 = r[0];
        const uint64_t in_off = (uint64_t)r0.x | ((uint64_t)r0.y << 32);
        const uint64_t out_off = (uint64_t)r0.z | ((uint64_t)r0.w << 32);
        const uint32_t len = r1.x;
        if constexpr (MODE == WG_MODE_SEAL || MODE == WG_MODE_MAC) {
          uint8_t* tp = P.out + out_off + (MODE == WG_MODE_SEAL ? len : 0u);
          if ((((uintptr_t)tp) & 15u) == 0) {
            *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
          }
        } else {  // OPEN: compare all 16 bytes, no early exit
          const uint8_t* tp = P.in + in_off + len;
          uint32_t diff = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
          ((uint32_t*)(rec + 8u * q + 2))[2] = diff ? 1u : 0u;
        }
      }
    }
  }
  if constexpr (MODE == WG_MODE_OPEN) {
    __syncthreads();
    for (uint32_t q = tid; q < np; q += WG_TPB) {
      const uint4 r1 = rec[8u * q + 1];
      const uint32_t bad = r1.y ? ((const uint32_t*)(rec + 8u * q + 2))[2] : 1u;
      if (P.status) P.status[p0 + q] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
      if (bad && r1.y) ((uint32_t*)(rec + 8u * q + 2))[2] = 2u;  // needs scrubbing
    }
    __syncthreads();
    for (uint32_t q = 0; q < np; ++q) {
      if (((const uint32_t*)(rec + 8u * q + 2))[2] != 2u) continue;
      const uint4 r0 = rec[8u * q];
      uint8_t* o = P.out + ((uint64_t)r0.z | ((uint64_t)r0.w << 32));
      const uint32_t len = rec[8u * q + 1].x;
      for (uint32_t i = tid; i < len; i += WG_TPB) o[i] = 0;  // scrub unauthenticated plaintext
    }
  }
}

// ---------------------------------------------------------------------------
// non-uniform plan: per-packet block counts -> (external scan) -> tile starts
template <int MODE, bool GENERAL>
__global__ void k_plan_count(const void* desc, uint32_t n, uint32_t max_len, uint32_t* nb) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t len = GENERAL ? ((const wg_aead_desc*)desc)[i].len : ((const wg_pkt*)desc)[i].len;
    nb[i] = len <= max_len ? pkt_blocks<MODE>(len) : pkt_blocks<MODE>(0);
  }
  if (i == n) nb[n] = 0;
}

// Tile t owns the packets whose first block lies in [t*C, (t+1)*C) of the
// batch-wide block sequence ("start-owned"): tiles hold < C + max_nb blocks
// and, as a packet owns >= 1 block, at most C packets.
__global__ void k_plan_tiles(const uint32_t* prefix, uint32_t n, uint32_t C, uint32_t* tile_start, uint32_t* ntiles,
                             uint32_t max_tiles) {
  const uint32_t total = prefix[n];
  const uint32_t T = (total + C - 1u) / C;
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) *ntiles = T;
  if (t > T || t > max_tiles) return;
  // first packet with prefix >= t*C
  const uint64_t key = (uint64_t)t * C;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)prefix[mid] < key) lo = mid + 1; else hi = mid;
  }
  tile_start[t] = (t == T) ? n : lo;
}

template __global__ void k_tile<WG_MODE_SEAL, false>(TileParams);
template __global__ void k_tile<WG_MODE_OPEN, false>(TileParams);
template __global__ void k_tile<WG_MODE_SEAL, true>(TileParams);
template __global__ void k_tile<WG_MODE_OPEN, true>(TileParams);
template __global__ void k_tile<WG_MODE_CIPHER, true>(TileParams);
template __global__ void k_tile<WG_MODE_MAC, true>(TileParams);
template __global__ void k_plan_count<WG_MODE_SEAL, false>(const void*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_plan_count<WG_MODE_OPEN, false>(const void*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_plan_count<WG_MODE_SEAL, true>(const void*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_plan_count<WG_MODE_OPEN, true>(const void*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_plan_count<WG_MODE_CIPHER, true>(const void*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_plan_count<WG_MODE_MAC, true>(const void*, uint32_t, uint32_t, uint32_t*);

}  // namespace wgk
