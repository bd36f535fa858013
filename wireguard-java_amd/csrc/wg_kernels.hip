// wg_kernels.hip — batched transport AEAD kernels for gfx950 (MI355X).
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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wg_device.h"
#include "wg_kernels.h"

namespace wgk {

using namespace wgd;

// In-kernel phase stamps, compiled only into the diagnostic library
// (make diag -> libwgaead_diag.so); the product build has none.
#ifdef WG_DIAG
#define WG_STAMP(i)                                                                      \
  do {                                                                                   \
    if (P.stamps && threadIdx.x == 0) {                                                  \
      uint64_t t_;                                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
      P.stamps[(size_t)blockIdx.x * 8 + (i)] = t_;                                       \
    }                                                                                    \
  } while (0)
#else
#define WG_STAMP(i) do {} while (0)
#endif

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
  WG_STAMP(0);
#ifdef WG_DIAG
  if (P.stamps && tid == 0) {
    P.stamps[(size_t)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memrealtime();
    P.stamps[(size_t)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
    P.stamps[(size_t)blockIdx.x * 8 + 7] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
  }
#endif

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
  WG_STAMP(1);

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
    WG_STAMP(2);
    return;
  }
  __syncthreads();
  WG_STAMP(2);

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

  WG_STAMP(3);
#ifdef WG_DIAG
  if (P.stamps && tid == 0) P.stamps[(size_t)blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memrealtime();
#endif
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

// ---------------------------------------------------------------------------
// k_stream — transport seal/open, one wave per workgroup, no barriers between waves.
//
// The wave is 8 SLOTS of 8 lanes. A slot streams one packet at a time, 512 bytes
// (8 ChaCha20 counter blocks) per ROUND:
//   1. lane j of the slot computes counter block 8*round + j (block 0 = the
//      Poly1305 key block, ChaCha20Poly1305.java:11-14; block b >= 1 = payload
//      bytes 64(b-1).., ChaCha20Poly1305.java:36) with its 64 payload bytes
//      prefetched before the rounds, XORs, stores, and leaves the MAC input
//      (ciphertext) of the round in a 4 KB LDS image;
//   2. the same 8 lanes advance an 8-strided Horner evaluation of the MAC
//      polynomial over the round's 16-byte chunks: lane j owns the message
//      positions congruent to j mod 8 (leading zero padding D = 8K - M aligns the
//      last position to lane 7) and multiplies by R = r^8 per position.
// On the packet's last round each lane scales its partial by r^(8-j), the slot
// sums its 8 partials with shuffles and lane 0 finishes the tag
// (ChaCha20Poly1305.java:63-93). Finished slots take the wave's next packet, so
// mixed lengths keep every slot busy. Register/LDS budget: ~5 KB LDS per wave,
// so a CU holds up to 32 waves.
constexpr uint32_t SLOT_LANES = 8;

struct StreamParams {
  const wg_pkt* desc;
  uint32_t n;
  uint32_t ppw;  // packets per wave (consecutive descriptors)
  uint32_t max_len;
  uint32_t key_slots;
  const uint8_t* in;
  uint64_t in_size;
  uint8_t* out;
  uint64_t out_size;
  const uint32_t* keys;
  uint32_t* status;
  uint64_t* stamps;  // WG_DIAG builds only: 8 x u64 per wave
  uint8_t* sink;     // k_coop: 1 MiB device scratch that absorbs the masked-off cooperative accesses
};

// 16-B transport header {u8 4, u8 0[3], u32 receiver_index, u64 counter}, little-endian
// (TransportPacket.java:18-35), written with 4-B or 1-B vector stores by alignment.
__device__ inline void put_header(uint8_t* h, uint32_t rx, uint64_t ctr) {
  const uint32_t w[4] = {4u, rx, (uint32_t)ctr, (uint32_t)(ctr >> 32)};
  if ((((uintptr_t)h) & 3u) == 0) {
    uint32_t* h32 = (uint32_t*)h;
#pragma unroll
    for (int k = 0; k < 4; ++k) h32[k] = w[k];
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) h[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  }
}

// Per-wave phase accounting for k_stream (diagnostic library only): cycles spent
// starting packets, in ChaCha, in Poly1305 and finishing, plus realtime start/end.
#ifdef WG_DIAG
#define WG_PH_DECL uint64_t ph_t = 0, ph_acc[4] = {0, 0, 0, 0}; const uint64_t ph_r0 = __builtin_amdgcn_s_memrealtime();
#define WG_PH_MARK() do { asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ph_t)::"memory"); } while (0)
#define WG_PH_ADD(k) do { uint64_t n_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(n_)::"memory"); ph_acc[k] += n_ - ph_t; ph_t = n_; } while (0)
#define WG_PH_STORE()                                                                             \
  do {                                                                                            \
    if (P.stamps && threadIdx.x == 0) {                                                           \
      uint64_t* o_ = P.stamps + (size_t)blockIdx.x * 8;                                           \
      o_[0] = ph_r0; o_[1] = __builtin_amdgcn_s_memrealtime();                                    \
      o_[2] = ph_acc[0]; o_[3] = ph_acc[1]; o_[4] = ph_acc[2]; o_[5] = ph_acc[3];                 \
      uint32_t hw_, xcc_;                                                                         \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                           \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                         \
      o_[6] = hw_; o_[7] = xcc_;                                                                  \
    }                                                                                             \
  } while (0)
#define WG_PH_STORE_WAVE(idx)                                                                     \
  do {                                                                                            \
    if (P.stamps && (threadIdx.x & 63u) == 0) {                                                   \
      uint64_t* o_ = P.stamps + (size_t)(idx) * 8;                                                \
      o_[0] = ph_r0; o_[1] = __builtin_amdgcn_s_memrealtime();                                    \
      o_[2] = ph_acc[0]; o_[3] = ph_acc[1]; o_[4] = ph_acc[2]; o_[5] = ph_acc[3];                 \
      uint32_t hw_, xcc_;                                                                         \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                           \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                         \
      o_[6] = hw_; o_[7] = xcc_;                                                                  \
    }                                                                                             \
  } while (0)
#else
#define WG_PH_STORE_WAVE(idx) do {} while (0)
#define WG_PH_DECL
#define WG_PH_MARK() do {} while (0)
#define WG_PH_ADD(k) do {} while (0)
#define WG_PH_STORE() do {} while (0)
#endif

// Progress-based wave priority: a wave drops its issue priority as it completes
// rounds (3, 2, 1, then 0), so the SIMD's oldest-first arbitration no longer lets
// one wave run ahead while the others idle at the end of a launch.
__device__ __forceinline__ void progress_prio(uint32_t done_rounds) {
  if (done_rounds == 0) __builtin_amdgcn_s_setprio(3);
  else if (done_rounds == 1) __builtin_amdgcn_s_setprio(2);
  else if (done_rounds == 2) __builtin_amdgcn_s_setprio(1);
  else if (done_rounds == 3) __builtin_amdgcn_s_setprio(0);
}

// V (variant bits, for A/B builds; bits 4/5 are timing ablations that skip Poly1305 / the keystream): bit3 ILP form of the Poly1305 multiply, bit0 prefetch payload before the rounds,
// bit1 re-read the key from LDS for the feed-forward, bit2 cap VGPRs for 8 waves/SIMD
template <int MODE, int V>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((V & 4) ? 8 : 1))) k_stream(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  __shared__ uint4 img[8 * 8 * 4];  // [slot][lane][4 chunks]: the round's MAC input
  __shared__ uint4 skey[8 * 2];     // per-slot ChaCha key
  __shared__ uint4 sotk[8 * 2];     // per-slot Poly1305 one-time key (r || s)
  __shared__ uint32_t spow[8 * 10]; // per-slot R = r^8 limbs and 5R (limbs 1..4)
  __shared__ uint32_t lpow[64 * 5]; // per-lane W = r^(8-j) limbs
  const uint32_t lane = threadIdx.x, s = lane >> 3, j = lane & 7u;
  const uint32_t sbase = lane & ~7u;
  const uint32_t w0 = blockIdx.x * P.ppw, w1 = min(P.n, w0 + P.ppw);
  uint32_t next = w0 + SLOT_LANES;  // wave-uniform
  uint32_t pkt = w0 + s;
  bool have = pkt < w1;
  uint32_t round = 0;
  // packet state (identical in the 8 lanes of a slot)
  uint64_t in_off = 0, out_off = 0;
  uint32_t len = 0, ctr_lo = 0, ctr_hi = 0, nb = 0, nc = 0, D = 0;
  bool valid = false;
  uint32_t acc[5];
  WG_PH_DECL
  uint32_t wave_rounds = 0;  // wave-uniform

  while (__any(have)) {
    if constexpr ((V & 64) != 0) progress_prio(wave_rounds++);
    WG_PH_MARK();
    if (have && round == 0) {  // start a packet: descriptor, bounds, key
      const uint4* dp = (const uint4*)(P.desc + pkt);
      const uint4 lo = dp[0], hi = dp[1];
      in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
      out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
      ctr_lo = hi.x; ctr_hi = hi.y; len = hi.z;
      const uint32_t ks_ = hi.w;
      valid = len <= P.max_len && ks_ < P.key_slots;
      const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
      const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
      valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
      valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
      nb = ((len + 63u) >> 6) + 1u;
      nc = (len + 15u) >> 4;
      const uint32_t M = nc + 1u, K = (M + 7u) >> 3;
      D = 8u * K - M;
      acc[0] = acc[1] = acc[2] = acc[3] = acc[4] = 0;
      if (j == 0 && valid) {
        const uint4* kp = (const uint4*)(P.keys + 8u * ks_);
        skey[2 * s] = kp[0];
        skey[2 * s + 1] = kp[1];
      }
    }
    __syncthreads();  // one wave per workgroup: orders the slot key writes
    WG_PH_ADD(0);

    // ---- ChaCha20: block b of the slot's packet ------------------------------------
    const uint32_t b = 8u * round + j;
    const bool act = have && valid && b < nb;
    const bool data = act && b > 0;
    const uint32_t off = 64u * (b - 1u);
    const uint32_t nbytes = data ? min(64u, len - off) : 0u;
    uint32_t w[16];
    if ((V & 1) && data) load_block(P.in + in_off + off, nbytes, w);  // in flight during the rounds
    if (act) {
      uint32_t ks[16];
      if constexpr (V & 32) {  // ablation: no keystream
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] = ctr_lo + b * i;
      } else if constexpr (V & 2) {
        chacha20_block_lds(&skey[2 * s], b, ctr_lo, ctr_hi, 0u, ks);
      } else {
        const uint4 ka = skey[2 * s], kb = skey[2 * s + 1];
        const uint32_t key[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
        chacha20_block(key, b, ctr_lo, ctr_hi, 0u, ks);
      }
      if (!(V & 1) && data) load_block(P.in + in_off + off, nbytes, w);
      if (!data) {
        sotk[2 * s] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
        sotk[2 * s + 1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
      } else {
        if constexpr (MODE == WG_MODE_OPEN) {
          if (nbytes < 64u) mask_block(nbytes, w);
          lds_store_block((uint8_t*)&img[4 * lane], w);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
        store_block(P.out + out_off + off, nbytes, w);
        if constexpr (MODE == WG_MODE_SEAL) {
          if (nbytes < 64u) mask_block(nbytes, w);
          lds_store_block((uint8_t*)&img[4 * lane], w);
        }
      }
    }
    __syncthreads();
    WG_PH_ADD(1);

    // ---- Poly1305 ------------------------------------------------------------------
    if (!(V & 16) && have && valid) {
      if (round == 0) {  // r and its powers: lane j gets r^(j+1); R = r^8, W = r^(8-j)
        const uint4 o = sotk[2 * s];
        uint32_t x[5];
        poly_r_limbs(o.x, o.y, o.z, o.w, x);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5], ys[5];
          shfl5(x, (int)(j >= st ? lane - st : lane), y);
          poly_scale5(y, ys);
          if (j >= st) { if constexpr (V & 8) poly_mul_ilp(x, y, ys); else poly_mul(x, y, ys); }
        }
        uint32_t R[5], W[5];
        shfl5(x, (int)(sbase + 7u), R);
        shfl5(x, (int)(sbase + 7u - j), W);
#pragma unroll
        for (int i = 0; i < 5; ++i) lpow[5 * lane + i] = W[i];
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < 5; ++i) spow[10 * s + i] = R[i];
#pragma unroll
          for (int i = 1; i < 5; ++i) spow[10 * s + 5 + i] = R[i] * 5u;
        }
      }
      uint32_t R[5], Rs[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) R[i] = spow[10 * s + i];
      Rs[0] = 0;
#pragma unroll
      for (int i = 1; i < 5; ++i) Rs[i] = spow[10 * s + 5 + i];
      // this round's message chunks: data blocks 8r..8r+7 -> chunks [4(8r-1), 4(8r+7)) of [0, nc)
      const uint32_t blo = max(8u * round, 1u);
      const uint32_t c_lo = 4u * (blo - 1u);
      const bool last = 8u * (round + 1u) >= nb;
      const uint32_t c_end = last ? nc + 1u : min(nc, 4u * (8u * round + 7u));
      // first chunk c >= c_lo with (c + D) % 8 == j
      uint32_t c = c_lo + ((j - ((c_lo + D) & 7u)) & 7u);
      for (; c < c_end; c += 8u) {
        if constexpr (V & 8) poly_mul_ilp(acc, R, Rs); else poly_mul(acc, R, Rs);
        uint32_t m0, m1, m2, m3;
        if (c < nc) {
          const uint32_t blk_lane = (c >> 2) + 1u - 8u * round;  // lane of the slot holding it
          const uint4 v = img[4u * (sbase + blk_lane) + (c & 3u)];
          m0 = v.x; m1 = v.y; m2 = v.z; m3 = v.w;
        } else {  // le64(0) || le64(len): no AAD on the transport path (ChaCha20Poly1305.java:88-90)
          m0 = 0; m1 = 0; m2 = len; m3 = 0;
        }
        uint32_t cl[5];
        poly_block_limbs(m0, m1, m2, m3, 1u << 24, cl);
#pragma unroll
        for (int i = 0; i < 5; ++i) acc[i] += cl[i];
      }
    }

    WG_PH_ADD(2);
    // ---- finish packets whose last round this was ------------------------------------
    const bool done = have && (!valid || 8u * (round + 1u) >= nb);
    if (done) {
      if (valid) {
        uint32_t W[5], Ws[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) W[i] = lpow[5 * lane + i];
        poly_scale5(W, Ws);
        if constexpr (V & 8) poly_mul_ilp(acc, W, Ws); else poly_mul(acc, W, Ws);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5];
          shfl5(acc, (int)(j + st < 8u ? lane + st : lane), y);
          if (j + st < 8u) {
#pragma unroll
            for (int i = 0; i < 5; ++i) acc[i] += y[i];
          }
        }
      }
      uint32_t bad = valid ? 0u : 1u;
      if (j == 0 && valid) {
        const uint4 sv = sotk[2 * s + 1];
        uint32_t tag[4];
        poly_finish(acc, sv.x, sv.y, sv.z, sv.w, tag);
        if constexpr (MODE == WG_MODE_SEAL) {
          uint8_t* tp = P.out + out_off + len;
          if ((((uintptr_t)tp) & 15u) == 0) {
            *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
          }
        } else {  // all 16 bytes compared, no early exit
          const uint8_t* tp = P.in + in_off + len;
          uint32_t diff = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
          bad = diff ? 1u : 0u;
        }
      }
      if constexpr (MODE == WG_MODE_OPEN) {
        bad = __shfl(bad, (int)sbase, 64);
        if (j == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
        if (bad && valid) {  // scrub the unauthenticated plaintext written this call
          uint8_t* o = P.out + out_off;
          for (uint32_t i = j; i < len; i += 8u) o[i] = 0;
        }
      }
    }
    // hand the wave's next packets to the slots that finished (ballot rank)
    const unsigned long long fin = __ballot(done && j == 0);
    if (done) {
      const uint32_t rank = (uint32_t)__popcll(fin & ((1ull << sbase) - 1ull));
      pkt = next + rank;
      have = pkt < w1;
      round = 0;
    } else if (have) {
      ++round;
    }
    next += (uint32_t)__popcll(fin);
    WG_PH_ADD(3);
  }
  WG_PH_STORE();
}

// ---------------------------------------------------------------------------
// k_pipe — k_stream's slot/round structure, software-pipelined: while a wave
// computes round r out of one LDS stage buffer, round r+1's payload streams into
// the other with coalesced global_load_lds_dwordx4 (1 KB per wave instruction, no
// VGPRs), so every wave overlaps its own HBM traffic with its own ChaCha20 and
// Poly1305 work instead of all waves alternating memory and compute in lockstep.
// Slot s of wave w processes packets w*ppw + s, +8, +16, ... (static successor,
// so the successor's descriptor and key are fetched a packet ahead).
// Stage layout: [buffer][slot][32 x 16-byte chunks]; chunk c of round r of a
// packet holds payload bytes 512r - 64 + 16c (round 0's chunks 0..3 are the key
// block's place). Only whole 16-byte chunks of 16-byte aligned packets are
// staged; a packet tail or an unaligned packet is read by its ChaCha lane.
// The same buffer then holds the round's MAC input (ciphertext) for Poly1305.
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int MODE, int V>
__global__ void __launch_bounds__(64) k_pipe(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  __shared__ uint4 stage[2 * 256];  // 2 x 4 KB
  __shared__ uint4 plan[8];         // per slot: {in_off lo, in_off hi, window start (signed), window end}
  __shared__ uint4 skey[8 * 2];
  __shared__ uint4 sotk[8 * 2];
  __shared__ uint32_t spow[8 * 10];
  __shared__ uint32_t lpow[64 * 5];
  const uint32_t lane = threadIdx.x, s = lane >> 3, j = lane & 7u;
  const uint32_t sbase = lane & ~7u;
  const uint32_t w0 = blockIdx.x * P.ppw, w1 = min(P.n, w0 + P.ppw);

  // current packet of the slot (identical in its 8 lanes)
  uint32_t pkt = w0 + s;
  bool have = pkt < w1;
  uint64_t in_off = 0, out_off = 0;
  uint32_t len = 0, ctr_lo = 0, ctr_hi = 0, nb = 0, nc = 0, D = 0, round = 0;
  bool valid = false, staged = false;
  uint32_t acc[5] = {0, 0, 0, 0, 0};
  // successor descriptor (packet pkt + 8), fetched a packet ahead
  uint4 sd_lo = make_uint4(0, 0, 0, 0), sd_hi = make_uint4(0, 0, 0, 0);
  uint4 nk_a = make_uint4(0, 0, 0, 0), nk_b = make_uint4(0, 0, 0, 0);

  auto decode = [&](uint4 lo, uint4 hi) {
    in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
    out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
    ctr_lo = hi.x; ctr_hi = hi.y; len = hi.z;
    valid = len <= P.max_len && hi.w < P.key_slots;
    const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
    valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
    staged = valid && ((((uintptr_t)P.in + in_off) & 15u) == 0);
    nb = ((len + 63u) >> 6) + 1u;
    nc = (len + 15u) >> 4;
    const uint32_t M = nc + 1u, K = (M + 7u) >> 3;
    D = 8u * K - M;
    round = 0;
    acc[0] = acc[1] = acc[2] = acc[3] = acc[4] = 0;
  };
  auto write_plan = [&](bool any, uint32_t r) {
    if (j == 0) {
      const uint32_t full_end = staged && any ? (len & ~15u) : 0u;
      plan[s] = make_uint4((uint32_t)in_off, (uint32_t)(in_off >> 32), 512u * r - 64u, full_end);
    }
  };
  auto issue_stage = [&](uint32_t buf) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t t = 2u * k + (lane >> 5), c = lane & 31u;
      const uint4 pl = plan[t];
      const int64_t o = (int64_t)(int32_t)pl.z + 16 * (int64_t)c;
      if (o >= 0 && o + 16 <= (int64_t)pl.w) {
        const uint64_t base = (uint64_t)pl.x | ((uint64_t)pl.y << 32);
        __builtin_amdgcn_global_load_lds((const void*)(P.in + base + (uint64_t)o), (void*)&stage[buf * 256u + 64u * k],
                                         16, 0, 0);
      }
    }
  };

  // ---- prologue: first packet of every slot, its key, its successor's descriptor
  if (have) {
    const uint4* dp = (const uint4*)(P.desc + pkt);
    decode(dp[0], dp[1]);
    if (j == 0 && valid) {
      const uint4* kp = (const uint4*)(P.keys + 8u * ((const uint4*)(P.desc + pkt))[1].w);
      skey[2 * s] = kp[0];
      skey[2 * s + 1] = kp[1];
    }
    if (pkt + 8u < w1) {
      const uint4* sp = (const uint4*)(P.desc + pkt + 8u);
      sd_lo = sp[0];
      sd_hi = sp[1];
    }
  }
  write_plan(have, 0);
  lds_fence();
  issue_stage(0);
  uint32_t buf = 0;

  while (__any(have)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this round's stage, keys, successor descriptors
    const uint32_t nrounds = (nb + 7u) >> 3;
    const bool last = have && (!valid || round + 1u >= nrounds);
    const bool has_succ = pkt + 8u < w1;
    // key of the successor: fetched now, published to LDS when it becomes current
    if (have && last && has_succ && j == 0) {
      const uint32_t ks_ = sd_hi.w < P.key_slots ? sd_hi.w : 0u;
      const uint4* kp = (const uint4*)(P.keys + 8u * ks_);
      nk_a = kp[0];
      nk_b = kp[1];
    }
    // ---- plan and issue the next round's stage ---------------------------------
    {
      // decode the successor into temporaries only for planning
      uint64_t t_in = in_off;
      uint32_t t_len = len, r_next = round + 1u;
      bool t_any = have && !last && valid;
      bool t_staged = staged;
      if (have && last && has_succ) {
        t_in = (uint64_t)sd_lo.x | ((uint64_t)sd_lo.y << 32);
        t_len = sd_hi.z;
        r_next = 0;
        t_any = t_len <= P.max_len && t_in <= P.in_size && (uint64_t)t_len <= P.in_size - t_in;
        t_staged = ((((uintptr_t)P.in + t_in) & 15u) == 0);
      }
      if (j == 0) {
        const uint32_t full_end = (t_any && t_staged) ? (t_len & ~15u) : 0u;
        plan[s] = make_uint4((uint32_t)t_in, (uint32_t)(t_in >> 32), 512u * r_next - 64u, full_end);
      }
      lds_fence();
      issue_stage(buf ^ 1u);
    }

    // ---- ChaCha20: block b of the slot's packet ------------------------------------
    uint4* st = &stage[buf * 256u + 32u * s];  // this slot's 512 bytes
    const uint32_t b = 8u * round + j;
    const bool act = have && valid && b < nb;
    const bool data = act && b > 0;
    const uint32_t off = 64u * (b - 1u);
    const uint32_t nbytes = data ? min(64u, len - off) : 0u;
    if (act) {
      uint32_t ks[16];
      chacha20_block_lds(&skey[2 * s], b, ctr_lo, ctr_hi, 0u, ks);
      if (!data) {
        sotk[2 * s] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
        sotk[2 * s + 1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
      } else {
        uint32_t w[16];
        if (staged) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rem = (int)nbytes - 16 * i;
            if (rem >= 16) {
              const uint4 v = st[4u * j + i];
              w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
            } else {
              uint32_t t4[4];
              load_chunk16(P.in + in_off + off + 16u * i, rem > 0 ? (uint32_t)rem : 0u, t4);
              w[4 * i] = t4[0]; w[4 * i + 1] = t4[1]; w[4 * i + 2] = t4[2]; w[4 * i + 3] = t4[3];
            }
          }
        } else {
          load_block(P.in + in_off + off, nbytes, w);
          if (nbytes < 64u) mask_block(nbytes, w);
        }
        if constexpr (MODE == WG_MODE_OPEN) {
          if (!staged || nbytes < 64u) lds_store_block((uint8_t*)&st[4u * j], w);  // MAC input, zero padded
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
        store_block(P.out + out_off + off, nbytes, w);
        if constexpr (MODE == WG_MODE_SEAL) {
          if (nbytes < 64u) mask_block(nbytes, w);
          lds_store_block((uint8_t*)&st[4u * j], w);  // MAC over the ciphertext just produced
        }
      }
    }
    lds_fence();

    // ---- Poly1305 over this round's chunks -----------------------------------------------
    if (have && valid) {
      if (round == 0) {  // r and its powers: lane j gets r^(j+1); R = r^8, W = r^(8-j)
        const uint4 o = sotk[2 * s];
        uint32_t x[5];
        poly_r_limbs(o.x, o.y, o.z, o.w, x);
#pragma unroll
        for (uint32_t stp = 1; stp < 8u; stp <<= 1) {
          uint32_t y[5], ys[5];
          shfl5(x, (int)(j >= stp ? lane - stp : lane), y);
          poly_scale5(y, ys);
          if (j >= stp) poly_mul(x, y, ys);
        }
        uint32_t R[5], W[5];
        shfl5(x, (int)(sbase + 7u), R);
        shfl5(x, (int)(sbase + 7u - j), W);
#pragma unroll
        for (int i = 0; i < 5; ++i) lpow[5 * lane + i] = W[i];
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < 5; ++i) spow[10 * s + i] = R[i];
#pragma unroll
          for (int i = 1; i < 5; ++i) spow[10 * s + 5 + i] = R[i] * 5u;
        }
        lds_fence();
      }
      uint32_t R[5], Rs[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) R[i] = spow[10 * s + i];
      Rs[0] = 0;
#pragma unroll
      for (int i = 1; i < 5; ++i) Rs[i] = spow[10 * s + 5 + i];
      const uint32_t blo = max(8u * round, 1u);
      const uint32_t c_lo = 4u * (blo - 1u);
      const bool lastr = 8u * (round + 1u) >= nb;
      const uint32_t c_end = lastr ? nc + 1u : min(nc, 4u * (8u * round + 7u));
      uint32_t c = c_lo + ((j - ((c_lo + D) & 7u)) & 7u);
      for (; c < c_end; c += 8u) {
        poly_mul(acc, R, Rs);
        uint32_t m0, m1, m2, m3;
        if (c < nc) {
          const uint4 v = st[c + 4u - 32u * round];
          m0 = v.x; m1 = v.y; m2 = v.z; m3 = v.w;
        } else {  // le64(0) || le64(len) (ChaCha20Poly1305.java:88-90)
          m0 = 0; m1 = 0; m2 = len; m3 = 0;
        }
        uint32_t cl[5];
        poly_block_limbs(m0, m1, m2, m3, 1u << 24, cl);
#pragma unroll
        for (int i = 0; i < 5; ++i) acc[i] += cl[i];
      }
    }

    // ---- finish packets whose last round this was ------------------------------------
    if (last) {
      if (valid) {
        uint32_t W[5], Ws[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) W[i] = lpow[5 * lane + i];
        poly_scale5(W, Ws);
        poly_mul(acc, W, Ws);
#pragma unroll
        for (uint32_t stp = 1; stp < 8u; stp <<= 1) {
          uint32_t y[5];
          shfl5(acc, (int)(j + stp < 8u ? lane + stp : lane), y);
          if (j + stp < 8u) {
#pragma unroll
            for (int i = 0; i < 5; ++i) acc[i] += y[i];
          }
        }
      }
      uint32_t bad = valid ? 0u : 1u;
      if (j == 0 && valid) {
        const uint4 sv = sotk[2 * s + 1];
        uint32_t tag[4];
        poly_finish(acc, sv.x, sv.y, sv.z, sv.w, tag);
        if constexpr (MODE == WG_MODE_SEAL) {
          uint8_t* tp = P.out + out_off + len;
          if ((((uintptr_t)tp) & 15u) == 0) {
            *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
          }
        } else {
          const uint8_t* tp = P.in + in_off + len;
          uint32_t diff = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
          bad = diff ? 1u : 0u;
        }
      }
      if constexpr (MODE == WG_MODE_OPEN) {
        bad = __shfl(bad, (int)sbase, 64);
        if (j == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
        if (bad && valid) {
          uint8_t* o = P.out + out_off;
          for (uint32_t i = j; i < len; i += 8u) o[i] = 0;
        }
      }
      // advance to the successor
      pkt += 8u;
      have = pkt < w1;
      if (have) {
        decode(sd_lo, sd_hi);
        if (j == 0 && valid) {
          skey[2 * s] = nk_a;
          skey[2 * s + 1] = nk_b;
        }
        if (pkt + 8u < w1) {
          const uint4* sp = (const uint4*)(P.desc + pkt + 8u);
          sd_lo = sp[0];
          sd_hi = sp[1];
        }
      }
    } else if (have) {
      ++round;
    }
    lds_fence();
    buf ^= 1u;
  }
}

// ---------------------------------------------------------------------------
// k_lean — k_stream's slot/round algorithm with the register footprint cut to
// <= 64 VGPRs (8 waves per SIMD): the slot's packet state, the per-lane Horner
// accumulator and the Poly1305 powers live in LDS between uses, the key is read
// from LDS on both sides of the rounds, and a block's payload is loaded after
// its keystream (latency covered by the other waves). gfx950 issues dependent
// add/xor streams at ~2.6 cycles only with ~8 waves per SIMD (tools/microbench4).
//   slot record (16 words): in_off lo/hi, out_off lo/hi | ctr lo/hi, len, valid |
//                           nb, nc, D, round | packet index (~0 = idle)
template <int MODE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) k_lean(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  __shared__ uint4 img[8 * 8 * 4];  // the round's MAC input, [slot][lane][4 chunks]
  __shared__ uint4 srec[8 * 4];     // slot records
  __shared__ uint4 skey[8 * 2];
  __shared__ uint4 sotk[8 * 2];
  __shared__ uint32_t spow[8 * 10];  // R = r^8 limbs, 5R limbs 1..4
  __shared__ uint32_t lpow[64 * 5];  // W = r^(8-j) per lane
  __shared__ uint32_t lacc[64 * 5];  // Horner accumulator per lane
  const uint32_t lane = threadIdx.x, s = lane >> 3, j = lane & 7u;
  const uint32_t sbase = lane & ~7u;
  const uint32_t w0 = blockIdx.x * P.ppw, w1 = min(P.n, w0 + P.ppw);

  // open packet `p` in slot `s` (called by the slot's lane j == 0)
  auto open_packet = [&](uint32_t p) {
    if (p >= w1) {
      srec[4 * s + 3] = make_uint4(~0u, 0, 0, 0);
      return;
    }
    const uint4* dp = (const uint4*)(P.desc + p);
    const uint4 lo = dp[0], hi = dp[1];
    const uint64_t in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
    const uint64_t out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
    const uint32_t len = hi.z;
    bool valid = len <= P.max_len && hi.w < P.key_slots;
    const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
    valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
    const uint32_t nb = ((len + 63u) >> 6) + 1u, nc = (len + 15u) >> 4;
    const uint32_t M = nc + 1u, K = (M + 7u) >> 3;
    srec[4 * s + 0] = lo;
    srec[4 * s + 1] = make_uint4(hi.x, hi.y, len, valid ? 1u : 0u);
    srec[4 * s + 2] = make_uint4(nb, nc, 8u * K - M, 0u);
    srec[4 * s + 3] = make_uint4(p, 0, 0, 0);
    if (valid) {
      const uint4* kp = (const uint4*)(P.keys + 8u * hi.w);
      skey[2 * s] = kp[0];
      skey[2 * s + 1] = kp[1];
    }
  };

  if (j == 0) open_packet(w0 + s);
#pragma unroll
  for (int i = 0; i < 5; ++i) lacc[5 * lane + i] = 0;
  uint32_t next = w0 + SLOT_LANES;  // wave-uniform
  lds_fence();

  while (true) {
    const uint4 r3 = srec[4 * s + 3];
    const bool have = r3.x != ~0u;
    if (!__any(have)) break;
    const uint4 r1 = srec[4 * s + 1];
    const uint4 r2 = srec[4 * s + 2];
    const bool valid = have && (r1.w & 1u);
    const uint32_t len = r1.z, nb = r2.x, round = r2.w;

    // ---- ChaCha20: block b of the slot's packet ------------------------------------
    const uint32_t b = 8u * round + j;
    if (valid && b < nb) {
      uint32_t ks[16];
      chacha20_block_lds(&skey[2 * s], b, r1.x, r1.y, 0u, ks);
      if (b == 0) {
        sotk[2 * s] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
        sotk[2 * s + 1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
      } else {
        const uint4 r0 = srec[4 * s];
        const uint32_t off = 64u * (b - 1u);
        const uint32_t n = min(64u, len - off);
        uint32_t w[16];
        load_block(P.in + ((uint64_t)r0.x | ((uint64_t)r0.y << 32)) + off, n, w);
        if constexpr (MODE == WG_MODE_OPEN) {
          if (n < 64u) mask_block(n, w);
          lds_store_block((uint8_t*)&img[4 * lane], w);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
        store_block(P.out + ((uint64_t)r0.z | ((uint64_t)r0.w << 32)) + off, n, w);
        if constexpr (MODE == WG_MODE_SEAL) {
          if (n < 64u) mask_block(n, w);
          lds_store_block((uint8_t*)&img[4 * lane], w);
        }
      }
    }
    lds_fence();

    // ---- Poly1305 over this round's chunks ---------------------------------------------
    if (valid) {
      if (round == 0) {  // lane j gets r^(j+1) by a product scan; R = r^8, W = r^(8-j)
        const uint4 o = sotk[2 * s];
        uint32_t x[5];
        poly_r_limbs(o.x, o.y, o.z, o.w, x);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5], ys[5];
          shfl5(x, (int)(j >= st ? lane - st : lane), y);
          poly_scale5(y, ys);
          if (j >= st) poly_mul(x, y, ys);
        }
        uint32_t t[5];
        shfl5(x, (int)(sbase + 7u - j), t);
#pragma unroll
        for (int i = 0; i < 5; ++i) lpow[5 * lane + i] = t[i];
        shfl5(x, (int)(sbase + 7u), t);
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < 5; ++i) spow[10 * s + i] = t[i];
#pragma unroll
          for (int i = 1; i < 5; ++i) spow[10 * s + 5 + i] = t[i] * 5u;
        }
        lds_fence();
      }
      const uint32_t nc = r2.y, D = r2.z;
      const uint32_t blo = max(8u * round, 1u);
      const uint32_t c_lo = 4u * (blo - 1u);
      const uint32_t c_end = (8u * (round + 1u) >= nb) ? nc + 1u : min(nc, 4u * (8u * round + 7u));
      uint32_t c = c_lo + ((j - ((c_lo + D) & 7u)) & 7u);
      if (c < c_end) {
        uint32_t acc[5], R[5], Rs[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) acc[i] = lacc[5 * lane + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) R[i] = spow[10 * s + i];
        Rs[0] = 0;
#pragma unroll
        for (int i = 1; i < 5; ++i) Rs[i] = spow[10 * s + 5 + i];
        for (; c < c_end; c += 8u) {
          poly_mul(acc, R, Rs);
          uint32_t m0, m1, m2, m3;
          if (c < nc) {
            const uint4 v = img[4u * (sbase + (c >> 2) + 1u - 8u * round) + (c & 3u)];
            m0 = v.x; m1 = v.y; m2 = v.z; m3 = v.w;
          } else {  // le64(0) || le64(len) (ChaCha20Poly1305.java:88-90)
            m0 = 0; m1 = 0; m2 = len; m3 = 0;
          }
          uint32_t cl[5];
          poly_block_limbs(m0, m1, m2, m3, 1u << 24, cl);
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[i] += cl[i];
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) lacc[5 * lane + i] = acc[i];
      }
    }

    // ---- finish packets whose last round this was ----------------------------------------
    const bool done = have && (!valid || 8u * (round + 1u) >= nb);
    if (done) {
      uint32_t bad = valid ? 0u : 1u;
      if (valid) {
        uint32_t acc[5], W[5], Ws[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) acc[i] = lacc[5 * lane + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) W[i] = lpow[5 * lane + i];
        poly_scale5(W, Ws);
        poly_mul(acc, W, Ws);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5];
          shfl5(acc, (int)(j + st < 8u ? lane + st : lane), y);
          if (j + st < 8u) {
#pragma unroll
            for (int i = 0; i < 5; ++i) acc[i] += y[i];
          }
        }
        if (j == 0) {
          const uint4 sv = sotk[2 * s + 1];
          const uint4 r0 = srec[4 * s];
          uint32_t tag[4];
          poly_finish(acc, sv.x, sv.y, sv.z, sv.w, tag);
          if constexpr (MODE == WG_MODE_SEAL) {
            uint8_t* tp = P.out + ((uint64_t)r0.z | ((uint64_t)r0.w << 32)) + len;
            if ((((uintptr_t)tp) & 15u) == 0) {
              *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
            }
          } else {
            const uint8_t* tp = P.in + ((uint64_t)r0.x | ((uint64_t)r0.y << 32)) + len;
            uint32_t diff = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
            bad = diff ? 1u : 0u;
          }
        }
      }
      if constexpr (MODE == WG_MODE_OPEN) {
        bad = __shfl(bad, (int)sbase, 64);
        if (j == 0 && P.status) P.status[r3.x] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
        if (bad && valid) {  // scrub the unauthenticated plaintext written this call
          const uint4 r0 = srec[4 * s];
          uint8_t* o = P.out + ((uint64_t)r0.z | ((uint64_t)r0.w << 32));
          for (uint32_t i = j; i < len; i += 8u) o[i] = 0;
        }
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) lacc[5 * lane + i] = 0;
    }
    // hand the wave's next packets to the slots that finished (ballot rank)
    const unsigned long long fin = __ballot(done && j == 0);
    lds_fence();
    if (j == 0 && have) {
      if (done) open_packet(next + (uint32_t)__popcll(fin & ((1ull << sbase) - 1ull)));
      else srec[4 * s + 2].w = round + 1u;
    }
    next += (uint32_t)__popcll(fin);
    lds_fence();
  }
}

// explicit instantiations used by wg_capi.hip
// ---------------------------------------------------------------------------
// k_wave — k_stream's slot/round algorithm laid out for 8 waves per SIMD:
// <= 64 VGPRs and 5024 B of LDS per wave (160 KB / 5 KB = 32 waves per CU).
//  * lane-derived values (slot, lane in slot, LDS addresses, shuffle sources) come
//    from an opaque copy of threadIdx.x in each phase, so the compiler recomputes
//    them (1-3 VALU) instead of keeping ~25 hoisted constants live across the rounds;
//  * the packet record (offsets, counter, length, validity) lives in LDS and is
//    re-read where needed; the ChaCha key is re-read for the feed-forward;
//  * W = r^(8-j) stays in 5 VGPRs (k_stream kept it in 1.25 KB of LDS); only
//    R = r^8 is stored, 5R is formed on the fly;
//  * the Poly1305 step per round is 4 predicated chunk steps at constant LDS
//    offsets: chunk c of the slot's round image sits at img[4 sbase + 4 - 32 round + c].
//  * WPG independent waves share a workgroup (each with its own LDS arrays, no
//    block barriers): one-wave workgroups are dispatched at only ~1 per 11 cycles
//    chip-wide, which left a 65536-packet launch with ~40% of its wave slots empty.
// Results are identical to k_stream (same Horner order, same finish).
// Variant bits V: 1 prefetch the round's payload before the ChaCha rounds,
// 2 amdgpu_waves_per_eu(8) (cap at 64 VGPRs), 4 progress-based s_setprio,
// 8 every lane reads the descriptor (round-0 payload requested with it),
// 16 rotl16 as SDWA xors (wg_device.h xor_rotl16_sdwa; measured no faster),
// 32 slot keys through scalar loads (fetch_slot_keys; measured no faster),
// 64 workgroup-lockstep rounds (one barrier per round), 128 slot-cooperative
// interleaved payload loads through the round image.
__device__ __forceinline__ uint32_t opaque_lane() {
  uint32_t x = threadIdx.x & 63u;
  asm volatile("" : "+v"(x));
  return x;
}
// orders this wave's LDS writes before its other lanes' reads (LDS is in order per wave)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Scalar loads of the keys of the slots whose bit 8s is set in `need` (lane 8s holds
// the slot's key index in `key_slot`), two slots per statement, written to skey.
// The loads and their wait sit in one asm statement (cdna_hip_programming.md §5.7).
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void fetch_slot_keys(const uint32_t* keys, uint32_t key_slot, unsigned long long need,
                                                uint4* skey) {
  const uint32_t lane = opaque_lane();
#pragma unroll
  for (int ss = 0; ss < 8; ss += 2) {
    const bool na = (need >> (8 * ss)) & 1ull, nb = (need >> (8 * ss + 8)) & 1ull;
    if (!na && !nb) continue;  // wave-uniform
    const uint32_t ka = __builtin_amdgcn_readlane(key_slot, 8 * ss);
    const uint32_t kb = __builtin_amdgcn_readlane(key_slot, 8 * ss + 8);
    const uint32_t* pa = keys + 8u * (na ? ka : 0u);
    const uint32_t* pb = keys + 8u * (nb ? kb : 0u);
    u32x8 a, b;
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx8 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(pa), "s"(pb));
    if (na && lane == 8u * ss) {
      skey[2 * ss] = make_uint4(a[0], a[1], a[2], a[3]);
      skey[2 * ss + 1] = make_uint4(a[4], a[5], a[6], a[7]);
    }
    if (nb && lane == 8u * ss + 8u) {
      skey[2 * ss + 2] = make_uint4(b[0], b[1], b[2], b[3]);
      skey[2 * ss + 3] = make_uint4(b[4], b[5], b[6], b[7]);
    }
  }
}

template <int MODE, int V, int WPG>
__global__ void __launch_bounds__(64 * WPG) __attribute__((amdgpu_waves_per_eu((V & 2) ? 8 : 1)))
k_wave(StreamParams P) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  __shared__ uint4 img_[WPG][8 * 8 * 4];  // 4096 B per wave: [slot][lane][4 chunks], the round's MAC input
  __shared__ uint4 skey_[WPG][8 * 2];     // 256 B: slot ChaCha key
  __shared__ uint4 sotk_[WPG][8 * 2];     // 256 B: slot Poly1305 one-time key r || s
  __shared__ uint4 srec_[WPG][8 * 2];     // 256 B: {in_off, out_off} {ctr lo, ctr hi, len, valid}
  __shared__ uint32_t spow_[WPG][8 * 5];  // 160 B: R = r^8 limbs
  const uint32_t wv = WPG == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4* const img = img_[wv];
  uint4* const skey = skey_[wv];
  uint4* const sotk = sotk_[wv];
  uint4* const srec = srec_[wv];
  uint32_t* const spow = spow_[wv];
  const uint32_t w0 = (blockIdx.x * WPG + wv) * P.ppw, w1 = min(P.n, w0 + P.ppw);
  uint32_t next = w0 + SLOT_LANES;  // wave-uniform
  uint32_t pkt = w0 + (opaque_lane() >> 3);
  bool have = pkt < w1;
  uint32_t round = 0;
  uint32_t acc[5], W[5];
  uint32_t key_slot = ~0u;  // V & 32: lane 0 of a starting slot holds its key slot
  WG_PH_DECL
  uint32_t wave_rounds = 0;  // wave-uniform

  // V & 64: the workgroup's waves advance round by round together (one barrier per
  // round; every wave runs the same trip count, idle once its slots are done), so a
  // workgroup's waves finish together instead of trickling out of the SIMDs.
  while ((V & 64) ? (__syncthreads_or(have ? 1 : 0) != 0) : __any(have)) {
    if constexpr ((V & 4) != 0) progress_prio(wave_rounds++);
    WG_PH_MARK();
    uint32_t w[16];
    if (have && round == 0) {  // start a packet: lane 0 of the slot fills the record
      const uint32_t lane = opaque_lane(), s = lane >> 3, j = lane & 7u;
      if ((V & 8) || j == 0) {  // V & 8: every lane reads the descriptor (one coalesced request)
        const uint4* dp = (const uint4*)(P.desc + pkt);
        const uint4 lo = dp[0], hi = dp[1];
        const uint64_t in_off = (uint64_t)lo.x | ((uint64_t)lo.y << 32);
        const uint64_t out_off = (uint64_t)lo.z | ((uint64_t)lo.w << 32);
        const uint32_t len = hi.z, ks_ = hi.w;
        bool valid = len <= P.max_len && ks_ < P.key_slots;
        const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
        const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
        valid = valid && in_off <= P.in_size && in_need <= P.in_size - in_off;
        valid = valid && out_off <= P.out_size && out_need <= P.out_size - out_off;
        if constexpr ((V & 8) != 0) {
          // round 0's payload is requested now, in parallel with lane 0's key fetch
          const uint32_t nbk = ((len + 63u) >> 6) + 1u;
          if (valid && j > 0 && j < nbk) load_block(P.in + in_off + 64u * (j - 1u), min(64u, len - 64u * (j - 1u)), w);
        }
        if (j == 0) {
          srec[2 * s] = lo;
          srec[2 * s + 1] = make_uint4(hi.x, hi.y, len, valid ? 1u : 0u);
          if constexpr ((V & 32) != 0) {
            if (valid) key_slot = ks_;
          } else if (valid) {
            const uint4* kp = (const uint4*)(P.keys + 8u * ks_);
            skey[2 * s] = kp[0];
            skey[2 * s + 1] = kp[1];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[i] = 0;
    }
    if constexpr ((V & 32) != 0) {
      // the starting slots' keys through the scalar cache: one L2 request per SQC
      // instead of one per wave, so a key shared by many packets (one session)
      // does not serialise every wave of the launch on one L2 channel
      const unsigned long long need = __ballot(key_slot != ~0u);  // bit 8s: slot s starts a valid packet
      if (need) fetch_slot_keys(P.keys, key_slot, need, skey);
      key_slot = ~0u;
    }
    wave_lds_sync();  // the record writes before the slot's other lanes read them
    WG_PH_ADD(0);

    // ---- ChaCha20: block b = 8 round + j of the slot's packet ----------------------
    {
      const uint32_t lane = opaque_lane(), s = lane >> 3, j = lane & 7u;
      const uint4 rc = srec[2 * s + 1];
      const uint32_t len = rc.z;
      const uint32_t nb = ((len + 63u) >> 6) + 1u;
      const uint32_t b = 8u * round + j;
      const bool act = have && rc.w && b < nb;
      const bool data = act && b > 0;
      const uint32_t off = 64u * (b - 1u);
      const uint32_t nbytes = data ? min(64u, len - off) : 0u;
      const bool prefetched = (V & 8) && round == 0;
      uint4 cp[4];  // V & 128: this lane's chunks 8i + j of the slot's 512-B round window
      if constexpr ((V & 128) != 0) {
        // the slot's 8 lanes read the window interleaved (128 contiguous bytes per
        // instruction) instead of one 64-B block each (tools/microbench8: 4.6 vs 3.6 TB/s)
        const uint4 ro = srec[2 * s];
        const uint8_t* base = P.in + ((uint64_t)ro.x | ((uint64_t)ro.y << 32));
        const bool a16 = (((uintptr_t)base) & 15u) == 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          const uint32_t c = 8u * i + j, bb = 8u * round + (c >> 2);
          const uint32_t coff = 64u * (bb - 1u) + 16u * (c & 3u);
          cp[i] = make_uint4(0, 0, 0, 0);
          if (have && rc.w && bb >= 1u && bb < nb && coff < len) {
            if (a16 && len - coff >= 16u) {
              cp[i] = *(const uint4*)(base + coff);
            } else {
              uint32_t w4[4];
              load_chunk16(base + coff, min(16u, len - coff), w4);
              cp[i] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
          }
        }
      } else if ((V & 1) && data && !prefetched) {
        const uint4 ro = srec[2 * s];
        load_block(P.in + ((uint64_t)ro.x | ((uint64_t)ro.y << 32)) + off, nbytes, w);
      }
      uint32_t ks[16];
      if (act) chacha20_block_lds<(V & 16) != 0>(&skey[2 * s], b, rc.x, rc.y, 0u, ks);
      if constexpr ((V & 128) != 0) {  // window chunks -> the slot's image; each lane takes its block
        wave_lds_sync();
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) img[32u * s + 8u * i + j] = cp[i];
        wave_lds_sync();
        if (data) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint4 v = img[4 * lane + q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
          }
        }
      }
      if (act) {
        if (!data) {
          sotk[2 * s] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
          sotk[2 * s + 1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
        } else {
          const uint4 ro = srec[2 * s];
          if (!(V & 1) && !(V & 128) && !prefetched)
            load_block(P.in + ((uint64_t)ro.x | ((uint64_t)ro.y << 32)) + off, nbytes, w);
          if constexpr (MODE == WG_MODE_OPEN && (V & 128) == 0) {  // V & 128: the image already holds it
            if (nbytes < 64u) mask_block(nbytes, w);
            lds_store_block((uint8_t*)&img[4 * lane], w);
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
          store_block(P.out + ((uint64_t)ro.z | ((uint64_t)ro.w << 32)) + off, nbytes, w);
          if constexpr (MODE == WG_MODE_SEAL) {
            if (nbytes < 64u) mask_block(nbytes, w);
            lds_store_block((uint8_t*)&img[4 * lane], w);
          }
        }
      }
    }
    wave_lds_sync();
    WG_PH_ADD(1);

    // ---- Poly1305 over this round's chunks ------------------------------------------
    const uint4 rc = srec[2 * (opaque_lane() >> 3) + 1];
    const bool valid = rc.w != 0;
    const uint32_t len = rc.z, nb = ((len + 63u) >> 6) + 1u, nc = (len + 15u) >> 4;
    if (have && valid) {
      const uint32_t lane = opaque_lane(), s = lane >> 3, j = lane & 7u, sbase = lane & ~7u;
      if (round == 0) {  // r and its powers: lane j gets r^(j+1); R = r^8, W = r^(8-j)
        const uint4 o = sotk[2 * s];
        uint32_t x[5];
        poly_r_limbs(o.x, o.y, o.z, o.w, x);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5], ys[5];
          shfl5(x, (int)(j >= st ? lane - st : lane), y);
          poly_scale5(y, ys);
          if (j >= st) poly_mul(x, y, ys);
        }
        shfl5(x, (int)(sbase + 7u - j), W);
        if (j == 7u) {
#pragma unroll
          for (int i = 0; i < 5; ++i) spow[5 * s + i] = x[i];
        }
      }
      uint32_t R[5], Rs[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) R[i] = spow[5 * s + i];
      poly_scale5(R, Rs);
      const uint32_t M = nc + 1u, D = 8u * ((M + 7u) >> 3) - M;
      const uint32_t c_lo = round ? 32u * round - 4u : 0u;
      const uint32_t c_end = min(nc, 32u * round + 28u);
      const uint32_t c0 = c_lo + ((j - ((c_lo + D) & 7u)) & 7u);
      const uint4* ip = &img[4u * sbase + 4u - 32u * round + c0];
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t) {
        if (c0 + 8u * t < c_end) {
          const uint4 v = ip[8u * t];
          poly_mul(acc, R, Rs);
          uint32_t cl[5];
          poly_block_limbs(v.x, v.y, v.z, v.w, 1u << 24, cl);
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[i] += cl[i];
        }
      }
    }

    WG_PH_ADD(2);
    // ---- finish packets whose last round this was ------------------------------------
    const bool done = have && (!valid || 8u * (round + 1u) >= nb);
    if (done) {
      const uint32_t lane = opaque_lane(), s = lane >> 3, j = lane & 7u, sbase = lane & ~7u;
      if (valid) {
        if (j == 7u) {  // the length block le64(0) || le64(len) is lane 7's last position
          uint32_t R[5], Rs[5];
#pragma unroll
          for (int i = 0; i < 5; ++i) R[i] = spow[5 * s + i];
          poly_scale5(R, Rs);
          poly_mul(acc, R, Rs);
          acc[2] += (len << 12) & M26;  // le64(len) sits at bit 64: limb 2 = bits 52..77
          acc[3] += len >> 14;
          acc[4] += 1u << 24;
        }
        uint32_t Ws[5];
        poly_scale5(W, Ws);
        poly_mul(acc, W, Ws);
#pragma unroll
        for (uint32_t st = 1; st < 8u; st <<= 1) {
          uint32_t y[5];
          shfl5(acc, (int)(j + st < 8u ? lane + st : lane), y);
          if (j + st < 8u) {
#pragma unroll
            for (int i = 0; i < 5; ++i) acc[i] += y[i];
          }
        }
      }
      uint32_t bad = valid ? 0u : 1u;
      if (j == 0 && valid) {
        const uint4 sv = sotk[2 * s + 1];
        uint32_t tag[4];
        poly_finish(acc, sv.x, sv.y, sv.z, sv.w, tag);
        const uint4 ro = srec[2 * s];
        if constexpr (MODE == WG_MODE_SEAL) {
          uint8_t* tp = P.out + ((uint64_t)ro.z | ((uint64_t)ro.w << 32)) + len;
          if ((((uintptr_t)tp) & 15u) == 0) {
            *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
          }
        } else {  // all 16 bytes compared, no early exit
          const uint8_t* tp = P.in + ((uint64_t)ro.x | ((uint64_t)ro.y << 32)) + len;
          uint32_t diff = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
          bad = diff ? 1u : 0u;
        }
      }
      if constexpr (MODE == WG_MODE_OPEN) {
        bad = __shfl(bad, (int)sbase, 64);
        if (j == 0 && P.status) P.status[pkt] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
        if (bad && valid) {  // scrub the unauthenticated plaintext written this call
          const uint4 ro = srec[2 * s];
          uint8_t* o = P.out + ((uint64_t)ro.z | ((uint64_t)ro.w << 32));
          for (uint32_t i = j; i < len; i += 8u) o[i] = 0;
        }
      }
    }
    // hand the wave's next packets to the slots that finished (ballot rank)
    const unsigned long long fin = __ballot(done && (opaque_lane() & 7u) == 0);
    if (done) {
      const uint32_t sbase = opaque_lane() & ~7u;
      const uint32_t rank = (uint32_t)__popcll(fin & ((1ull << sbase) - 1ull));
      pkt = next + rank;
      have = pkt < w1;
      round = 0;
    } else if (have) {
      ++round;
    }
    next += (uint32_t)__popcll(fin);
    wave_lds_sync();  // the next packet's record overwrites this one's
    WG_PH_ADD(3);
  }
  WG_PH_STORE_WAVE(blockIdx.x * WPG + wv);
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
#define WG_STREAM_INST(V)                                                \
  template __global__ void k_stream<WG_MODE_SEAL, V>(StreamParams); \
  template __global__ void k_stream<WG_MODE_OPEN, V>(StreamParams);
WG_STREAM_INST(0) WG_STREAM_INST(1) WG_STREAM_INST(2) WG_STREAM_INST(3)
WG_STREAM_INST(4) WG_STREAM_INST(5) WG_STREAM_INST(6) WG_STREAM_INST(7)
WG_STREAM_INST(9) WG_STREAM_INST(11) WG_STREAM_INST(15) WG_STREAM_INST(17) WG_STREAM_INST(33) WG_STREAM_INST(49)
WG_STREAM_INST(65) WG_STREAM_INST(73)
template __global__ void k_lean<WG_MODE_SEAL>(StreamParams);
template __global__ void k_lean<WG_MODE_OPEN>(StreamParams);
template __global__ void k_pipe<WG_MODE_SEAL, 0>(StreamParams);
template __global__ void k_pipe<WG_MODE_OPEN, 0>(StreamParams);

}  // namespace wgk
