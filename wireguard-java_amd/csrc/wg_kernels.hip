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
// Slow path (packet tails, unaligned packets): predicated byte accesses.
__device__ __forceinline__ void load_block(const uint8_t* src, uint32_t n, uint32_t w[16]) {
  if (n == 64u && (((uintptr_t)src) & 15u) == 0) {
    const uint4* p = (const uint4*)src;
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w; w[12] = d.x; w[13] = d.y; w[14] = d.z; w[15] = d.w;
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((uint32_t)(4 * k + b) < n) v |= (uint32_t)src[4 * k + b] << (8 * b);
      w[k] = v;
    }
  }
}

__device__ __forceinline__ void store_block(uint8_t* dst, uint32_t n, const uint32_t w[16]) {
  if (n == 64u && (((uintptr_t)dst) & 15u) == 0) {
    uint4* p = (uint4*)dst;
    p[0] = make_uint4(w[0], w[1], w[2], w[3]);
    p[1] = make_uint4(w[4], w[5], w[6], w[7]);
    p[2] = make_uint4(w[8], w[9], w[10], w[11]);
    p[3] = make_uint4(w[12], w[13], w[14], w[15]);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((uint32_t)(4 * k + b) < n) dst[4 * k + b] = (uint8_t)(w[k] >> (8 * b));
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
// LDS tile header: per-packet records (struct of arrays) followed by the image.
struct TileLds {
  uint32_t* blk;     // [mp + 1] tile-local first block of packet q
  uint32_t* len;     // [mp]
  uint32_t* aadlen;  // [mp]
  uint32_t* flags;   // [mp] bit0 = valid
  uint32_t* key;     // [mp * 8] ChaCha key (AEAD/CIPHER) or one-time key (MAC)
  uint32_t* nonce;   // [mp * 4] n0, n1, n2, ctr0
  uint32_t* otk;     // [mp * 8] Poly1305 one-time key from block 0
  uint32_t* verdict; // [mp]
  uint64_t* in_off;  // [mp]
  uint64_t* out_off; // [mp]
  uint64_t* aad_off; // [mp]
  uint8_t* img;      // image bytes
};

__device__ __forceinline__ TileLds carve(uint8_t* base, uint32_t mp) {
  TileLds t;
  t.in_off = (uint64_t*)base;
  t.out_off = t.in_off + mp;
  t.aad_off = t.out_off + mp;
  uint32_t* u = (uint32_t*)(t.aad_off + mp);
  t.blk = u; u += mp + 1;
  t.len = u; u += mp;
  t.aadlen = u; u += mp;
  t.flags = u; u += mp;
  t.verdict = u; u += mp;
  t.key = u; u += 8 * mp;
  t.nonce = u; u += 4 * mp;
  t.otk = u; u += 8 * mp;
  t.img = base + tile_header_bytes(mp);
  return t;
}

__device__ __forceinline__ void shfl5(const uint32_t v[5], int src, uint32_t o[5]) {
#pragma unroll
  for (int i = 0; i < 5; ++i) o[i] = __shfl(v[i], src, 64);
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
  TileLds L = carve(lds_raw, P.max_tile_pkts);

  // ---- packet records --------------------------------------------------------
  for (uint32_t q = tid; q < np; q += WG_TPB) {
    Pkt pk = load_pkt<GENERAL>(P.desc, p0 + q);
    uint32_t len = pk.len;
    bool ok = len <= P.max_len && pk.key_slot < P.key_slots;
    if (P.uniform) ok = ok && len == P.max_len;
    // bounds against the caller's buffers
    uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
    uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
    if (MODE == WG_MODE_MAC) out_need = 16u;
    ok = ok && pk.in_off <= P.in_size && in_need <= P.in_size - pk.in_off;
    ok = ok && pk.out_off <= P.out_size && out_need <= P.out_size - pk.out_off;
    if (GENERAL && AEAD && pk.aad_len)
      ok = ok && pk.aad_off <= P.aad_size && (uint64_t)pk.aad_len <= P.aad_size - pk.aad_off;
    L.len[q] = len;
    L.aadlen[q] = pk.aad_len;
    L.flags[q] = ok ? 1u : 0u;
    L.verdict[q] = 0u;
    L.in_off[q] = pk.in_off;
    L.out_off[q] = pk.out_off;
    L.aad_off[q] = pk.aad_off;
    L.nonce[4 * q + 0] = pk.n0; L.nonce[4 * q + 1] = pk.n1; L.nonce[4 * q + 2] = pk.n2; L.nonce[4 * q + 3] = pk.ctr0;
    const uint4* kp = (const uint4*)(P.keys + 8u * (ok ? pk.key_slot : 0u));
    uint4 ka = kp[0], kb = kp[1];
    uint32_t* kd = L.key + 8 * q;
    kd[0] = ka.x; kd[1] = ka.y; kd[2] = ka.z; kd[3] = ka.w; kd[4] = kb.x; kd[5] = kb.y; kd[6] = kb.z; kd[7] = kb.w;
    L.blk[q] = P.uniform ? q * P.nb_uniform : P.blk_prefix[p0 + q] - P.blk_prefix[p0];
  }
  if (tid == 0) L.blk[np] = P.uniform ? np * P.nb_uniform : P.blk_prefix[p1] - P.blk_prefix[p0];
  __syncthreads();

  // ---- phase 1: ChaCha20 over every counter block of the tile ---------------
  const uint32_t nblk = L.blk[np];
  for (uint32_t b = tid; b < nblk; b += WG_TPB) {
    uint32_t q;
    if (P.uniform) {
      q = P.nb_uniform == 1u ? b : __umulhi(b, P.nb_magic);
    } else {  // last q with blk[q] <= b
      uint32_t lo = 0, hi = np;
      while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (L.blk[mid] <= b) lo = mid; else hi = mid;
      }
      q = lo;
    }
    if (!(L.flags[q] & 1u)) continue;
    const uint32_t j = b - L.blk[q];
    const uint32_t len = L.len[q];
    const uint32_t d = AEAD ? j - 1u : j;  // data block index
    uint8_t* img = L.img + 64u * (L.blk[q] - (AEAD ? q : 0u));

    if constexpr (MODE == WG_MODE_MAC) {
      uint32_t off = 64u * d, n = min(64u, len - off);
      uint32_t w[16];
      load_block(P.in + L.in_off[q] + off, n, w);
      mask_block(n, w);
      lds_store_block(img + off, w);
      continue;
    } else {
      uint32_t key[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) key[i] = L.key[8 * q + i];
      const uint32_t n0 = L.nonce[4 * q + 0], n1 = L.nonce[4 * q + 1], n2 = L.nonce[4 * q + 2];
      const uint32_t ctr = (MODE == WG_MODE_CIPHER) ? L.nonce[4 * q + 3] + j : j;
      uint32_t ks[16];
      chacha20_block(key, ctr, n0, n1, n2, ks);
      if (AEAD && j == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) L.otk[8 * q + i] = ks[i];
        continue;
      }
      const uint32_t off = 64u * d, n = min(64u, len - off);
      uint32_t w[16];
      load_block(P.in + L.in_off[q] + off, n, w);
      if constexpr (MODE == WG_MODE_OPEN) {
        mask_block(n, w);
        lds_store_block(img + off, w);  // MAC over the received ciphertext
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] ^= ks[i];
      store_block(P.out + L.out_off[q] + off, n, w);
      if constexpr (MODE == WG_MODE_SEAL) {
        mask_block(n, w);
        lds_store_block(img + off, w);  // MAC over the ciphertext just produced
      }
    }
  }
  if constexpr (MODE == WG_MODE_CIPHER) return;
  __syncthreads();

  // ---- phase 2: Poly1305, G lanes per packet --------------------------------
  {
    const uint32_t G = P.poly_g;
    const uint32_t ppw = 64u / G;           // packets per wave
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const uint32_t gq = lane / G, j = lane - gq * G;
    const uint32_t base = gq * G;           // first lane of the group
    const bool lane_used = gq < ppw;
    for (uint32_t qb = wave * ppw; qb < np; qb += (WG_TPB / 64u) * ppw) {
      const uint32_t q = qb + gq;
      const bool act = lane_used && q < np && (L.flags[q] & 1u);
      // r, s from the one-time key
      uint32_t k0, k1, k2, k3, s0, s1, s2, s3;
      {
        const uint32_t* src = AEAD ? L.otk : L.key;
        uint32_t qq = act ? q : 0u;
        k0 = src[8 * qq + 0]; k1 = src[8 * qq + 1]; k2 = src[8 * qq + 2]; k3 = src[8 * qq + 3];
        s0 = src[8 * qq + 4]; s1 = src[8 * qq + 5]; s2 = src[8 * qq + 6]; s3 = src[8 * qq + 7];
      }
      uint32_t r[5], rs[5];
      poly_r_limbs(k0, k1, k2, k3, r);
      // powers: lane j of the group ends with r^(j+1)
      uint32_t x[5] = {r[0], r[1], r[2], r[3], r[4]};
      for (uint32_t st = 1; st < G; st <<= 1) {
        uint32_t y[5], ys[5];
        shfl5(x, (int)(lane >= st ? lane - st : lane), y);
        poly_scale5(y, ys);
        if (j >= st) poly_mul(x, y, ys);
      }
      uint32_t R[5], Rs[5], W[5], Ws[5];
      shfl5(x, (int)min(base + G - 1u, 63u), R);
      shfl5(x, (int)min(base + G - 1u - j, 63u), W);
      poly_scale5(R, Rs);
      poly_scale5(W, Ws);
      (void)rs;

      uint32_t acc[5] = {0, 0, 0, 0, 0};
      if (act) {
        const uint32_t len = L.len[q], alen = L.aadlen[q];
        const uint32_t na = (alen + 15u) >> 4, nc = (len + 15u) >> 4;
        const uint32_t M = (MODE == WG_MODE_MAC) ? nc : na + nc + 1u;
        const uint32_t K = (M + G - 1u) / G;
        const int D = (int)(K * G - M);
        const uint8_t* img = L.img + 64u * (L.blk[q] - (AEAD ? q : 0u));
        for (uint32_t k = 0; k < K; ++k) {
          if (k) poly_mul(acc, R, Rs);
          const int t = (int)(j + k * G) - D;
          if (t < 0) continue;
          uint32_t w[4];
          uint32_t hib = 1u << 24;
          const uint32_t tt = (uint32_t)t;
          if (MODE == WG_MODE_MAC) {
            uint4 v = *(const uint4*)(img + 16u * tt);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            const uint32_t rem = len - 16u * tt;
            if (rem < 16u) {  // final partial block: 0x01 pad, no 2^128 bit (poly1305-donna-64.h:162-168)
              hib = 0;
              const uint32_t sh = 8u * (rem & 3u);
              const uint32_t wi = rem >> 2;
              w[0] |= (wi == 0) ? (1u << sh) : 0u;
              w[1] |= (wi == 1) ? (1u << sh) : 0u;
              w[2] |= (wi == 2) ? (1u << sh) : 0u;
              w[3] |= (wi == 3) ? (1u << sh) : 0u;
            }
          } else if (tt < na) {
            const uint32_t o = 16u * tt;
            load_chunk16(P.aad + L.aad_off[q] + o, min(16u, alen - o), w);
          } else if (tt < na + nc) {
            uint4 v = *(const uint4*)(img + 16u * (tt - na));
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
          } else {  // le64(aad_len) || le64(ct_len) (ChaCha20Poly1305.java:88-90)
            w[0] = alen; w[1] = 0; w[2] = len; w[3] = 0;
          }
          uint32_t c[5];
          poly_block_limbs(w[0], w[1], w[2], w[3], hib, c);
#pragma unroll
          for (int i = 0; i < 5; ++i) acc[i] += c[i];
        }
        poly_mul(acc, W, Ws);
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
        poly_finish(acc, s0, s1, s2, s3, tag);
        const uint32_t len = L.len[q];
        if constexpr (MODE == WG_MODE_SEAL) {
          uint8_t* tp = P.out + L.out_off[q] + len;
#pragma unroll
          for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
        } else if constexpr (MODE == WG_MODE_MAC) {
          uint8_t* tp = P.out + L.out_off[q];
#pragma unroll
          for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
        } else {  // OPEN: compare (full 16 bytes, no early exit)
          const uint8_t* tp = P.in + L.in_off[q] + len;
          uint32_t diff = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
          L.verdict[q] = diff ? 1u : 0u;
        }
      }
    }
  }

  if constexpr (MODE == WG_MODE_OPEN) {
    __syncthreads();
    for (uint32_t q = 0; q < np; ++q) {
      const bool valid = L.flags[q] & 1u;
      const uint32_t bad = valid ? L.verdict[q] : 1u;
      if (tid == 0 && P.status) P.status[p0 + q] = bad ? WG_PKT_BADTAG : WG_PKT_OK;
      if (bad && valid) {  // scrub the unauthenticated plaintext
        uint8_t* o = P.out + L.out_off[q];
        for (uint32_t i = tid; i < L.len[q]; i += WG_TPB) o[i] = 0;
      }
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

// explicit instantiations used by wg_capi.hip
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
