// wg_transport.hip — the transport-data seal/open kernel for gfx950 (product path).
//
// Replaces the per-packet SymmetricKeypair.cipher / decipher
// (ax.xz.wireguard.noise/src/main/java/ax/xz/wireguard/noise/handshake/SymmetricKeypair.java:63-83)
// over a batch of independent packets: ChaCha20 keystream from counter 1, Poly1305 key from
// block 0, MAC over ct || pad16 || le64(0) || le64(len) (ChaCha20Poly1305.java:31-93), with the
// reference's nonce LE64(counter) || 0^4 (SymmetricKeypair.java:52-61).
//
// Layout (k_transport<MODE>): a wave is 8 SLOTS of 8 lanes; a slot owns one packet at a
// time and streams it in ROUNDS of 8 ChaCha20 counter blocks (512 bytes):
//   * lane j of the slot computes block b = 8 round + j in registers (block 0 = the
//     Poly1305 one-time key), XORs its 64 payload bytes, stores them, and leaves the
//     round's MAC input (the ciphertext) in a 4 KB per-wave LDS image;
//   * the same 8 lanes advance an 8-strided Horner evaluation of the MAC polynomial
//     over the image (lane j owns positions = j mod 8, multiplier r^8, front padding
//     so the length block lands on lane 7); on the last round lane j scales its partial
//     by r^(8-j), the slot sums the 8 partials and lane 0 finishes the tag.
// ChaCha20: the first column round of columns 1..3 depends only on the key and the nonce, so
// lanes 1..3 of a slot compute it once per packet and every block takes it by ds_swizzle
// broadcast (chacha20_block_hoisted: -3% VALU instructions on C1). Poly1305: the length block
// is written into the image by the lane whose counter block holds it, so the Horner steps
// read it like ciphertext; each step's product chains every limb's carry into the next limb's
// v_mad_u64_u32 accumulator (poly_mul: 5 fewer instructions per step than five independent
// chains with the carries added afterwards; C1 +1.2%, C2 +0.2% in round 3, where round 2's
// kernel had measured the independent chains +3% on C2). The
// r-power scan and the slot sum exchange limbs through DPP (row_shr / quad_perm), which stays
// in the VALU instead of an LDS round trip in the middle of a dependent chain.
// Slots are persistent: slot g of S processes batch positions g, 2S-1-g, 2S+g, ... (a
// snake over the grid). Mixed-length batches are first ordered longest-first on the
// device (k_lpt_*), so the snake deals every slot one long and one short packet
// (LPT); uniform batches take positions in order. The next packet's descriptor is
// prefetched one packet ahead (one dword per lane), so a slot never waits on a
// dependent descriptor load when it starts a packet.
//
// IO: a lane's 64 payload bytes are fetched before the ARX rounds with LDS-DMA
// (global_load_lds, 16 B per lane per instruction) into the wave's chunk-major LDS image,
// so no registers are held across the rounds; chunks holding a valid byte are read whole
// (an aligned 16-B read never leaves the granule of its first byte) and masked. Unaligned
// inputs stage aligned dwords through registers (v_alignbyte). Stores are dwordx4 for
// 16-B aligned outputs, dword + bytes for 4-B aligned ones, bytes otherwise.
// Per-slot state (offsets, counter, length, flags, R = r^8, 5R, s, key) lives in a 128-B
// LDS record. A wave whose 8 slots share one key slot fetches the key through the scalar
// cache. Open writes the plaintext in the same pass and zero-fills it again if the tag does
// not verify (the host per-packet wrappers copy back only verified plaintext, as
// ChaCha20Poly1305.java:40-56 leaves dst untouched).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wg_device.h"
#include "wg_kernels.h"
#include "wg_stitch.h"

namespace wgt {

using namespace wgd;

#ifndef WG_TW
#define WG_TW 4
#endif
constexpr uint32_t TW = WG_TW;      // waves per workgroup
constexpr uint32_t LPT_BINS = 130;  // round counts 0..129 (65535-B payload = 1025 blocks = 129 rounds)

// AllowedIPs tables of the receive side (wg_rx.hip) as the open kernel reads them when
// wg_open_batch is called with WG_F_RX_FILTER: one struct in device memory, rebuilt whenever a
// filter or the slot -> filter map changes.
constexpr uint32_t kNoFilter = 0xFFFFFFFFu;
struct RxTables {
  const uint32_t* slot_filter;  // per key slot: filter id or kNoFilter (NULL: no map set)
  const uint32_t* hdr;          // per filter: root4, root6 (global node indices)
  const uint32_t* entries;      // nodes x 256 entries: next node | bit 31 "a prefix ended in this byte"
  uint32_t nfilters;
  uint32_t key_slots;
};

// TransportManager.processDecryptedTransport for one opened packet whose tag verified
// (TransportManager.java:98-119): a keepalive (len 0, :103-105), an address family that is not
// IPv4/IPv6 or a packet too short for the destination (destinationIPOf, :124-130, throws), or a
// destination outside the key slot's AllowedIPs (IPFilter.search, util/IPFilter.java:49-61).
// p: the plaintext (global memory, this launch's output). Shared by k_rx_filter and the fused
// open (WG_F_RX_FILTER).
__device__ inline uint32_t rx_verdict(const RxTables& T, const uint8_t* p, uint32_t len, uint32_t key_slot) {
  if (len == 0) return WG_PKT_KEEPALIVE;
  const uint32_t ver = p[0] >> 4;
  uint32_t nbytes, at;
  if (ver == 4) {
    nbytes = 4;
    at = 16;
  } else if (ver == 6) {
    nbytes = 16;
    at = 24;
  } else {
    return WG_PKT_BADIP;
  }
  if (len < at + nbytes) return WG_PKT_BADIP;
  if (!T.slot_filter || key_slot >= T.key_slots) return WG_PKT_OK;
  const uint32_t f = T.slot_filter[key_slot];
  if (f == kNoFilter) return WG_PKT_OK;
  uint32_t node = f < T.nfilters ? T.hdr[2 * f + (ver == 6 ? 1 : 0)] : 0u;  // never set: empty filter
  bool found = false;
  for (uint32_t L = 0; L < nbytes && node; ++L) {
    const uint32_t e = T.entries[(size_t)node * 256 + p[at + L]];
    found |= (e >> 31) != 0;
    node = e & 0x7FFFFFFFu;
  }
  return found ? WG_PKT_OK : WG_PKT_FILTERED;
}

struct TransportParams {
  const wg_pkt* desc;
  const uint32_t* order;  // batch position -> packet index (longest first); nullptr = identity
  uint32_t n;
  uint32_t slots;         // S = (64 / G) x waves in the grid
  uint32_t max_len;
  uint32_t key_slots;
  const uint8_t* in;
  uint64_t in_size;
  uint8_t* out;
  uint64_t out_size;
  const uint32_t* keys;   // device key table, 8 words per slot
  uint32_t* status;       // open: per-packet WG_PKT_*
  uint32_t prio_step;     // rounds per issue-priority level (0: no priority changes)
  const RxTables* rx;     // open with WG_F_RX_FILTER: receive-side verdict in the status (else NULL)
  const uint32_t* n_long; // k_*_mixed: device count of the packets at the front of the order that take
                          // 16-lane slots (written by k_lpt_scatter); NULL otherwise. With bin_cnt (one-launch
                          // planning, k_lpt_one) it only marks the launch as mixed.
  // one-launch planning (k_lpt_one, batches of max_len <= 2048): the longest-first order is SPARSE, key k's
  // packets at order[k * bin_cap ...], bin_cnt[k] of them; the kernel reads the counts into bc (mixed_part)
  // and maps a batch position to its packet through them (pkt_at). pos_base: the position of this part's
  // first packet in the whole order (the short part starts after the long one). split: keys > split are long.
  const uint32_t* bin_cnt;
  uint32_t bin_cap;
  uint32_t pos_base;
  uint32_t split;
  uint32_t split2;  // k_step_mixed with GT = 2: keys <= split2 (> 0) take 2-lane slots, after the GS-lane part
  // dynamic claims (k_step_claim, mixed-length batches): the longest-first order is dealt
  // as claim_nc interleaved sub-orders (positions c, c + nc, c + 2 nc, ...), sub-order c to the workgroups
  // b with b % nc == c; each slot starts on a static position and claims every later one from its
  // sub-order's counter (claim[16 c], one 64-B line each, reset to claim_base by k_lpt_scatter), so a
  // slot that finishes early takes the next-longest packet instead of a fixed one
  uint32_t* claim;
  uint32_t claim_nc;      // a power of two dividing the grid
  uint32_t claim_base;    // slots per sub-order = the counters' initial value
  uint2* chain_out;       // seal half of k_step_claim: per position {next position, next packet} of its slot
  const uint2* chain_in;  // open half: the same chain, replayed (slot g opens exactly what it sealed)
  // 4-lane slots, one packet per slot (plan_transport): waves in one workgroup generation (workgroups
  // per CU x CUs x waves per workgroup); every odd generation takes its longest-first positions in
  // reverse, so the waves that share a SIMD get long and short packets in turn (0: no reversal)
  uint32_t wave_gen;
#ifdef WG_DIAG
  uint64_t* stamps;       // diagnostic build only: 10 x u64 per wave (cycles per phase, start/end times)
#endif
};

// Per-wave phase accounting, compiled only into the diagnostic library (make diag):
// cycles spent in each phase of the round loop, summed over the wave's rounds.
#ifdef WG_DIAG
#define WG_PH_DECL uint64_t ph_[7] = {0, 0, 0, 0, 0, 0, 0}; uint64_t ph_t = __builtin_amdgcn_s_memtime(); \
  const uint64_t ph_r0 = __builtin_amdgcn_s_memrealtime(); (void)ph_r0;
#define WG_PH(k) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); ph_[k] += n_ - ph_t; ph_t = n_; } while (0)
#define WG_PH_STORE(idx)                                                                       \
  do {                                                                                         \
    if (P.stamps && (threadIdx.x & 63u) == 0) {                                                \
      uint64_t* o_ = P.stamps + (size_t)(idx) * 10;                                            \
      for (int k_ = 0; k_ < 7; ++k_) o_[k_] = ph_[k_];                                         \
      o_[8] = ph_r0;                                                                           \
      o_[9] = __builtin_amdgcn_s_memrealtime();                                                \
    }                                                                                          \
  } while (0)
#elif defined(WG_MARKS)  // asm comments at the phase boundaries (tools/isa_phases.py)
#define WG_PH_DECL
#define WG_PH(k) asm volatile(";; WGMARK " #k)
#define WG_PH_STORE(idx) do {} while (0)
#else
#define WG_PH_DECL
#define WG_PH(k) do {} while (0)
#define WG_PH_STORE(idx) do {} while (0)
#endif

// ---- lane exchange inside a slot of G lanes (G = 4, 8 or 16) ------------------------
// ds_swizzle bitmask mode inside each 32-lane half: src = ((lane & and) | or) ^ xor.
template <int G, int K>
__device__ __forceinline__ uint32_t bcastg(uint32_t v) {  // every lane of the slot reads lane K of it
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "slots of 2, 4, 8 or 16 lanes");
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (0x20 - G) | (K << 5));
}
template <int K>
__device__ __forceinline__ uint32_t bcast8(uint32_t v) { return bcastg<8, K>(v); }
template <int X>
__device__ __forceinline__ uint32_t xorg(uint32_t v) {  // lane reads lane ^ X (X < 16)
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1f | (X << 10));
}

// A slot's copy of one 32-B descriptor (wg_pkt = 8 dwords): with 8 or 16 lanes, lane j holds dword j & 7
// (w.x); with 4 lanes, lane j holds dwords 2j and 2j + 1 (w.x, w.y: one 8-B load, desc_load4); with 2 lanes,
// dwords 4j .. 4j + 3 (one 16-B load, desc_load2). desc_word<G, K> gives every lane of the slot dword K.
__device__ __forceinline__ uint2 desc_load4(const wg_pkt* d, uint32_t i, uint32_t j) {
  return i != ~0u ? ((const uint2*)(d + i))[j & 3u] : make_uint2(0u, 0u);
}
__device__ __forceinline__ uint4 desc_load2(const wg_pkt* d, uint32_t i, uint32_t j) {
  return i != ~0u ? ((const uint4*)(d + i))[j & 1u] : make_uint4(0u, 0u, 0u, 0u);
}
template <int G, int K>
__device__ __forceinline__ uint32_t desc_word(const uint4& w) {
  if constexpr (G == 2) return bcastg<2, K / 4>((K & 3) == 0 ? w.x : (K & 3) == 1 ? w.y : (K & 3) == 2 ? w.z : w.w);
  else if constexpr (G == 4) return bcastg<4, K / 2>((K & 1) ? w.y : w.x);
  else return bcastg<G, K>(w.x);
}

// The same exchanges through DPP (VALU, no LDS round trip) for the dependent chains of the
// r-power scan and the slot sum: row_shr:K (lane j reads j - K inside its 16-lane row; lanes j < K
// of a slot get garbage and must not use it), lane ^ 1, lane ^ 2 (quad_perm), lane ^ 4 (two half
// moves) and lane ^ 8 (row_ror:8, 16-lane slots).
template <int K>
__device__ __forceinline__ uint32_t shr_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 | K, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t xor1_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t xor2_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ uint32_t xor4_dpp(uint32_t v) {
  // lanes 4-7 of a slot (banks 1, 3) read j - 4 (row_shr:4), lanes 0-3 (banks 0, 2) read j + 4 (row_shl:4)
  const int t = __builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xa, false);
  return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x104, 0xf, 0x5, false);
}
__device__ __forceinline__ uint32_t xor8_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
}

// slot-record flags beyond valid / alignment (SlotRec.meta.w): an open whose plaintext range
// overlaps its ciphertext || tag range verifies first (no stores) and decrypts in a second pass
constexpr uint32_t kVerifyFirst = 16u, kDecryptPass = 32u;

// ---- validity of one transport descriptor (shared by seal, open and the framing) ----
template <int MODE>
__device__ __forceinline__ bool transport_valid(uint64_t in_off, uint64_t out_off, uint32_t len, uint32_t ks,
                                                uint32_t max_len, uint32_t key_slots, uint64_t in_size,
                                                uint64_t out_size) {
  const uint64_t in_need = (uint64_t)len + (MODE == WG_MODE_OPEN ? 16u : 0u);
  const uint64_t out_need = (uint64_t)len + (MODE == WG_MODE_SEAL ? 16u : 0u);
  return len <= max_len && ks < key_slots && in_off <= in_size && in_need <= in_size - in_off &&
         out_off <= out_size && out_need <= out_size - out_off;
}

// 16 bytes at p (any alignment), `avail` (1..16) of them inside the packet: the aligned dwords
// covering them (none leaves the granule of a valid byte), realigned with v_alignbyte
__device__ __forceinline__ uint4 chunk_any(const uint8_t* p, uint32_t avail) {
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
  const uint32_t* q = (const uint32_t*)(p - sh);
  const uint32_t nw = (sh + avail + 3u) >> 2;
  uint32_t W[5];
#pragma unroll
  for (uint32_t k = 0; k < 5; ++k) W[k] = k < nw ? q[k] : 0u;
  return make_uint4(__builtin_amdgcn_alignbyte(W[1], W[0], sh), __builtin_amdgcn_alignbyte(W[2], W[1], sh),
                    __builtin_amdgcn_alignbyte(W[3], W[2], sh), __builtin_amdgcn_alignbyte(W[4], W[3], sh));
}

// bytes >= cb (1..15) of a 16-B chunk zeroed: dword k keeps clamp(8 cb - 32 k, 0, 32) low bits
__device__ __forceinline__ uint4 mask_chunk(uint4 v, uint32_t cb) {
  int c8 = (int)(8u * cb);
  asm volatile("" : "+v"(c8));  // keep the mask arithmetic in the (rare) partial-chunk path
  uint32_t t[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] &= ~(uint32_t)(~0ull << min(max(c8 - 32 * k, 0), 32));
  return make_uint4(t[0], t[1], t[2], t[3]);
}

// cb (1..16) bytes of a chunk to p: oal bit 2 = p 16-B aligned, bit 3 = p 4-B aligned
__device__ __forceinline__ void store_chunk(uint8_t* p, uint32_t cb, uint4 o, uint32_t oal) {
  if (cb == 16u && (oal & 4u)) {
    *(uint4*)p = o;
    return;
  }
  const uint32_t t[4] = {o.x, o.y, o.z, o.w};
  if (oal & 8u) {
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const int r = (int)cb - 4 * (int)k;
      if (r >= 4) {
        ((uint32_t*)p)[k] = t[k];
      } else if (r > 0) {
        uint8_t* q = p + 4u * k;
        q[0] = (uint8_t)t[k];
        if (r > 1) q[1] = (uint8_t)(t[k] >> 8);
        if (r > 2) q[2] = (uint8_t)(t[k] >> 16);
      }
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < 16u; ++i)
      if (i < cb) p[i] = (uint8_t)(t[i >> 2] >> (8u * (i & 3u)));
  }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;

__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* p) {
  if ((((uintptr_t)p) & 3u) == 0) return *(const uint32_t*)p;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ void store_u32_any(uint8_t* p, uint32_t v) {
  if ((((uintptr_t)p) & 3u) == 0) {
    *(uint32_t*)p = v;
    return;
  }
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// orders this wave's LDS writes before its other lanes' reads
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t batch_pos(uint32_t g, uint32_t k, uint32_t S) {
  return k * S + ((k & 1u) ? S - 1u - g : g);
}

#define WG_CONST __attribute__((address_space(4)))  // constant address space: scalar loads

// batch position -> packet index: the identity, the dense longest-first order, or the sparse one of k_lpt_one
// (keys descending, key k's packets at order[k * bin_cap + i])
constexpr uint32_t kFastBins = 6;  // keys 0..5: every packet of at most 2,048 B (33 blocks, 5 rounds of 8)
// the same one-launch plan for other mixed batches whose keys fit 32 bins (max_len <= 15,808 B: C2's 9,000-B
// packets are key 18), read by k_step<8, 4, ..., kWideBins>
constexpr uint32_t kWideBins = 32;
// k_lpt_one's per-key counters, kCntStride words apart (every planner workgroup adds to each once). 16 (a
// 64-B line each) measured the same as 1: the planner's 5.1 us is not atomic contention
// (profiles/r06_cnt_stride_ab.jsonl)
#ifndef WG_CNT_STRIDE
#define WG_CNT_STRIDE 1
#endif
constexpr uint32_t kCntStride = WG_CNT_STRIDE;
template <int MX>  // MX: bins of the sparse order (kFastBins for the short-packet plan, kWideBins), 0: dense
__device__ __forceinline__ uint32_t pkt_at(const TransportParams& P, uint32_t pos) {
  if (MX && P.bin_cap) {
    // the counts through the scalar cache (constant for the launch), not held in SGPRs across the body
    // (branch-free: the position's key region and its offset in it, one select per key)
    const WG_CONST uint32_t* bc = (const WG_CONST uint32_t*)P.bin_cnt;
    const uint32_t p = P.pos_base + pos;
    uint32_t start = 0, at = 0;
#pragma unroll
    for (int k = MX - 1; k >= 0; --k) {
      const uint32_t c = bc[k * kCntStride];
      at = (p >= start) ? (uint32_t)k * P.bin_cap + (p - start) : at;
      start += c;
    }
    return P.order[at];
  }
  return P.order ? P.order[pos] : pos;
}

// ---- the kernel ------------------------------------------------------------------------
// Register budget: <= 64 VGPRs, so 8 waves share a SIMD (the payload stream and the ARX
// rounds of other waves hide each other's latency). What is constant for a packet lives
// in a 128-B LDS record per slot and is re-read where it is used; lane-derived values are
// recomputed from an opaque copy of the lane id instead of being held across the rounds.
struct SlotRec {  // per slot, in LDS
  uint4 addr;     // {in_off lo, in_off hi, out_off lo, out_off hi} (pointers are rebuilt from the kernel
                  // arguments, so the compiler keeps global, not flat, memory instructions)
  uint4 meta;     // {ctr lo, ctr hi, len, flags}: bit 0 valid, bit 1 input / bit 2 output 16-B aligned,
                  // bit 3 output 4-B aligned
  uint4 R0;       // R = r^8 limbs 0..3
  uint4 R1;       // {R4, 5 R1, 5 R2, 5 R3}
  uint4 R2;       // {5 R4, -, -, -}
  uint4 s;        // Poly1305 s
  uint4 key[2];   // ChaCha20 key
};
static_assert(sizeof(SlotRec) == 128, "slot record is 128 B");


__device__ __forceinline__ uint32_t opaque_lane() {
  uint32_t x = threadIdx.x & 63u;
  asm volatile("" : "+v"(x));
  return x;
}

// The per-wave body of k_transport (and of each half of k_duplex / k_step): workgroup `blk` of the
// direction's grid; img / rec are this wave's 4-KB image and slot records in LDS. G = lanes per
// slot: 8 (8 slots per wave, rounds of 8 blocks) or 16 (4 slots, rounds of 16 blocks = 1 KB:
// long packets take half as many rounds, so a mixed-length batch can pair them longest-first at
// 8 waves per SIMD).
// iter: rounds this wave has run so far in the launch (the issue-priority schedule spans both
// halves of a k_step launch).
// Where a slot's packets come from (PM): kPosStatic, the snake over the grid (batch_pos); kPosClaim, a
// static first position, then claims from the slot's sub-order counter, logged in P.chain_out when set;
// kPosChain, the positions a kPosClaim seal half logged, in the same order.
constexpr int kPosStatic = 0, kPosClaim = 1, kPosChain = 2;

// ST (stitched Horner): a round's Horner steps run in the NEXT round of the packet, interleaved
// into the first kStitchDR double rounds of its ChaCha20 block (wg_stitch.h); the next round's payload DMA is
// issued after them, so the image still holds the round's MAC input while they read it. A packet's last
// round takes its Horner steps after its XOR phase as before (nothing follows it to hide them in).
// MX: the launch is a k_*_mixed part (its positions may map through k_lpt_one's sparse order)
template <int MODE, int G = 8, bool VF = false, int PM = kPosStatic, bool ST = false, int MX = 0>
__device__ __forceinline__ void transport_body(const TransportParams& P, uint32_t blk, uint32_t wv, uint4* const img,
                                               SlotRec* const rec, uint32_t& iter) {
  static_assert(MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN, "transport modes only");
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "slots of 2, 4, 8 or 16 lanes");
  static_assert(G != 2 || (MX && !VF && !ST), "2-lane slots: the short-packet split plan's tiny packets only");
#ifdef WG_HORNER2
  static_assert(G != 2, "the two-chunk Horner assumes G >= 4");
#endif
  static_assert(!VF || MODE == WG_MODE_OPEN, "verify-first is an open variant");
  static_assert(!(ST && VF), "the verify-first open keeps the sequential Horner");
  constexpr uint32_t SH = G == 2 ? 1u : G == 4 ? 2u : G == 8 ? 3u : 4u;  // log2 G
  constexpr uint32_t JM = G - 1u;
  // a slot's record (SlotRec); 2-lane slots keep an 80-B one, so 32 of them per wave leave the launch at 6
  // workgroups per CU: no key (read from the key table each round, the slot's key index in meta.w >> 8), no
  // 5 R limbs (formed where used), s = {R1.y, R1.z, R1.w, R2.x} beside R4 = R1.x
  constexpr uint32_t kRecStride = G == 2 ? 80u : (uint32_t)sizeof(SlotRec);
  auto RS = [rec](uint32_t si) -> SlotRec& { return *(SlotRec*)((char*)rec + si * kRecStride); };
  if (P.prio_step && iter == 0) __builtin_amdgcn_s_setprio(3);  // first instruction: a fresh wave is never starved
  const uint32_t S = P.slots;
  uint32_t wg = blk * TW + wv;  // this wave's index in the grid
  if constexpr (G == 4) {
    if (P.wave_gen) {  // odd generations reversed (a bijection: the last, partial one over its own size)
      const uint32_t k = wg / P.wave_gen, i = wg - k * P.wave_gen;
      const uint32_t size = min(P.wave_gen, gridDim.x * TW - k * P.wave_gen);
      if (k & 1u) wg = k * P.wave_gen + (size - 1u - i);
    }
  }
  const uint32_t g = wg * (64u / G) + (opaque_lane() >> SH);

  // descriptor prefetch: the next packet's wg_pkt spread over the slot's lanes (desc_load)
  uint32_t gen = 0;
  uint32_t nxt;
  // kPosClaim / kPosChain: the sub-order of this workgroup and the positions of the next / current packet
  const uint32_t csub = PM != kPosStatic ? blk & (P.claim_nc - 1u) : 0u;
  uint32_t npos = 0, cpos = 0;
  {
    uint32_t pos;
    if constexpr (PM == kPosStatic) {
      pos = batch_pos(g, 0, S);
    } else {  // slot index inside the sub-order's workgroups, then the sub-order's position of it
      const uint32_t gl = (blk / P.claim_nc) * (TW * (64u / G)) + (g - blk * TW * (64u / G));
      pos = csub + P.claim_nc * gl;
    }
    npos = pos;
    nxt = pos < P.n ? pkt_at<MX>(P, pos) : ~0u;
  }
  uint4 dn = make_uint4(0u, 0u, 0u, 0u);  // this lane's part of the next descriptor (desc_word)
  if constexpr (G == 2) {
    dn = desc_load2(P.desc, nxt, opaque_lane());
  } else if constexpr (G == 4) {
    const uint2 w = desc_load4(P.desc, nxt, opaque_lane());
    dn.x = w.x;
    dn.y = w.y;
  } else {
    dn.x = nxt != ~0u ? ((const uint32_t*)(P.desc + nxt))[opaque_lane() & 7u] : 0u;
  }

  bool have = false;
  uint32_t pkt = 0, round = 0;
  uint32_t acc[5], W[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = W[i] = 0;

  // lane j of a slot holds the packet's first-round column (j & 3) (a, b, c, d); lanes 1..3
  // feed the other lanes' blocks through ds_swizzle broadcasts
  uint32_t hc[4] = {0u, 0u, 0u, 0u};
  // Progress-based issue priority (mixed-length batches; prio_step = 0 for uniform ones): a SIMD
  // arbitrates VALU issue by priority, then age, so with equal priorities the oldest of its 8
  // waves runs ahead and the waves finish one after another. A wave drops one priority level
  // every prio_step rounds instead, so the waves that have done the least work issue first
  // (C2 +2%, C1 -2%: DESIGN.md §4.2).
  WG_PH_DECL
  while (true) {
    if (P.prio_step) {
      const uint32_t lvl = iter / P.prio_step;
      if (iter % P.prio_step == 0 && lvl <= 3u && lvl > 0u) {
        if (lvl == 1) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      ++iter;
    }
    // ---- slots without a packet take their next one ------------------------------------
    if (!have && nxt != ~0u) {
      const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
      pkt = nxt;
#ifdef WG_DIAG
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(dn.x), "+v"(dn.y), "+v"(dn.z), "+v"(dn.w));
      WG_PH(6);
#endif
      const uint32_t d0 = desc_word<G, 0>(dn), d1 = desc_word<G, 1>(dn), d2 = desc_word<G, 2>(dn),
                     d3 = desc_word<G, 3>(dn);
      const uint32_t len = desc_word<G, 6>(dn), ks = desc_word<G, 7>(dn);
      const uint64_t in_off = (uint64_t)d0 | ((uint64_t)d1 << 32);
      const uint64_t out_off = (uint64_t)d2 | ((uint64_t)d3 << 32);
      const bool valid =
          transport_valid<MODE>(in_off, out_off, len, ks, P.max_len, P.key_slots, P.in_size, P.out_size);
      const uintptr_t ia = (uintptr_t)(P.in + in_off), oa = (uintptr_t)(P.out + out_off);
      uint32_t al = ((ia & 15u) == 0 ? 2u : 0u) | ((oa & 15u) == 0 ? 4u : 0u) | ((oa & 3u) == 0 ? 8u : 0u);
      // open with the plaintext range overlapping the ciphertext || tag range (in place): verify the
      // tag first and decrypt in a second pass, so a forged packet's bytes stay as they were
      // (ChaCha20Poly1305.java:40-56 verifies before it decrypts)
      if (VF && valid && len && ia < oa + len && oa < ia + len + 16u) al |= kVerifyFirst;
      // The session key. Vector loads come back in order through the CU's L1, so at a launch's
      // start a key load would queue behind the payload DMA of every wave already running on
      // the CU; when every slot of the wave uses one key (one session per wave: C1, C3) it comes
      // through the scalar cache instead, which no payload traffic passes.
      const uint32_t ks0 = __builtin_amdgcn_readfirstlane(ks);
      if (!__any(valid && ks != ks0) && ks0 < P.key_slots) {
        const WG_CONST uint32_t* kp = (const WG_CONST uint32_t*)P.keys + 8u * ks0;
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          k[i] = kp[i];  // s_load_dwordx8
#ifndef WG_NO_SKEY
          asm volatile("" : "+s"(k[i]));  // keep it scalar (no per-lane reload)
#endif
        }
        uint32_t v = k[0];
#pragma unroll
        for (uint32_t i = 1; i < 8u; ++i) v = j == i ? k[i] : v;
        if constexpr (G == 2) {  // 2 lanes: no key in the record
        } else if constexpr (G == 4) {  // 4 lanes: key words j and j + 4
          uint32_t v2 = k[4];
#pragma unroll
          for (uint32_t i = 1; i < 4u; ++i) v2 = j == i ? k[4u + i] : v2;
          if (valid) {
            ((uint32_t*)RS(s).key)[j] = v;
            ((uint32_t*)RS(s).key)[j + 4u] = v2;
          }
        } else if (valid && j < 8u) {
          ((uint32_t*)RS(s).key)[j] = v;
        }
      } else if (G == 2) {
      } else if (valid && G == 4) {
        ((uint32_t*)RS(s).key)[j] = P.keys[8u * ks + j];
        ((uint32_t*)RS(s).key)[j + 4u] = P.keys[8u * ks + j + 4u];
      } else if (valid && j < 8u) {
        ((uint32_t*)RS(s).key)[j] = P.keys[8u * ks + j];
      }
      // all lanes active: swizzles read live lanes
      const uint32_t c0 = desc_word<G, 4>(dn), c1 = desc_word<G, 5>(dn);
      if (j == 0) {
        RS(s).addr = make_uint4(d0, d1, d2, d3);
        RS(s).meta = make_uint4(c0, c1, len, (valid ? 1u : 0u) | al | (G == 2 && valid ? ks << 8 : 0u));
      }
      round = 0;
      have = true;
      // prefetch the descriptor of the slot's following packet
      ++gen;
      if constexpr (PM == kPosStatic) {
        const uint32_t pos = batch_pos(g, gen, S);
        nxt = pos < P.n ? pkt_at<MX>(P, pos) : ~0u;
      } else if constexpr (PM == kPosClaim) {
        cpos = npos;
        uint32_t k = 0;
        if (j == 0) k = atomicAdd(P.claim + 16u * csub, 1u);
        const uint32_t pos = csub + P.claim_nc * bcastg<G, 0>(k);
        nxt = pos < P.n ? (P.order ? P.order[pos] : pos) : ~0u;
        npos = nxt != ~0u ? pos : ~0u;
        if (P.chain_out && j == 0) P.chain_out[cpos] = make_uint2(npos, nxt);
      } else {  // kPosChain
        cpos = npos;
        const uint2 cn = P.chain_in[cpos];  // every lane of the slot reads the same 8 B
        npos = cn.x;
        nxt = cn.y;
      }
      if constexpr (G == 2) {
        dn = desc_load2(P.desc, nxt, j);
      } else if constexpr (G == 4) {
        const uint2 w = desc_load4(P.desc, nxt, j);
        dn.x = w.x;
        dn.y = w.y;
      } else {
        dn.x = nxt != ~0u ? ((const uint32_t*)(P.desc + nxt))[j & 7u] : 0u;
      }
    }
    if (!__any(have)) break;
    wave_lds_sync();  // the slot records before the lanes read them
    WG_PH(0);

    // this round's packet parameters, read once (meta = {ctr lo, ctr hi, len, flags})
    const uint4 meta = RS(opaque_lane() >> SH).meta;
    const uint32_t len = meta.z;
    const uint32_t nb = (meta.w & 1u) ? ((len + 63u) >> 6) + 1u : 0u;
    // ST: slots whose previous round (not their packet's last) still owes its Horner steps
    const bool pend = ST && have && round > 0u && (meta.w & 1u);
    const bool stitch = ST && __any(pend);
    uint32_t x[16];
    {
      // ---- payload prefetch: LDS-DMA straight into this lane's slice of the image ---------
      // (no registers held across the ARX rounds; with stitched Horner steps pending, after them)
      const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
      const uint32_t b = G * round + j;
      auto payload_dma = [&]() {
      if (have && b < nb && b > 0u) {
        const uint32_t off = 64u * (b - 1u);
        const uint32_t nbytes = min(64u, len - off);
        const uint4 ad = RS(s).addr;
        const uint8_t* src = P.in + (((uint64_t)ad.x | ((uint64_t)ad.y << 32)) + off);
        if (meta.w & 2u) {
          // chunks holding a valid byte, each read whole (an aligned 16-B read stays in the granule
          // of its first byte); lane i's chunk q lands at img[q * 64 + i]
          __builtin_amdgcn_global_load_lds((gbl_cvoid*)src, (lds_void*)&img[0], 16, 0, 0);
          if (nbytes > 16u) __builtin_amdgcn_global_load_lds((gbl_cvoid*)(src + 16), (lds_void*)&img[64], 16, 0, 0);
          if (nbytes > 32u) __builtin_amdgcn_global_load_lds((gbl_cvoid*)(src + 32), (lds_void*)&img[128], 16, 0, 0);
          if (nbytes > 48u) __builtin_amdgcn_global_load_lds((gbl_cvoid*)(src + 48), (lds_void*)&img[192], 16, 0, 0);
        } else {  // unaligned input: the same image, staged through registers one chunk at a time
#pragma unroll
          for (uint32_t q = 0; q < 4u; ++q)
            if (16u * q < nbytes) img[64u * q + lane] = chunk_any(src + 16u * q, min(16u, nbytes - 16u * q));
        }
      }
      };
      if (!stitch) payload_dma();
      // ---- ChaCha20: block b = 8 round + j ----------------------------------------------
      if (G > 2 && __any(have && round == 0)) {  // a new packet: its columns 1..3 of the first round, once
        const uint32_t c = j & 3u;
        const uint4* kl = RS(s).key;
        const uint4 ka = kl[0], kb = kl[1];
        uint32_t a = c == 1u ? 0x3320646eu : c == 2u ? 0x79622d32u : 0x6b206574u;
        uint32_t bb = c == 1u ? ka.y : c == 2u ? ka.z : ka.w;
        uint32_t cc = c == 1u ? kb.y : c == 2u ? kb.z : kb.w;
        uint32_t d = c == 1u ? meta.x : c == 2u ? meta.y : 0u;
        chacha20_qr(a, bb, cc, d);
        if (have && round == 0) {
          hc[0] = a; hc[1] = bb; hc[2] = cc; hc[3] = d;
        }
      }
      if constexpr (G == 2) {  // no lanes 1..3 to hold the hoisted columns: the whole block
        // (every lane computes a block, also one whose slot has no packet and whose record is stale: its key
        // index is 0 then, and any index is clamped to the table)
        const uint32_t kidx = have ? min(meta.w >> 8, P.key_slots - 1u) : 0u;
        chacha20_block_full((const uint4*)(P.keys + 8u * kidx), b, meta.x, meta.y, 0u, x);
      } else {
        const uint32_t H[12] = {bcastg<G, 1>(hc[0]), bcastg<G, 1>(hc[1]), bcastg<G, 1>(hc[2]), bcastg<G, 1>(hc[3]),
                                bcastg<G, 2>(hc[0]), bcastg<G, 2>(hc[1]), bcastg<G, 2>(hc[2]), bcastg<G, 2>(hc[3]),
                                bcastg<G, 3>(hc[0]), bcastg<G, 3>(hc[1]), bcastg<G, 3>(hc[2]), bcastg<G, 3>(hc[3])};
        if constexpr (!ST) {
          chacha20_block_hoisted(RS(s).key, b, meta.x, meta.y, 0u, H, x);
        } else {
          // the same block in two parts: the first kStitchDR double rounds (with the pending Horner steps of the
          // previous round when any slot has them), then the payload DMA, then the rest and the feed-forward
          const uint4* kl = RS(s).key;
          uint4 ka = kl[0], kb = kl[1];
          x[0] = 0x61707865u; x[1] = H[0]; x[2] = H[4]; x[3] = H[8];
          x[4] = ka.x; x[5] = H[1]; x[6] = H[5]; x[7] = H[9];
          x[8] = kb.x; x[9] = H[2]; x[10] = H[6]; x[11] = H[10];
          x[12] = b; x[13] = H[3]; x[14] = H[7]; x[15] = H[11];
          if (stitch) {
            // the previous round kp's window: chunks [4 G kp - 4, 4 G kp + 4 G - 4) (round 0's first four are the
            // zeroed key-block lane, so every lane takes exactly four steps); lane j's chunks c0 + G t sit in one
            // image row (c0 & 3), G / 4 lanes apart. Lanes without a pending round compute on a clamped address
            // and their accumulator is not used (a new packet resets it in its round 0 scan).
            const uint32_t kp = round - 1u;
            const uint32_t nc = (len + 15u) >> 4, M = nc + 1u, Dp = G * ((M + JM) >> SH) - M;
            const uint32_t u = 4u * G * kp + ((j - ((4u * G * kp - 4u + Dp) & JM)) & JM);  // c0 + 4
            const uint32_t lanepart = ((u >> 2) - G * kp) & (G / 4u - 1u);
            const uint32_t addr = (uint32_t)(uintptr_t)&img[64u * (u & 3u) + (lane & ~JM) + lanepart];
            const uint4 q0 = RS(s).R0, q1 = RS(s).R1, q2 = RS(s).R2;
            const uint32_t R[5] = {q0.x, q0.y, q0.z, q0.w, q1.x};
            const uint32_t Rs[4] = {q1.y, q1.z, q1.w, q2.x};
            // a lane whose first chunk of round 0's window lies before the data (u < 4: chunks -4..-1) adds it
            // without the 2^128 bit, so the zeroed chunk adds nothing to its still-zero accumulator
            const uint32_t hib0 = (kp == 0u && u < 4u) ? 0u : (1u << 24);
            chacha20_rounds_stitch_asm<G>(x, acc, R, Rs, addr, hib0);
            payload_dma();
          } else {
            chacha20_rounds_head_asm(x);
          }
          chacha20_rounds_tail_asm(x);
          asm volatile("" ::: "memory");
          ka = kl[0];
          kb = kl[1];
          x[0] += 0x61707865u; x[1] += 0x3320646eu; x[2] += 0x79622d32u; x[3] += 0x6b206574u;
          x[4] += ka.x; x[5] += ka.y; x[6] += ka.z; x[7] += ka.w;
          x[8] += kb.x; x[9] += kb.y; x[10] += kb.z; x[11] += kb.w;
          x[12] += b; x[13] += meta.x; x[14] += meta.y;
        }
      }
    }

    const bool mac_pass = !VF || !(meta.w & kDecryptPass);  // the second pass of a verify-first open only decrypts
    if (__any(have && round == 0 && mac_pass)) {  // round 0: lane 0 of the slot holds the one-time key r || s
      const uint32_t lane = opaque_lane(), s = lane >> SH;
      if (have && round == 0 && mac_pass && (lane & JM) == 0) {
        RS(s).R0 = make_uint4(x[0], x[1], x[2], x[3]);  // raw r, replaced by R = r^8 below
        if constexpr (G == 2) {
          RS(s).R1 = make_uint4(0u, x[4], x[5], x[6]);
          RS(s).R2.x = x[7];
        } else {
          RS(s).s = make_uint4(x[4], x[5], x[6], x[7]);
        }
      }
    }

    WG_PH(1);
    // ---- XOR, store, MAC input into the image, one 16-B chunk at a time ----------------------
    {
      const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
      const uint32_t b = G * round + j;
      if (have && b < nb && b > 0u) {
        const uint32_t off = 64u * (b - 1u);
        const uint32_t nbytes = min(64u, len - off);
        const uint4 ad = RS(s).addr;
        uint8_t* dst = P.out + (((uint64_t)ad.z | ((uint64_t)ad.w << 32)) + off);
        const uint32_t oal = meta.w & 12u;  // bit 2: 16-B aligned output, bit 3: 4-B aligned
        // the payload DMA (and the staged loads) must have landed in LDS: the compiler does not
        // always see the LDS-DMA -> ds_read dependence, so wait for it explicitly
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          if (16u * q < nbytes) {
            const uint32_t cb = min(16u, nbytes - 16u * q);  // valid bytes in this chunk
            uint4 v = img[64u * q + lane];  // payload (the compiler waits for the DMA before this read)
            // open: the MAC input is the zero-padded ciphertext; seal masks the ciphertext below instead
            if (MODE == WG_MODE_OPEN && cb < 16u) v = mask_chunk(v, cb);
            if constexpr (MODE == WG_MODE_OPEN) {
              if (cb < 16u) img[64u * q + lane] = v;  // the MAC input is the zero-padded ciphertext
            }
            uint4 o = make_uint4(x[4 * q] ^ v.x, x[4 * q + 1] ^ v.y, x[4 * q + 2] ^ v.z, x[4 * q + 3] ^ v.w);
            if constexpr (MODE == WG_MODE_SEAL) {
              if (cb < 16u) o = mask_chunk(o, cb);
              img[64u * q + lane] = o;  // the MAC input is the ciphertext
            }
            if (!VF || (meta.w & (kVerifyFirst | kDecryptPass)) != kVerifyFirst)
              store_chunk(dst + 16u * q, cb, o, oal);
          }
        }
      }
      // ST: the key-block lane's image slice is round 0's chunks -4..-1 of the stitched window: zero
      if (ST && have && round == 0u && j == 0u) {
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) img[64u * q + lane] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    // the length block le64(0) || le64(len) is MAC chunk nc (the first after the data): the lane
    // whose counter block holds it writes it into the image, so the Horner steps read it like data
    {
      const uint32_t lane = opaque_lane(), j = lane & JM;
      const uint32_t nc = (len + 15u) >> 4;
      if (have && (meta.w & 1u) && G * round + j == (nc >> 2) + 1u) {
        img[64u * (nc & 3u) + lane] = make_uint4(0u, 0u, len, 0u);
      }
    }
    wave_lds_sync();
    WG_PH(2);

    // ---- round 0: r^1..r^G (lane j gets r^(j+1)), R = r^G, W = r^(G-j) --------------------
    // (after the XOR phase, so the 32 registers of keystream and payload are free again)
    if (__any(have && round == 0 && mac_pass)) {
      if (have && round == 0 && mac_pass) {
        const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
        const uint4 rr = RS(s).R0;
        uint32_t y[5];
        poly_r_limbs(rr.x, rr.y, rr.z, rr.w, y);
#pragma unroll
        for (uint32_t st = 1; st < G; st <<= 1) {
          uint32_t z[5], zs[5];
#pragma unroll
          for (int i = 0; i < 5; ++i)
            z[i] = st == 1 ? shr_dpp<1>(y[i]) : st == 2 ? shr_dpp<2>(y[i]) : st == 4 ? shr_dpp<4>(y[i]) : shr_dpp<8>(y[i]);
          poly_scale5(z, zs);
          if (j >= st) poly_mul(y, z, zs);
        }
        uint32_t R[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          R[i] = bcastg<G, G - 1>(y[i]);
          W[i] = xorg<G - 1>(y[i]);
          acc[i] = 0;
        }
        if (j == 0) {
#ifdef WG_HORNER2
          // R and Q = R^2 (the two-chunk Horner step); their 5x forms are formed where used
          uint32_t Q[5] = {R[0], R[1], R[2], R[3], R[4]}, Rs[5];
          poly_scale5(R, Rs);
          poly_mul(Q, R, Rs);
          RS(s).R0 = make_uint4(R[0], R[1], R[2], R[3]);
          RS(s).R1 = make_uint4(R[4], Q[0], Q[1], Q[2]);
          RS(s).R2 = make_uint4(Q[3], Q[4], 0u, 0u);
#else
          RS(s).R0 = make_uint4(R[0], R[1], R[2], R[3]);
          if constexpr (G == 2) {
            RS(s).R1.x = R[4];
          } else {
            RS(s).R1 = make_uint4(R[4], 5u * R[1], 5u * R[2], 5u * R[3]);
            RS(s).R2 = make_uint4(5u * R[4], 0u, 0u, 0u);
          }
#endif
        }
      }
      wave_lds_sync();
    }

    WG_PH(3);
    // ---- Poly1305 over this round's chunks (ST: only a packet's last round; the others run stitched) -------
    if (have && (meta.w & 1u) && mac_pass && (!ST || G * (round + 1u) >= nb)) {
      const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
      {
        const uint32_t nc = (len + 15u) >> 4;
        const uint32_t M = nc + 1u, D = G * ((M + JM) >> SH) - M;
        const uint32_t c_lo = round ? 4u * G * round - 4u : 0u;
        // chunk nc (after the data) is the length block le64(0) || le64(len): taken here when it
        // falls inside this round's window, at the finish otherwise
        const uint32_t c_end = min(nc + 1u, 4u * G * round + 4u * G - 4u);
        const uint32_t c0 = c_lo + ((j - ((c_lo + D) & JM)) & JM);
        // chunk ci of the round sits in lane (ci >> 2) + 1 - G round of the slot, row ci & 3
        const uint4* ip = &img[64u * (c0 & 3u) + (lane & ~JM) + ((c0 + 4u) >> 2) - G * round];
        const uint4 q0 = RS(s).R0, q1 = RS(s).R1, q2 = RS(s).R2;
#ifdef WG_HORNER2
        // (opt-in, -DWG_HORNER2) two chunks per reduction where the round has them:
        // acc = acc R^2 + m_t R + m_(t+1). Bit-exact, but it spills 2 VGPRs in k_step<8> and ran
        // C1 1.2% slower (C2 equal) in an alternating A/B (profiles/r04_horner2_ab.txt)
        const uint32_t R[5] = {q0.x, q0.y, q0.z, q0.w, q1.x};
        const uint32_t Rs[5] = {0u, 5u * q0.y, 5u * q0.z, 5u * q0.w, 5u * q1.x};
        const uint32_t Q[5] = {q1.y, q1.z, q1.w, q2.x, q2.y};
        const uint32_t Qs[5] = {0u, 5u * q1.z, 5u * q1.w, 5u * q2.x, 5u * q2.y};
        const uint32_t nst = c0 < c_end ? min(4u, (c_end - c0 + G - 1u) / G) : 0u;  // chunks this round
#pragma unroll
        for (uint32_t t = 0; t < 4u; t += 2u) {
          if (t < nst) {
            const uint4 v = ip[(G / 4u) * t];
            uint32_t m0[5];
            poly_block_limbs(v.x, v.y, v.z, v.w, 1u << 24, m0);
            if (t + 1u < nst) {
              if (round != 0 || t != 0) {
                poly_mul2(acc, Q, Qs, m0, R, Rs);
              } else {  // a packet's first two chunks: acc = m0 R (acc is still 0)
#pragma unroll
                for (int i = 0; i < 5; ++i) acc[i] = m0[i];
                poly_mul(acc, R, Rs);
              }
              // the second chunk is read after the product (its limbs are not live across it)
              const uint4 w = ip[(G / 4u) * (t + 1u)];
              uint32_t m1[5];
              poly_block_limbs(w.x, w.y, w.z, w.w, 1u << 24, m1);
#pragma unroll
              for (int i = 0; i < 5; ++i) acc[i] += m1[i];
            } else {
              if (round != 0 || t != 0) poly_mul(acc, R, Rs);
#pragma unroll
              for (int i = 0; i < 5; ++i) acc[i] += m0[i];
            }
          }
        }
#else
        const uint32_t R[5] = {q0.x, q0.y, q0.z, q0.w, q1.x};
        const uint32_t Rs[5] = {0u, G == 2 ? 5u * q0.y : q1.y, G == 2 ? 5u * q0.z : q1.z, G == 2 ? 5u * q0.w : q1.w,
                                G == 2 ? 5u * q1.x : q2.x};
#pragma unroll
        for (uint32_t t = 0; t < 4u; ++t) {
          if (c0 + G * t < c_end) {
            // (2-lane slots: chunk c0 + 2 t alternates rows, so its place is computed per step)
            uint4 v = G == 2 ? img[64u * ((c0 + 2u * t) & 3u) + (lane & ~JM) + ((c0 + 2u * t + 4u) >> 2) - G * round]
                             : ip[(G / 4u) * t];
            // acc is still 0 before a packet's first chunk (round 0, t = 0): no product needed
            if (round != 0 || t != 0) poly_mul(acc, R, Rs);
            uint32_t cl[5];
            poly_block_limbs(v.x, v.y, v.z, v.w, 1u << 24, cl);
#pragma unroll
            for (int i = 0; i < 5; ++i) acc[i] += cl[i];
          }
        }
#endif
      }
    }

    WG_PH(4);
    // ---- finish the packets whose last round this was ---------------------------------------
    const bool done = have && G * (round + 1u) >= nb;  // invalid packets (nb = 0) finish at once
    if (__any(done)) {
      if (done) {  // slot-uniform: every lane of a finishing slot is here
        const uint32_t lane = opaque_lane(), s = lane >> SH, j = lane & JM;
        const bool valid = meta.w & 1u;
        if (mac_pass) {
          if (valid) {
            if (j == JM && ((len + 15u) >> 4) >= 4u * G * round + 4u * G - 4u) {  // length block not taken in the loop
              const uint4 q0 = RS(s).R0, q1 = RS(s).R1;
              const uint32_t R[5] = {q0.x, q0.y, q0.z, q0.w, q1.x};
#ifdef WG_HORNER2
              const uint32_t Rs[5] = {0u, 5u * q0.y, 5u * q0.z, 5u * q0.w, 5u * q1.x};
#else
              const uint4 q2 = RS(s).R2;
              const uint32_t Rs[5] = {0u, G == 2 ? 5u * q0.y : q1.y, G == 2 ? 5u * q0.z : q1.z,
                                      G == 2 ? 5u * q0.w : q1.w, G == 2 ? 5u * q1.x : q2.x};
#endif
              poly_mul(acc, R, Rs);
              acc[2] += (len << 12) & M26;  // le64(len) at bit 64: limb 2 holds bits 52..77
              acc[3] += len >> 14;
              acc[4] += 1u << 24;
            }
            uint32_t Ws[5];
            poly_scale5(W, Ws);
            poly_mul(acc, W, Ws);
          }
#pragma unroll
          for (int i = 0; i < 5; ++i) {  // slot sum (every lane of the slot ends with it)
            acc[i] += xor1_dpp(acc[i]);
            if constexpr (G >= 4) acc[i] += xor2_dpp(acc[i]);
            if constexpr (G >= 8) acc[i] += xor4_dpp(acc[i]);
            if constexpr (G == 16) acc[i] += xor8_dpp(acc[i]);
          }
        }
        const uint4 ad = RS(s).addr;
        const uint8_t* inp = P.in + ((uint64_t)ad.x | ((uint64_t)ad.y << 32));
        uint8_t* outp = P.out + ((uint64_t)ad.z | ((uint64_t)ad.w << 32));
        uint32_t bad = valid ? 0u : 1u;
        bool again = false;  // a verify-first open whose tag verified: the decrypt pass comes next
        if (mac_pass && valid && j == 0) {
          const uint4 sv = G == 2 ? make_uint4(RS(s).R1.y, RS(s).R1.z, RS(s).R1.w, RS(s).R2.x) : RS(s).s;
          uint32_t tag[4];
          poly_finish(acc, sv.x, sv.y, sv.z, sv.w, tag);
          if constexpr (MODE == WG_MODE_SEAL) {
            uint8_t* tp = outp + len;
            if ((((uintptr_t)tp) & 15u) == 0) {
              *(uint4*)tp = make_uint4(tag[0], tag[1], tag[2], tag[3]);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) store_u32_any(tp + 4 * i, tag[i]);
            }
          } else {  // all 16 bytes compared, no early exit
            const uint8_t* tp = inp + len;
            uint32_t diff = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) diff |= load_u32_any(tp + 4 * i) ^ tag[i];
            bad = diff ? 1u : 0u;
          }
        }
        if constexpr (MODE == WG_MODE_OPEN) {
          bad = bcastg<G, 0>(bad);
          again = VF && mac_pass && !bad && (meta.w & kVerifyFirst);
        }
        if constexpr (MODE == WG_MODE_OPEN) {
          if (again) {  // decrypt pass: the same rounds again, keystream XOR and stores only
            if (j == 0) RS(s).meta.w = meta.w | kDecryptPass;
            round = ~0u;  // incremented to 0 below
          } else {
            if (j == 0 && P.status) {
              uint32_t st = bad ? WG_PKT_BADTAG : WG_PKT_OK;
              if (!bad && P.rx) {  // fused receive-side check on the plaintext this slot wrote
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's plaintext stores have landed
                st = rx_verdict(*P.rx, outp, len, P.desc[pkt].key_slot);
              }
              P.status[pkt] = st;
            }
            if (bad && valid && (!VF || !(meta.w & kVerifyFirst))) {  // scrub the unauthenticated plaintext written
              for (uint32_t i = j; i < len; i += G) outp[i] = 0;
            }
            have = false;
          }
        } else {
          have = false;
        }
      }
    }
    if (have) ++round;
    wave_lds_sync();  // this round's image and records before the next round rewrites them
    WG_PH(5);
  }
  WG_PH_STORE(blk * TW + wv);
}

// VF: an open whose input and output buffers overlap (the host checks the two ranges): packets
// that overlap themselves verify first (kVerifyFirst); every other launch takes the one-pass body
template <int MODE, int G = 8, bool VF = false>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(8))) k_transport(TransportParams P) {
  __shared__ uint4 img_[TW][4 * 64];         // 4 KB per wave: [chunk q][lane] = the round's payload / MAC input
  __shared__ SlotRec rec_[TW][64 / G < 8 ? 8 : 64 / G];  // one record per slot: 1 KB per wave (2 KB with 4-lane slots)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t iter = 0;
  transport_body<MODE, G, VF>(P, blockIdx.x, wv, img_[wv], rec_[wv], iter);
}

// ---- mixed-length batches: 16-lane slots for the long packets, 8- (or 4-) lane slots for the rest ----
// The batch is ordered longest-first (k_lpt_*); the n_long packets at its front (more than
// `split` rounds of 8 blocks) take 16-lane slots, so no slot runs much more than `split` rounds.
// GS: lanes of the short packets' slots (8, or 4 for batches of short packets: half the ChaCha20 lanes
// a 40-B packet leaves idle, and the per-packet work shared by 16 packets of a wave instead of 8).
// Every slot holds ONE packet and the grid has as many workgroups as that takes (more than are
// resident): the hardware dispatcher starts each new workgroup as an old one retires, longest
// packets first. Workgroups [0, b16) run the 16-lane body, [b16, b16 + b8) the 8-lane body; the
// rest of the (host-sized, upper-bound) grid exits at once.
template <int GS = 8, int GT = 0>
__device__ __forceinline__ int mixed_part(const TransportParams& P, uint32_t blk, TransportParams& Q, uint32_t& qblk) {
  Q = P;
  uint32_t nl, nt = 0;
  if (P.bin_cnt) {  // one-launch planning: the bins' counts, the long packets those of keys above the split
    nl = 0;
#pragma unroll
    for (uint32_t k = 0; k < kFastBins; ++k) {
      const uint32_t c = ((const WG_CONST uint32_t*)P.bin_cnt)[k * kCntStride];
      nl += k > P.split ? c : 0u;
      if constexpr (GT != 0) nt += k <= P.split2 ? c : 0u;  // (split2 = 0: only key 0, the invalid packets)
    }
    nl = min(nl, P.n);
    if constexpr (GT != 0) nt = P.split2 ? min(nt, P.n - nl) : 0u;
  } else {
    nl = min(__builtin_amdgcn_readfirstlane(*(const WG_CONST uint32_t*)P.n_long), P.n);
  }
  const uint32_t b16 = (nl + 4u * TW - 1u) / (4u * TW);
  if (blk < b16) {
    Q.n = nl;
    Q.slots = b16 * TW * 4u;
    qblk = blk;
    return 16;
  }
  constexpr uint32_t spw = 64u / GS;  // short slots per wave
  const uint32_t ns = P.n - nl - nt, bs = (ns + spw * TW - 1u) / (spw * TW);
  if (blk - b16 < bs) {
    if (P.bin_cnt) Q.pos_base = nl;  // the sparse order's positions run on past the long packets
    else Q.order = P.order + nl;
    Q.n = ns;
    Q.slots = bs * TW * spw;
    qblk = blk - b16;
    return GS;
  }
  if constexpr (GT != 0) {  // the tiny packets (keys <= split2, at the end of the order) in GT-lane slots
    constexpr uint32_t tpw = 64u / GT;
    const uint32_t bt = (nt + tpw * TW - 1u) / (tpw * TW);
    if (blk - b16 - bs < bt) {
      Q.pos_base = nl + ns;
      Q.n = nt;
      Q.slots = bt * TW * tpw;
      qblk = blk - b16 - bs;
      return GT;
    }
  }
  return 0;
}

template <int MODE, bool VF = false, int GS = 8>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(8))) k_transport_mixed(TransportParams P) {
  __shared__ uint4 img_[TW][4 * 64];
  __shared__ SlotRec rec_[TW][64 / GS];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  TransportParams Q;
  uint32_t qb = 0, iter = 0;
  const int g = mixed_part<GS>(P, blockIdx.x, Q, qb);
  if (g == 16) transport_body<MODE, 16, VF, kPosStatic, false, (int)kFastBins>(Q, qb, wv, img_[wv], rec_[wv], iter);
  else if (g == GS) transport_body<MODE, GS, VF, kPosStatic, false, (int)kFastBins>(Q, qb, wv, img_[wv], rec_[wv], iter);
}

#ifndef WG_STITCH_WPE
#define WG_STITCH_WPE 5  // waves per SIMD the stitched kernels' register allocation targets (96 VGPRs: no spill)
#endif
// GT = 2: a third part after the GS-lane one, the tiny packets (keys <= split2) in 2-lane slots (32 per wave:
// a 40-B packet's two blocks fill its lanes instead of half of a 4-lane slot). Its records need twice the LDS.
template <int GS = 8, bool ST = false, int GT = 0>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(ST ? WG_STITCH_WPE : 8)))
k_step_mixed(TransportParams S, TransportParams O) {
  __shared__ uint4 img_[TW][4 * 64];
  // slot records: 128 B per GS- or 16-lane slot, 80 B per 2-lane slot (transport_body's kRecStride)
  constexpr uint32_t kRecU4 = GT ? ((64 / GS) * 8 > (64 / GT) * 5 ? (64 / GS) * 8 : (64 / GT) * 5) : (64 / GS) * 8;
  __shared__ uint4 recraw_[TW][kRecU4];
  SlotRec* const rec = (SlotRec*)recraw_[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  TransportParams QS, QO;
  uint32_t qb = 0, qb2 = 0, iter = 0;
  const int g = mixed_part<GS, GT>(S, blockIdx.x, QS, qb);
  (void)mixed_part<GS, GT>(O, blockIdx.x, QO, qb2);  // the same split: the open batch has the seal's lengths
  if (g == 16) {
    transport_body<WG_MODE_SEAL, 16, false, kPosStatic, ST, (int)kFastBins>(QS, qb, wv, img_[wv], rec, iter);
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
    transport_body<WG_MODE_OPEN, 16, false, kPosStatic, ST, (int)kFastBins>(QO, qb, wv, img_[wv], rec, iter);
  } else if (g == GS) {
    transport_body<WG_MODE_SEAL, GS, false, kPosStatic, ST, (int)kFastBins>(QS, qb, wv, img_[wv], rec, iter);
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
    transport_body<WG_MODE_OPEN, GS, false, kPosStatic, ST, (int)kFastBins>(QO, qb, wv, img_[wv], rec, iter);
  } else if constexpr (GT != 0) {
    if (g == GT) {
      transport_body<WG_MODE_SEAL, GT, false, kPosStatic, false, (int)kFastBins>(QS, qb, wv, img_[wv], rec, iter);
      asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
      transport_body<WG_MODE_OPEN, GT, false, kPosStatic, false, (int)kFastBins>(QO, qb, wv, img_[wv], rec, iter);
    }
  }
}

// One launch, two directions (wg_duplex_batch): a node's outgoing batch sealed and its
// incoming batch opened side by side. Workgroups [0, 2m) alternate seal / open (m = the
// smaller grid), the rest belong to the larger direction; each half runs exactly the
// k_transport body on its own grid, so the bytes written are those of the two separate
// launches. The two halves share the LDS declared here (one image + records per wave).
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(8)))
k_duplex(TransportParams S, TransportParams O, uint32_t seal_blocks, uint32_t open_blocks) {
  __shared__ uint4 img_[TW][4 * 64];
  __shared__ SlotRec rec_[TW][8];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t m = min(seal_blocks, open_blocks);
  const uint32_t b = blockIdx.x;
  bool seal;
  uint32_t idx;
  if (b < 2u * m) {
    seal = (b & 1u) == 0u;
    idx = b >> 1;
  } else {
    seal = seal_blocks > open_blocks;
    idx = b - m;
  }
  uint32_t iter = 0;
  if (seal) transport_body<WG_MODE_SEAL>(S, idx, wv, img_[wv], rec_[wv], iter);
  else transport_body<WG_MODE_OPEN>(O, idx, wv, img_[wv], rec_[wv], iter);
}

// One launch, one dependent step (wg_duplex_batch with WG_F_AFTER_SEAL): every wave seals its
// packets and then opens the same batch positions of the open batch, which read what its own
// seal wrote (open packet i is ordered after seal packet i, include/wgaead.h). Both halves use one
// grid and one packet order, so slot g opens exactly the packets it sealed. The waves that finish
// sealing first start opening while the others still seal: the seal launch's tail and the open
// launch's start, which two back-to-back launches leave partly idle, overlap.
// WPE: the waves per SIMD the register allocation targets. 8 (64 VGPRs) everywhere, except a grid
// that holds at most half the resident waves anyway (the persistent longest-first pairs of a
// mixed batch: 4 waves per SIMD), which takes the WPE = 4 build (66 VGPRs and no SGPR spills,
// against 64 VGPRs and 12 SGPRs spilled to VGPR lanes; WG_STEP_WPE4=0 for the other).
// Test hook of k_step (WG_TEST_STEP_FLIP, never set in production): between the two halves, lane 0 of
// each slot flips bit 0 of the tag its seal wrote for the slot's first packet (batch position g) when
// that packet's index is a multiple of S.test_flip. The open half then rejects it and the ciphertext
// differs from the reference, so the bench's check of the k_step output it timed must fail
// (tests/test_gpu_bench.py). Outside transport_body: the product body's code is unchanged.
template <int G>
__device__ __forceinline__ void step_test_flip(const TransportParams& S, uint32_t blk, uint32_t wv, uint32_t flip) {
  const uint32_t lane = threadIdx.x & 63u, g = (blk * TW + wv) * (64u / G) + lane / G;
  if ((lane & (G - 1u)) == 0u && g < S.n) {
    const uint32_t i = S.order ? S.order[g] : g;
    const wg_pkt d = S.desc[i];
    if ((i & (flip - 1u)) == 0u &&
        transport_valid<WG_MODE_SEAL>(d.in_off, d.out_off, d.len, d.key_slot, S.max_len, S.key_slots, S.in_size,
                                      S.out_size))
      S.out[d.out_off + d.len] ^= 1u;
  }
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
}

// FLIP: the test-hook instantiation (WG_TEST_STEP_FLIP), launched only by the test library (WG_TEST_HOOKS);
// the product instantiations carry no hook code at all.
template <int G = 8, int WPE = 8, bool FLIP = false, bool ST = false, int MX = 0>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(WPE)))
k_step(TransportParams S, TransportParams O, uint32_t test_flip) {
  __shared__ uint4 img_[TW][4 * 64];
  __shared__ SlotRec rec_[TW][64 / G < 8 ? 8 : 64 / G];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t iter = 0;  // one issue-priority schedule over both halves (plan_transport: prio_step of the step)
  transport_body<WG_MODE_SEAL, G, false, kPosStatic, ST, MX>(S, blockIdx.x, wv, img_[wv], rec_[wv], iter);
  // the open reads the ciphertext and tags this wave just stored: wait until the stores are
  // performed and drop this CU's L1 lines (an in-place seal read the plaintext through them)
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
  if constexpr (FLIP) step_test_flip<G>(S, blockIdx.x, wv, test_flip);
  transport_body<WG_MODE_OPEN, G, false, kPosStatic, ST, MX>(O, blockIdx.x, wv, img_[wv], rec_[wv], iter);
}

// k_step with dynamic claims (mixed-length batches, WG_CLAIM): the seal half claims its slots' packets
// from the sub-order counters and logs them per position; the open half replays that log, so slot g
// opens exactly what it sealed (the same wave wrote it: the half boundary below orders the accesses).
template <int G = 8, int WPE = 4>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(WPE)))
k_step_claim(TransportParams S, TransportParams O) {
  __shared__ uint4 img_[TW][4 * 64];
  __shared__ SlotRec rec_[TW][8];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t iter = 0;
  transport_body<WG_MODE_SEAL, G, false, kPosClaim>(S, blockIdx.x, wv, img_[wv], rec_[wv], iter);
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
  transport_body<WG_MODE_OPEN, G, false, kPosChain>(O, blockIdx.x, wv, img_[wv], rec_[wv], iter);
}

// ---- longest-first order for mixed-length batches (LPT) ----------------------------------
// key = rounds of the packet (invalid lengths sort last); counting sort into descending keys.
template <int MODE>
__device__ __forceinline__ uint32_t lpt_key(const wg_pkt* d, uint32_t i, uint32_t max_len) {
  const uint32_t len = d[i].len;
  if (len > max_len) return 0u;
  const uint32_t nb = ((len + 63u) >> 6) + 1u;
  return (nb + 7u) >> 3;
}

// Two launches, no global atomics and no memset: k_lpt_hist writes one histogram per block
// over a contiguous range of the batch; k_lpt_scatter (same grid) gives each block its base
// per key from all blocks' histograms (keys above it in every block, this key in the blocks
// before it) and ranks its packets in LDS.
constexpr uint32_t LPT_THREADS = 1024, LPT_MAX_BLOCKS = 64;

__device__ __forceinline__ void lpt_range(uint32_t n, uint32_t& lo, uint32_t& hi) {
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  lo = min(n, blockIdx.x * per);
  hi = min(n, lo + per);
}

template <int MODE>
__global__ void __launch_bounds__(LPT_THREADS) k_lpt_hist(const wg_pkt* d, uint32_t n, uint32_t max_len,
                                                          uint32_t* bh) {
  __shared__ uint32_t h[LPT_BINS];
  for (uint32_t k = threadIdx.x; k < LPT_BINS; k += LPT_THREADS) h[k] = 0;
  __syncthreads();
  uint32_t lo, hi;
  lpt_range(n, lo, hi);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += LPT_THREADS) atomicAdd(&h[lpt_key<MODE>(d, i, max_len)], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < LPT_BINS; k += LPT_THREADS) bh[blockIdx.x * LPT_BINS + k] = h[k];
}

// order[pos] = packet, keys descending
template <int MODE>
__global__ void __launch_bounds__(LPT_THREADS) k_lpt_scatter(const wg_pkt* d, uint32_t n, uint32_t max_len,
                                                             const uint32_t* bh, uint32_t* order, uint32_t split,
                                                             uint32_t* n_long, uint32_t* claim, uint32_t claim_nc,
                                                             uint32_t claim_base) {
  // the dynamic-claim counters of the launch this order is for (k_step_claim): one 64-B line each
  if (claim && blockIdx.x == 0 && threadIdx.x < claim_nc) claim[16u * threadIdx.x] = claim_base;
  __shared__ uint32_t all[LPT_MAX_BLOCKS * LPT_BINS];  // every block's histogram (coalesced load)
  __shared__ uint32_t tot[LPT_BINS], base[LPT_BINS];
  for (uint32_t e = threadIdx.x; e < gridDim.x * LPT_BINS; e += LPT_THREADS) all[e] = bh[e];
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < LPT_BINS; k += LPT_THREADS) {
    uint32_t t = 0, before = 0;
    for (uint32_t b = 0; b < gridDim.x; ++b) {
      const uint32_t v = all[b * LPT_BINS + k];
      t += v;
      before += b < blockIdx.x ? v : 0u;
    }
    tot[k] = t;
    base[k] = before;
  }
  __syncthreads();
  if (threadIdx.x < 64u) {  // packets with a larger key come first: wave 0 scans the keys
    // in descending order, lane l holding positions 3l..3l+2 (key LPT_BINS-1-p)
    static_assert(3u * 64u >= LPT_BINS, "three keys per lane");
    const uint32_t l = threadIdx.x;
    uint32_t v[3], own = 0;
#pragma unroll
    for (uint32_t q = 0; q < 3u; ++q) {
      const uint32_t p = 3u * l + q;
      v[q] = p < LPT_BINS ? tot[LPT_BINS - 1u - p] : 0u;
      own += v[q];
    }
    uint32_t inc = own;
#pragma unroll
    for (uint32_t off = 1; off < 64u; off <<= 1) {
      const uint32_t up = __shfl_up(inc, off, 64);
      inc += l >= off ? up : 0u;
    }
    uint32_t acc = inc - own;
#pragma unroll
    for (uint32_t q = 0; q < 3u; ++q) {
      const uint32_t p = 3u * l + q;
      if (p < LPT_BINS) tot[LPT_BINS - 1u - p] = acc;
      acc += v[q];
    }
    // the packets with more than `split` rounds (keys > split) come first: their count is the
    // exclusive prefix at key `split`
    if (n_long && blockIdx.x == 0 && split + 1u < LPT_BINS) {
      const uint32_t p = LPT_BINS - 1u - split;  // position of key `split` in the descending scan
      if (l == p / 3u) {
        uint32_t a = inc - own;
        for (uint32_t q = 0; q < p % 3u; ++q) a += v[q];
        *n_long = a;
      }
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < LPT_BINS; k += LPT_THREADS) base[k] += tot[k];
  __syncthreads();
  uint32_t lo, hi;
  lpt_range(n, lo, hi);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += LPT_THREADS) order[atomicAdd(&base[lpt_key<MODE>(d, i, max_len)], 1u)] = i;
}

// k_lpt_one's counter set per call: the counts kCntStride words apart, the fused step's publication count at
// kPlanDone), two sets used in turn
constexpr uint32_t kPlanDone = kWideBins * kCntStride > 32u ? kWideBins * kCntStride : 32u;
constexpr uint32_t kPlanSet = kPlanDone + 32u;  // words per set (the publication count on a line of its own)

// The body of k_lpt_one for block `blk` of `nblk` with `threads` threads over NB keys: h / base are NB words of LDS.
// A thread takes KPT packets per trip, their descriptor loads issued together, and when the block's range is
// one trip (the usual case) keeps the keys for the scatter pass: two load latencies per plan, not 2 x trips.
template <int MODE, int KPT = 1, uint32_t NB = kFastBins>
__device__ __forceinline__ void lpt_one_body(const wg_pkt* d, uint32_t n, uint32_t max_len, uint32_t* cnt,
                                             uint32_t* cnt_next, uint32_t* order, uint32_t blk, uint32_t nblk,
                                             uint32_t threads, uint32_t* h, uint32_t* base) {
  if (threadIdx.x < NB) h[threadIdx.x] = 0;
  // the next call's counts ([0, NB)) and k_step_mixed_fused's publication count (kPlanDone: its own line,
  // away from the counts' atomics)
  if (blk == 0 && ((threadIdx.x < kWideBins * kCntStride && threadIdx.x % kCntStride == 0u) || threadIdx.x == kPlanDone))
    cnt_next[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t per = (n + nblk - 1u) / nblk;
  const uint32_t lo = min(n, blk * per), hi = min(n, lo + per);
  const uint32_t lane = threadIdx.x & 63u, span = threads * KPT;
  // LDS atomics are aggregated per wave and key: one ballot per key, then ONE ds_add_rtn in which lane k adds
  // key k's lane count to slots[k] (six independent adds, not a chain of six round trips), one bpermute for
  // each lane's base in its key and mbcnt for its rank among the wave's lanes of that key
  auto wave_rank = [&](uint32_t* slots, uint32_t key) {  // this lane's rank among the wave's lanes of its key
    uint64_t mine = 0;
    uint32_t cnt_k = 0;
#pragma unroll
    for (uint32_t k = 0; k < NB; ++k) {
      const uint64_t m = __ballot(key == k);
      mine = key == k ? m : mine;
      cnt_k = lane == k ? (uint32_t)__popcll(m) : cnt_k;
    }
    uint32_t b = 0;
    if (cnt_k) b = atomicAdd(&slots[lane], cnt_k);  // lanes 0..NB-1 only (cnt_k = 0 elsewhere)
    b = __shfl(b, (int)(key < NB ? key : 0u), 64);
    return b + (uint32_t)__popcll(mine & ((1ull << lane) - 1ull));
  };
  auto keys_at = [&](uint32_t i0, uint32_t (&key)[KPT]) {  // every lane of a wave takes part in each trip
#pragma unroll
    for (int t = 0; t < KPT; ++t) {
      const uint32_t i = i0 + t * threads + threadIdx.x;
      key[t] = i < hi ? lpt_key<MODE>(d, i, max_len) : NB;
    }
  };
  uint32_t key[KPT];
  for (uint32_t i0 = lo; i0 < hi; i0 += span) {
    keys_at(i0, key);
#pragma unroll
    for (int t = 0; t < KPT; ++t) (void)wave_rank(h, key[t]);
  }
  __syncthreads();
  if (threadIdx.x < NB) {
    const uint32_t k = threadIdx.x, c = h[k];
    base[k] = k * n + (c ? atomicAdd(&cnt[k * kCntStride], c) : 0u);
  }
  __syncthreads();
  const bool one_trip = hi - lo <= span;
  for (uint32_t i0 = lo; i0 < hi; i0 += span) {
    if (!one_trip) keys_at(i0, key);
#pragma unroll
    for (int t = 0; t < KPT; ++t) {
      const uint32_t i = i0 + t * threads + threadIdx.x;
      const uint32_t at = wave_rank(base, key[t]);
      if (i < hi) order[at] = i;
    }
  }
}

// One launch instead of k_lpt_hist + k_lpt_scatter, for batches whose keys fit kFastBins (max_len <= 2,048 B,
// the short-packet plan): each block counts its range's keys in LDS, takes its base in every non-empty key
// with ONE atomicAdd on that key's global counter, and ranks its packets into the key's region of a sparse
// order (key k at order[k * n]). No grid-wide barrier: the consumer derives the positions from the counts.
// The counters are double-buffered by call (cnt for this call, zero on entry; cnt_next zeroed here for the
// next), so no memset launch either. Order inside a key: arbitrary (every position of the order is a packet).
// (THREADS, KPT: the block shape)
template <int MODE, uint32_t THREADS = LPT_THREADS, int KPT = 1, uint32_t NB = kFastBins>
__global__ void __launch_bounds__(THREADS) k_lpt_one(const wg_pkt* d, uint32_t n, uint32_t max_len, uint32_t* cnt,
                                                     uint32_t* cnt_next, uint32_t* order) {
  __shared__ uint32_t h[NB], base[NB];
  lpt_one_body<MODE, KPT, NB>(d, n, max_len, cnt, cnt_next, order, blockIdx.x, gridDim.x, THREADS, h, base);
}

// k_step_mixed with its planning folded in (WG_LPT_FUSED, the short-packet plan): workgroups [0, np) plan as
// k_lpt_one does and then publish (their stores acknowledged, one release count per workgroup in cnt[kPlanDone]); the
// other workgroups wait for all np publications (one acquire poll per workgroup, s_sleep between polls) and
// then run k_step_mixed's body. The planners are the lowest workgroup indices, so they are dispatched before
// any waiting workgroup can occupy the machine. A wait is bounded (kPlanWaitTicks of s_memrealtime); a
// workgroup that runs out of it writes *err and does no work, and the host fails the next call.
constexpr uint64_t kPlanWaitTicks = 5000000;  // 50 ms at 100 MHz
#ifdef WG_DIAG  // diagnostic build: s_memrealtime per workgroup (tools/fused_timing.py): a planner's start and
                // publication, a consumer's arrival, release from the wait and end
constexpr size_t kFusedStampOff = 400000;
#define WG_FUSED_STAMP(j, v) \
  if (S.stamps && threadIdx.x == 0) S.stamps[kFusedStampOff + 3u * blockIdx.x + (j)] = (v)
#else
#define WG_FUSED_STAMP(j, v)
#endif
template <int GS = 8, bool ST = false>
__global__ void __launch_bounds__(64 * TW) __attribute__((amdgpu_waves_per_eu(ST ? WG_STITCH_WPE : 8)))
k_step_mixed_fused(TransportParams S, TransportParams O, uint32_t np, uint32_t* cnt, uint32_t* cnt_next, uint32_t* err,
                   uint32_t poll) {
  __shared__ uint4 img_[TW][4 * 64];
  __shared__ SlotRec rec_[TW][64 / GS];
  WG_FUSED_STAMP(0, __builtin_amdgcn_s_memrealtime());
  if (blockIdx.x < np) {
    uint32_t* h = (uint32_t*)&img_[0][0];
    lpt_one_body<WG_MODE_SEAL, 4>(S.desc, S.n, S.max_len, cnt, cnt_next, (uint32_t*)S.order, blockIdx.x, np, 64u * TW,
                               h, h + 8);
    // every wave's order stores acknowledged by its L2, then one release (one L2 write-back) per workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&cnt[kPlanDone], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    WG_FUSED_STAMP(1, __builtin_amdgcn_s_memrealtime());
    return;
  }
  __shared__ uint32_t go;
  if (threadIdx.x == 0) {
    uint32_t ok = 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // relaxed polls (an acquire per poll would invalidate the L2 every time), one acquire fence after
    // poll (WG_FUSED_POLL, A/B): 0 agent-scope loads, 1 system-scope loads, 2 read-modify-writes (performed at
    // the coherence point), at a quarter of the rate
    auto published = [&]() {
      if (poll == 1) return __hip_atomic_load(&cnt[kPlanDone], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (poll == 2) return __hip_atomic_fetch_add(&cnt[kPlanDone], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return __hip_atomic_load(&cnt[kPlanDone], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    while (published() < np) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kPlanWaitTicks) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0u;
        break;
      }
      __builtin_amdgcn_s_sleep(8);  // ~0.2 us: the polls of every waiting workgroup meet at one line
      if (poll == 2) {
        __builtin_amdgcn_s_sleep(8);
        __builtin_amdgcn_s_sleep(8);
        __builtin_amdgcn_s_sleep(8);
      }
    }
    // no agent-scope acquire here: its L2 invalidation, made by every waiting workgroup at about the same time,
    // cost the step 28 us (IMIX, profiles/r06_fused_ab.jsonl). None is needed on this hardware path: the plan's
    // lines cannot be in this XCD's L2 (a dispatch starts with the L2s invalidated, and no workgroup of this
    // launch reads them before the plan is published: the planners only write them, by stores and by atomics
    // performed at the device's coherence point), and the planners' release wrote them back; only this CU's
    // L1 is invalidated, as between a step's halves
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
    go = ok;
    WG_FUSED_STAMP(1, __builtin_amdgcn_s_memrealtime());
  }
  __syncthreads();
  if (!go) return;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  TransportParams QS, QO;
  uint32_t qb = 0, qb2 = 0, iter = 0;
  const uint32_t blk = blockIdx.x - np;
  const int g = mixed_part<GS>(S, blk, QS, qb);
  (void)mixed_part<GS>(O, blk, QO, qb2);
  if (g == 16) {
    transport_body<WG_MODE_SEAL, 16, false, kPosStatic, ST, (int)kFastBins>(QS, qb, wv, img_[wv], rec_[wv], iter);
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
    transport_body<WG_MODE_OPEN, 16, false, kPosStatic, ST, (int)kFastBins>(QO, qb, wv, img_[wv], rec_[wv], iter);
  } else if (g == GS) {
    transport_body<WG_MODE_SEAL, GS, false, kPosStatic, ST, (int)kFastBins>(QS, qb, wv, img_[wv], rec_[wv], iter);
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
    transport_body<WG_MODE_OPEN, GS, false, kPosStatic, ST, (int)kFastBins>(QO, qb, wv, img_[wv], rec_[wv], iter);
  }
  WG_FUSED_STAMP(2, __builtin_amdgcn_s_memrealtime());
}

// ---- wire framing (TransportPacket.java:18-35) --------------------------------------------
// 16-B transport header {u8 4, u8 0[3], u32 receiver_index, u64 counter}, little-endian,
// written with 4-B or 1-B stores by alignment.
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

// One thread per packet: header of every packet the seal kernel accepted (the same
// validity test), at out_off - 16 (UnencryptedOutgoingTransport.java:14-18 writes the
// type and receiver index, EncryptedOutgoingTransport.java:11-14 the counter).
__global__ void __launch_bounds__(256) k_frame_seal(const wg_pkt* __restrict__ d, uint32_t n,
                                                    const uint32_t* __restrict__ rx, uint32_t max_len,
                                                    uint32_t key_slots, uint64_t in_size,
                                                    uint8_t* __restrict__ out, uint64_t out_size) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const wg_pkt p = d[i];
  if (p.out_off < 16 ||
      !transport_valid<WG_MODE_SEAL>(p.in_off, p.out_off, p.len, p.key_slot, max_len, key_slots, in_size, out_size))
    return;
  put_header(out + p.out_off - 16, rx[p.key_slot], p.counter);
}

// Open descriptors straight from received wire packets (UndecryptedIncomingTransport.java:20-33):
// ciphertext at +16, plaintext right after the packet in the same buffer (:30).
__global__ void __launch_bounds__(256) k_parse_open(const uint8_t* __restrict__ wire, uint64_t wire_size,
                                                    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                    const uint32_t* __restrict__ slot, uint32_t n,
                                                    wg_pkt* __restrict__ d, uint32_t* __restrict__ st) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i];
  const uint32_t wl = len[i];
  wg_pkt p;
  p.in_off = o + 16;
  p.out_off = o + wl;
  p.key_slot = slot[i];
  p.counter = 0;
  p.len = WG_LEN_INVALID;
  // packet [o, o+wl) plus its plaintext [o+wl, o+2wl-32) must lie inside the buffer
  bool ok = wl >= 32 && o <= wire_size && (uint64_t)wl <= wire_size - o && (uint64_t)wl - 32 <= wire_size - o - wl;
  if (ok) {
    const uint8_t* h = wire + o;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = load_u32_any(h + 4 * k);
    ok = (w[0] & 0xffu) == 4u;  // only the type byte is checked (UndecryptedIncomingTransport.java:24-26)
    if (ok) {
      p.counter = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
      p.len = wl - 32;
    }
  }
  d[i] = p;
  if (st) st[i] = ok ? WG_PKT_OK : WG_PKT_BADHDR;
}

}  // namespace wgt
