// wg_pp.hip — the per-packet entry points wg_seal1 / wg_open1 served by a persistent
// device kernel (included by wg_capi.hip).
//
// The reference seals / opens one packet per synchronous call from ForkJoinPool workers
// (TransportManager.java:41,79,152-158 -> SymmetricKeypair.java:63-83). Those calls stay
// per-packet and synchronous. A small persistent kernel (k_pp: W server units, each one
// four-wave workgroup) serves them through pinned memory with no launch on the per-packet path:
//   caller: claims a FREE entry i of the kRing-entry ring (a CAS on a host-side state word; a
//           thread starts at its own unit's entries, no ticket order), copies the packet + header
//           {seq, mode, len, counter, key} into in-slot i (pinned, fine-grained host memory), then
//           toggles bit i of the doorbell words (one atomic XOR: the publication, after every
//           other byte);
//   unit w: owns entries [w E, (w + 1) E), E = kRing / W. Its wave 0 polls the unit's doorbell
//           word(s) (two system-scope polls in flight, staggered) and picks EVERY entry whose bit
//           differs from its acknowledged copy, in index order (out-of-order service: a caller that
//           is descheduled between claiming and publishing delays nobody but itself). Per entry
//           the four waves read the header and payload (16-B system-scope loads, one PCIe round
//           trip), waves 0..2 run the ChaCha20 blocks (four lanes per block, DPP quad rotations)
//           while wave 3 computes block 0 and the Poly1305 powers r^1..r^64 (a DPP product scan)
//           and, for an open, the tag of the received ciphertext; a seal's tag follows the
//           cipher. The unit writes ct||tag / plaintext into out-slot i (16-B system-scope
//           stores), waits for them, then stores done[i] = seq << 8 | status;
//   caller: spins on done[i] in its own memory, copies the result out (open: only when the
//           tag verified, so dst stays untouched on a bad tag, ChaCha20Poly1305.java:51-55),
//           and frees the entry. A call that fails after publishing (a refused launch, a stream
//           error) leaves its entry ORPHAN: the next server serves it like any other, and the
//           entry is reclaimed once its completion word shows up, so no entry is ever lost.
// The session key travels in the slot header from a host mirror of the key table (the
// reference keeps its keys in host memory too, SymmetricKeypair.java:40-50), so the
// persistent kernel never reads a device key table that wg_keys_set may rewrite under it.
// Exit is collective: the first unit that finds the whole server idle for idle_us (a shared
// last-activity stamp), or the launch older than life_ms, raises a quit flag; every unit
// serves what it has already seen and leaves, the last one raises the host-visible exit flag,
// and the next caller relaunches. The context's stop flag ends every unit at its next poll.
// Packets longer than a slot (> kPPMaxLen, beyond the reference pipeline's 4-KB buffers) take
// the host batch path.
#pragma once

namespace wgpp {

using namespace wgd;
using wgt::mask_chunk;

constexpr uint32_t kRing = 512;                 // entries (concurrent per-packet calls)
constexpr uint32_t kHdr = 64;                   // in-slot header bytes
constexpr uint32_t kData = 4096;                // payload bytes per slot
constexpr uint32_t kInSlot = kHdr + kData;      // in-slot stride
constexpr uint32_t kOutSlot = kData;            // out-slot stride
constexpr uint32_t kPPMaxLen = kData - 16;      // 4080: payload + tag fit a slot
constexpr uint32_t kMaxWaves = 64;              // server units (the API's "waves")
constexpr uint32_t kUnitWaves = 4;              // waves per unit (one workgroup)
constexpr uint32_t kUnitThreads = 64u * kUnitWaves;
constexpr uint32_t kCipherWaves = 3;            // waves 0..2: ChaCha20 blocks; wave 3: Poly1305
constexpr uint32_t kMacWave = 3;
constexpr uint32_t kInQ = kInSlot / 16;         // 16-B units of an in-slot (260)
constexpr uint32_t kFirstQ = 128;               // read right after the doorbell: header + 1984 B
constexpr uint32_t kCmdLeave = ~0u;

struct Hdr {          // first 64 B of an in-slot (host-written)
  uint64_t seq;       // ticket + 1: written last
  uint64_t counter;   // transport counter (nonce = LE64(counter) || 0^4)
  uint32_t mode;      // WG_MODE_SEAL / WG_MODE_OPEN
  uint32_t len;       // payload bytes (open: ct, the tag follows)
  uint32_t key[8];
  uint32_t _pad[2];
};
static_assert(sizeof(Hdr) == kHdr, "slot header is 64 B");

struct Ctl {          // pinned, host-written
  uint32_t stop;
  uint32_t _pad[15];
};

constexpr uint32_t kBells = kRing / 64;  // doorbell words: bit i % 64 of word i / 64 toggles per publication

struct PPParams {
  const uint8_t* in;      // device alias: kRing in-slots
  uint8_t* out;           // device alias: kRing out-slots
  uint64_t* done;         // device alias: kRing completion words
  const uint64_t* bell;   // device alias: kBells doorbell words (host-toggled)
  const Ctl* ctl;         // device alias
  uint64_t* exit_flag;    // device alias (pinned): gen, written by the last unit to exit
  uint8_t* ack;           // device memory: per entry, the doorbell parity already served (kept across launches)
  uint32_t* exited;       // device memory (8-B aligned): {units exited in this launch, quit flag} (zeroed)
  uint32_t* quit;         // = exited + 1: raised by the first unit that decides the server leaves
  uint64_t* last;         // device memory: s_memrealtime of the last service in this launch (zeroed)
  uint64_t* svc;          // device alias (pinned): per entry, s_memrealtime ticks from the unit seeing its
                          // doorbell bit to its completion store (wg_pp_last_call's device service time)
  uint32_t waves;         // W units (power of two, 1..64): unit w owns entries [w E, (w + 1) E), E = kRing / W
  uint32_t gen;
  uint64_t idle_ticks;    // s_memrealtime ticks (100 MHz)
  uint64_t life_ticks;
};

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

#ifdef WG_PP_STAMPS  // tools/pp_stamps.hip only: s_memrealtime per phase of each ticket
__device__ uint64_t g_pp_stamps[4096][10];  // [8]: the serving unit's XCC id, [9]: its unit index
#define PP_STAMP(t, k) \
  if (threadIdx.x == 0) g_pp_stamps[(t) % 4096u][k] = __builtin_amdgcn_s_memrealtime()
#else
#define PP_STAMP(t, k) do {} while (0)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16 B of pinned host memory per lane at system scope (sc0 sc1: the load misses the CU's caches,
// so nothing stale of an earlier use of the slot comes back and no cache invalidate is needed; the
// doorbell poll reads the same way). Issued unconditionally by every lane of a wave (lanes with
// nothing to read point at the slot's first 16 B) and not waited for: vm_wait before the value is
// used (the compiler does not count asm loads; the "+v" operands keep every use after the wait).
__device__ __forceinline__ u32x4 ld_sys128(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void vm_wait(u32x4& a) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(a) : : "memory"); }
__device__ __forceinline__ void vm_wait(u32x4& a, u32x4& b) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b) : : "memory");
}
// 16 B per lane to pinned host memory, system scope (write-through to the host)
__device__ __forceinline__ void st_sys128(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

// ---- ChaCha20 on the four lanes of a quad ---------------------------------------------------
// Lane q of a quad holds column q of the block's state (a = x[q], b = x[4 + q], c = x[8 + q],
// d = x[12 + q]), so a column round is one quarter round per lane and a diagonal round is the same
// after rotating b, c, d across the quad by 1, 2, 3 lanes (DPP quad_perm, no LDS). A block costs a
// lane 10 x (2 x 12 + 6) dependent instructions instead of 10 x 96: one wave on its own is bound by
// the dependent-issue latency, not the issue rate (one block per lane 1.2 us, two interleaved
// 2.0 us at 2.4 GHz, tools/pp_stamps), so a unit spreads the blocks over three waves.
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
constexpr int kQ1 = 0x39, kQ2 = 0x4e, kQ3 = 0x93;  // quad_perm [1,2,3,0], [2,3,0,1], [3,0,1,2]

__device__ __forceinline__ void chacha20_quad(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
#pragma unroll 1
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      a += b; d ^= a; d = rotl16(d);
      c += d; b ^= c; b = rotl(b, 12);
      a += b; d ^= a; d = rotl8(d);
      c += d; b ^= c; b = rotl(b, 7);
      if (half == 0) {  // columns -> diagonals: lane q takes b of column q+1, c of q+2, d of q+3
        b = quad_perm<kQ1>(b); c = quad_perm<kQ2>(c); d = quad_perm<kQ3>(d);
      } else {          // and back
        b = quad_perm<kQ3>(b); c = quad_perm<kQ2>(c); d = quad_perm<kQ1>(d);
      }
    }
  }
}

// ---- Poly1305 across a wave with DPP --------------------------------------------------------
// y <- y * (DPP-moved y) where TAKE; the multiply runs on every lane, the select keeps the others
template <int CTRL, int ROWS>
__device__ __forceinline__ void pow_scan_step(uint32_t y[5], bool take) {
  uint32_t z[5], zs[5], t[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    z[i] = (uint32_t)__builtin_amdgcn_update_dpp((int)y[i], (int)y[i], CTRL, ROWS, 0xf, false);
    t[i] = y[i];
  }
  poly_scale5(z, zs);
  poly_mul<false>(t, z, zs);  // a lone wave: no s_nop between the products (wg_device.h)
#pragma unroll
  for (int i = 0; i < 5; ++i) y[i] = take ? t[i] : y[i];
}
// x + (DPP-moved x), lanes the move does not reach adding 0
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
  return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118, kBcast15 = 0x142,
              kBcast31 = 0x143;

// The tag of the MAC image `mac` (nc ciphertext chunks; the last partial one is masked here, the
// length block is formed here) under one-time key pk, on one wave. Padded to 64 T chunks with D
// zero chunks in front, lane j takes positions P = 64 t + 63 - j, whose weight r^(64 T - P) =
// R^(T-1-t) r^(j+1) (R = r^64): acc_j = sum_t m(P) R^(T-1-t), and the polynomial is
// sum_j acc_j r^(j+1). y holds r^(j+1) (pow_scan), R = r^64.
__device__ __forceinline__ void mac_tag(const uint4* mac, uint32_t len, uint32_t nc, const uint32_t y[5],
                                        const uint32_t R[5], const uint32_t pk[8], uint32_t tag[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t Rs[5], ys[5];
  poly_scale5(R, Rs);
  poly_scale5(y, ys);
  const uint32_t M = nc + 1u;
  const uint32_t T = (M + 63u) >> 6;
  const uint32_t D = 64u * T - M;
  uint32_t acc[5] = {0, 0, 0, 0, 0};
  for (uint32_t t = 0; t < T; ++t) {
    if (t) poly_mul<false>(acc, R, Rs);
    const uint32_t p = 64u * t + 63u - lane;
    if (p >= D) {
      const uint32_t c = p - D;
      uint4 v = c < nc ? mac[c] : make_uint4(0u, 0u, len, 0u);  // chunk nc: le64(aad len 0) || le64(len)
      if (c + 1u == nc && (len & 15u)) v = mask_chunk(v, len & 15u);
      uint32_t cl[5];
      poly_block_limbs(v.x, v.y, v.z, v.w, 1u << 24, cl);
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[i] += cl[i];
    }
  }
  poly_mul<false>(acc, y, ys);
  // sum over the wave: each row of 16 (limbs stay < 2^31), carry, then the four row sums
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    acc[i] = dpp_add<kRowShr1, 0xf>(acc[i]);
    acc[i] = dpp_add<kRowShr2, 0xf>(acc[i]);
    acc[i] = dpp_add<kRowShr4, 0xf>(acc[i]);
    acc[i] = dpp_add<kRowShr8, 0xf>(acc[i]);
  }
  {
    uint32_t c;
    c = acc[0] >> 26; acc[0] &= M26; acc[1] += c;
    c = acc[1] >> 26; acc[1] &= M26; acc[2] += c;
    c = acc[2] >> 26; acc[2] &= M26; acc[3] += c;
    c = acc[3] >> 26; acc[3] &= M26; acc[4] += c;
    c = acc[4] >> 26; acc[4] &= M26; acc[0] += 5u * c;
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    acc[i] = dpp_add<kBcast15, 0xa>(acc[i]);  // lane 31: rows 0 + 1, lane 63: rows 2 + 3
    acc[i] = dpp_add<kBcast31, 0xc>(acc[i]);  // lane 63: all four
    acc[i] = __builtin_amdgcn_readlane(acc[i], 63);
  }
  poly_finish(acc, pk[4], pk[5], pk[6], pk[7], tag);
}

// A server unit's LDS
struct Unit {
  uint4 raw[kInQ + 4];           // header | payload (+ tag) as read
  uint4 img_out[kData / 16 + 4]; // the result (seal: ct || tag; open: the plaintext)
  uint32_t cmd;                  // the entry to serve next (kCmdLeave: the unit leaves)
  uint32_t status;               // open: WG_PKT_* from the MAC wave
};

// One packet by the whole unit (all four waves). spec: the unit's last packet needed more than the
// first 2 KB of its slot, so this one reads the whole slot in the first round trip.
__device__ void pp_serve(Unit& U, const PPParams& P, uint32_t i, uint64_t t_seen, bool& spec) {
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  const u32x4* src = (const u32x4*)(P.in + (size_t)i * kInSlot);
  u32x4* raw4 = (u32x4*)U.raw;
  // header + payload after the doorbell was seen (the host wrote them before it). Each load, its wait
  // and its use sit in one wave-uniform branch (no copy of an asm load's register can be taken before
  // its wait), and a wave with nothing to read issues nothing: extra reads of the slot's first line
  // from idle waves made the round trip 0.9 us longer; the first 2 KB are read by wave 0 alone (two
  // loads per lane)
  if (spec && wave == 0u) {
    u32x4 v0 = ld_sys128(src + tid), v1 = ld_sys128(src + min(kUnitThreads + lane, kInQ - 1u));
    vm_wait(v0, v1);
    raw4[tid] = v0;
    if (lane < kInQ - kUnitThreads) raw4[kUnitThreads + lane] = v1;
  } else if (!spec && wave == 0u) {
    u32x4 v0 = ld_sys128(src + lane), v1 = ld_sys128(src + 64u + lane);
    vm_wait(v0, v1);
    raw4[lane] = v0;
    raw4[64u + lane] = v1;
  } else if (spec) {
    u32x4 v0 = ld_sys128(src + tid);
    vm_wait(v0);
    raw4[tid] = v0;
  }
  __syncthreads();
  const Hdr& hd = *(const Hdr*)U.raw;
  const uint32_t mode = __builtin_amdgcn_readfirstlane(hd.mode);
  const uint32_t len = __builtin_amdgcn_readfirstlane(hd.len);
  const uint64_t seq = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(hd.seq >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)hd.seq);
  PP_STAMP(seq, 1);
#ifdef WG_PP_STAMPS
  if (tid == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_pp_stamps[seq % 4096u][0] = t_seen;
    g_pp_stamps[seq % 4096u][8] = xcc & 15u;
    g_pp_stamps[seq % 4096u][9] = blockIdx.x;
  }
#endif
  if (len > kPPMaxLen || (mode != WG_MODE_SEAL && mode != WG_MODE_OPEN)) {  // refused by the host before
    if (tid == 0)                                                             // publishing; never expected
      __hip_atomic_store(P.done + i, (seq << 8) | 0xffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    return;
  }
  const bool open = mode == WG_MODE_OPEN;
  const uint32_t n_in = len + (open ? 16u : 0u);
  const uint32_t nq = kHdr / 16 + ((n_in + 15u) >> 4);  // 16-B units of the slot in use (<= 260)
  if (nq > (spec ? kInQ : kFirstQ)) {  // past the first 2 KB: one more round trip for the rest
    const uint32_t k = kFirstQ + tid;
    if (kFirstQ + 64u * wave < nq) {   // waves with something to read
      u32x4 v = ld_sys128(src + min(k, nq - 1u));
      vm_wait(v);
      if (k < nq) raw4[k] = v;
    }
    __syncthreads();
  }
  spec = nq > kFirstQ;
  PP_STAMP(seq, 2);
#ifdef WG_PP_STAMPS
  const uint64_t cyc0 = __builtin_amdgcn_s_memtime();  // shader clock over the compute (slot 7)
#endif

  const uint32_t nc = (len + 15u) >> 4;          // ciphertext chunks
  const uint32_t nb = ((len + 63u) >> 6) + 1u;   // ChaCha20 blocks incl. the key block
  const uint32_t q = lane & 3u, g = lane >> 2;   // quad g, column q
  const uint32_t* hw = (const uint32_t*)U.raw;   // the header's words: counter at 2, key at 6
  const uint32_t k0 = hw[6 + q], k1 = hw[10 + q];
  const uint32_t sig = q == 0u ? 0x61707865u : q == 1u ? 0x3320646eu : q == 2u ? 0x79622d32u : 0x6b206574u;
  const uint32_t dn = q == 1u ? hw[2] : q == 2u ? hw[3] : 0u;  // state word 12 + q (q > 0): the nonce
  const uint4* img_in = U.raw + kHdr / 16;
  uint32_t y[5], R[5], pk[8];
  if (wave < kCipherWaves) {
    // blocks 16 wave + g, + 48 per round: ct (seal) / plaintext (open) into img_out, the last chunk's
    // bytes past len zeroed (the seal MAC image)
    const uint32_t* in_w = (const uint32_t*)img_in;
    uint32_t* out_w = (uint32_t*)U.img_out;
    for (uint32_t base = 16u * wave; base < nb; base += 16u * kCipherWaves) {
      const uint32_t b = base + g;
      uint32_t a = sig, bb = k0, c = k1, d = q ? dn : b;
      chacha20_quad(a, bb, c, d);
      const uint32_t ks[4] = {a + sig, bb + k0, c + k1, d + (q ? dn : b)};
      if (b >= 1u && b < nb) {
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
          const uint32_t ch = 4u * (b - 1u) + j;  // chunk; this lane: its dword q (keystream word 4 j + q)
          if (ch < nc) {
            const int rem = (int)len - (int)(16u * ch + 4u * q);
            const uint32_t m = rem >= 4 ? ~0u : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
            const uint32_t w = 4u * ch + q;
            out_w[w] = (ks[j] ^ in_w[w]) & m;
          }
        }
      }
    }
  } else {
    // the MAC wave: block 0 again (the one-time key), r^(j+1) per lane, and for an open the tag now:
    // its MAC image is the received ciphertext, which nobody writes
    uint32_t a = sig, bb = k0, c = k1, d = q ? dn : 0u;
    chacha20_quad(a, bb, c, d);
    a += sig;
    bb += k0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pk[k] = __builtin_amdgcn_readlane(a, k);
      pk[4 + k] = __builtin_amdgcn_readlane(bb, k);
    }
    poly_r_limbs(pk[0], pk[1], pk[2], pk[3], y);
    const uint32_t i16 = lane & 15u;  // a product scan: row_shr 1, 2, 4, 8 in each row, then row broadcasts
    pow_scan_step<kRowShr1, 0xf>(y, i16 >= 1u);
    pow_scan_step<kRowShr2, 0xf>(y, i16 >= 2u);
    pow_scan_step<kRowShr4, 0xf>(y, i16 >= 4u);
    pow_scan_step<kRowShr8, 0xf>(y, i16 >= 8u);
    pow_scan_step<kBcast15, 0xa>(y, (lane & 16u) != 0u);  // rows 1, 3 x r^16
    pow_scan_step<kBcast31, 0xc>(y, lane >= 32u);         // rows 2, 3 x r^32
#pragma unroll
    for (int k = 0; k < 5; ++k) R[k] = __builtin_amdgcn_readlane(y[k], 63);
    if (open) {
      uint32_t tag[4];
      mac_tag(img_in, len, nc, y, R, pk, tag);
      const uint32_t tag_in = lane < 16u ? ((const uint8_t*)img_in)[len + lane] : 0u;
      // all 16 bytes compared, no early exit
      const uint32_t mine = lane < 16u ? ((tag[lane >> 2] >> (8u * (lane & 3u))) & 0xffu) ^ tag_in : 0u;
      const uint32_t st = __any(mine != 0u) ? WG_PKT_BADTAG : WG_PKT_OK;
      if (lane == 0) U.status = st;
    }
  }
  __syncthreads();
  PP_STAMP(seq, 3);
  if (!open) {  // the seal MAC image is the ciphertext: the tag after the cipher waves
    if (wave == kMacWave) {
      uint32_t tag[4];
      mac_tag(U.img_out, len, nc, y, R, pk, tag);
      if (lane < 16u) ((uint8_t*)U.img_out)[len + lane] = (uint8_t)(tag[lane >> 2] >> (8u * (lane & 3u)));
    }
    __syncthreads();
  }
  PP_STAMP(seq, 4);
#ifdef WG_PP_STAMPS
  if (tid == 0) g_pp_stamps[seq % 4096u][7] = __builtin_amdgcn_s_memtime() - cyc0;
#endif
  const uint32_t status = open ? U.status : (uint32_t)WG_PKT_OK;
  // result: 16-B system-scope stores, one per thread (the out-slot is 4 KB, so the bytes past n_out in
  // the last 16 stay inside it); open writes the plaintext only when the tag verified
  const uint32_t n_out = status == WG_PKT_OK ? len + (open ? 0u : 16u) : 0u;
  if (tid < ((n_out + 15u) >> 4))
    st_sys128(P.out + (size_t)i * kOutSlot + 16u * tid, ((const u32x4*)U.img_out)[tid]);
  PP_STAMP(seq, 5);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's result bytes have landed
  __syncthreads();                                  // ... and every other wave's
  PP_STAMP(seq, 6);
  if (tid == 0) {
    // the service time first (only with WG_PP_CALL_STAMPS: one more PCIe write per packet): it is
    // ordered before the completion word the caller polls for
    if (P.svc) {
      __hip_atomic_store(P.svc + i, __builtin_amdgcn_s_memrealtime() - t_seen, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      // two relaxed stores to different addresses are not ordered by the memory model: the completion word
      // is issued only once this store has been performed (both are system-scope write-through stores), so a
      // caller that sees the completion also sees this value. (A release store here would also write back the
      // whole L2 before the completion: 2.9-ms calls in r06b.)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(P.done + i, (seq << 8) | status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// lane k's 64-bit value (k wave-uniform). readlane returns int: each half goes through uint32_t, or
// a low half with bit 31 set would sign-extend over the high half when the two are combined
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t k) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k);
  return ((uint64_t)hi << 32) | lo;
}

// One doorbell poll in flight per unit. Two or four in flight (staggered) found a publication sooner
// but congested the device's PCIe reads: the payload read after the doorbell took 1.9-3.5 (two) and
// 6.3 us (four) instead of 1.4, and a one-caller call 8-17 us instead of 7.7
// (profiles/r05_pp_poll_ab.jsonl). Only the first two polls after a service overlap, the second
// kPostServeStagger x 64 cycles behind: 1 caller p50 7.7 -> 6.8-7.0 us, 16 callers 2.4-2.6 -> 2.6-2.7
// GiB/s (20, 26, 34, 44: profiles/r05_pp_stagger_ab.jsonl).
constexpr uint32_t kPostServeStagger = 26;
__global__ void __launch_bounds__(kUnitThreads) k_pp(PPParams P) {
  __shared__ Unit U;
  const uint32_t w = blockIdx.x;
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  const uint32_t E = kRing / P.waves;           // entries of this unit: [base, base + E)
  const uint32_t base = w * E;
  const uint32_t nwords = (E + 63u) >> 6;       // doorbell words this unit reads (E >= 64)
  const uint32_t word0 = base >> 6;
  const uint32_t sub = base & 63u;              // E < 64: the unit's bits inside one word
  const uint64_t wmask = E >= 64u ? ~0ull : (((1ull << E) - 1ull) << sub);
  // wave 0 polls and picks; lane k holds doorbell word k of the unit's range: the acknowledged
  // parity (from the per-entry bytes the previous launch left) and the entries seen but not served
  uint64_t ack = 0, pend = 0;
  if (wave == 0) {
    for (uint32_t k = 0; k < nwords; ++k) {
      const uint32_t e = 64u * (word0 + k) + lane;
      const bool mine = e >= base && e < base + E;
      const uint64_t m = __ballot(mine && P.ack[e] != 0);
      if (lane == k) ack = m;
    }
  }
  // one poll = one load per lane: lanes < nwords the doorbell words, 33 {exited, quit}, 34 the last
  // service stamp, every other lane the stop word
  const uint64_t* paddr = lane < nwords   ? P.bell + word0 + lane
                          : lane == 33u   ? (const uint64_t*)P.exited
                          : lane == 34u   ? (const uint64_t*)P.last
                                          : (const uint64_t*)&P.ctl->stop;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool leave_after = false;  // wave 0: quit seen; leave once what was seen is served
  bool spec = false;
  uint64_t t_seen = 0;
  for (;;) {
    if (wave == 0) {
      if (!__any(pend != 0) && !leave_after) {
        auto look = [&](uint64_t v) -> int {  // 0: nothing, 1: serve, 2: leave
          if (__builtin_amdgcn_readlane((uint32_t)v, 32)) return 2;  // stop
          const uint64_t p = lane < nwords ? (v ^ ack) & wmask : 0ull;
          const bool quit = __builtin_amdgcn_readlane((uint32_t)(v >> 32), 33) != 0;
          if (__any(p != 0)) {
            pend = p;
            leave_after = quit;
            return 1;
          }
          if (quit) return 2;
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          const uint64_t l = lane_u64(v, 34);
          // another unit may have stamped `last` after this poll read it: no idle time then
          const uint64_t ref = l > t0 ? l : t0;
          const uint64_t since = now > ref ? now - ref : 0u;
          if (since > P.idle_ticks || now - t0 > P.life_ticks) {  // the whole server leaves together
            if (lane == 0) __hip_atomic_store(P.quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 2;
          }
          return 0;
        };
        int act = 0;
        {  // right after a service (when a caller's next packet is likeliest): a second poll about half
           // a round trip behind the first, then one at a time
          const uint64_t v1 = __hip_atomic_load(paddr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __builtin_amdgcn_s_sleep(kPostServeStagger);
          const uint64_t v2 = __hip_atomic_load(paddr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((act = look(v1)) == 0) act = look(v2);
        }
        for (uint32_t backoff = 0; act == 0;) {  // one poll at a time, at most 2 x 256 cycles apart
          const uint64_t v = __hip_atomic_load(paddr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((act = look(v)) != 0) break;
          if (backoff < 2u) ++backoff;
          for (uint32_t k = 0; k < backoff; ++k) __builtin_amdgcn_s_sleep(4);
        }
        if (act == 2) pend = 0;
      }
      uint32_t cmd = kCmdLeave;
      if (__any(pend != 0)) {  // the lowest pending entry
        uint32_t k = 0;
        while (lane_u64(pend, k) == 0) ++k;
        const uint64_t pk = lane_u64(pend, k);
        const uint32_t bit = (uint32_t)__builtin_ctzll(pk);
        cmd = 64u * (word0 + k) + bit;
        if (lane == k) {
          pend &= ~(1ull << bit);
          ack ^= 1ull << bit;
        }
        t_seen = __builtin_amdgcn_s_memrealtime();
      }
      if (lane == 0) U.cmd = cmd;
    }
    __syncthreads();
    const uint32_t cmd = __builtin_amdgcn_readfirstlane(U.cmd);
    if (cmd == kCmdLeave) break;
    pp_serve(U, P, cmd, t_seen, spec);  // ends with a barrier: every wave has read U.cmd
    if (wave == 0) {
      const bool more = __any(pend != 0);
      if (lane == 0 && !more)
        __hip_atomic_store(P.last, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (wave != 0) return;
  // this unit's acknowledged parity back to the per-entry bytes, for the next launch
  for (uint32_t k = 0; k < nwords; ++k) {
    const uint64_t a = lane_u64(ack, k);
    const uint32_t e = 64u * (word0 + k) + lane;
    if (e >= base && e < base + E) P.ack[e] = (uint8_t)((a >> lane) & 1ull);
  }
  if (lane == 0) {
    __threadfence();
    if (atomicAdd(P.exited, 1u) == P.waves - 1u)
      __hip_atomic_store(P.exit_flag, (uint64_t)P.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace wgpp

namespace {

// host-side state of a ring entry
enum : uint32_t { kFree = 0, kBusy = 1, kOrphan = 2 };

// CPUs this process can keep busy: its affinity mask, capped by a cgroup v2 CPU quota
// (cpu.max "quota period"; "max" = none). A GPU box here allows 16 CPUs of time while the
// affinity covers 256.
inline uint32_t host_cpus() {
  cpu_set_t set;
  uint32_t n = 0;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = (uint32_t)CPU_COUNT(&set);
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    unsigned long long period = 0;
    if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
      const unsigned long long quota = strtoull(q, nullptr, 10);
      const uint32_t c = (uint32_t)std::max<unsigned long long>(1, quota / period);
      n = n ? std::min(n, c) : c;
    }
    fclose(f);
  }
  return n ? n : 1u;
}

struct PPServer {
  wg_ctx* c = nullptr;
  hipStream_t stream = nullptr;
  uint8_t* host = nullptr;   // pinned, fine-grained: in-slots | out-slots | done | bells | ctl | exit flag
  uint8_t* dev = nullptr;    // its device alias
  uint8_t* d_ack = nullptr;  // device: per-entry served doorbell parity
  uint32_t* d_exited = nullptr;  // device: {exited, quit} then the 8-B last-activity stamp
  std::unique_ptr<std::atomic<uint32_t>[]> state;  // per entry: kFree / kBusy / kOrphan
  std::unique_ptr<std::atomic<uint64_t>[]> pub;    // per entry: seq of its last publication
  std::atomic<uint64_t> calls{0};                  // call numbers (WG_PP_STAMPS builds: seq = call + 1)
  std::atomic<uint32_t> threads{0};                // calling threads seen (each takes the next wave)
  std::mutex launch_mu;
  std::atomic<uint64_t> running{0};  // gen of the launched kernel (0: none yet)
  uint64_t gen = 0;                  // guarded by launch_mu
  uint32_t waves = 16, idle_us = 20000, life_ms = 250;
  std::atomic<uint64_t> launches{0};
  // packets served, one counter per group of units (wg_batcher_stats sums them): callers of different
  // units do not write one shared line per call
  static constexpr uint32_t kShards = 16;
  struct alignas(64) Shard {
    std::atomic<uint64_t> n{0};
  };
  Shard served[kShards];
  uint64_t packets() const {
    uint64_t t = 0;
    for (const Shard& x : served) t += x.n.load(std::memory_order_relaxed);
    return t;
  }
  int fail_launches = 0;  // test hook (WG_PP_TEST_FAIL_LAUNCHES): refuse this many launches
  uint32_t spin_limit = 4096;     // polls of the completion word before a waiting caller sleeps (WG_PP_SPIN)
  // more calls in flight than this: 64 polls, then sleep (WG_PP_SPIN_CALLERS). Default: the CPUs the
  // process may use (host_cpus: its affinity, capped by a cgroup CPU quota), so polling callers never
  // outnumber them (64 / 128 callers on a 16-CPU quota: p999 74 / 88 ms polling, 0.3 / 0.5 ms not)
  uint32_t spin_callers = ~0u;
  std::atomic<uint32_t> active{0};  // calls between ticket and completion
  // callers asleep on a futex per entry, woken by the waker thread (pp_sleep / pp_waker)
  std::unique_ptr<std::atomic<uint32_t>[]> wake, waiting;
  std::atomic<uint32_t> sleepers{0};
  std::atomic<bool> waker_started{false};
  // waker threads (entry i served by waker i % count): one spends a futex wake (a syscall) per sleeping
  // caller's completion and capped the callers past the CPU count at about 1.2 GiB/s; four reached
  // 1.9-2.7 GiB/s for 24-128 callers with no quota throttling (profiles/r05_pp_wakers_ab.jsonl).
  // Default: a quarter of the CPUs the process may use, 1..4 (WG_PP_WAKERS overrides, 1..16)
  std::vector<std::thread> wakers;
  uint32_t n_wakers = 1;
  std::atomic<bool> waker_quit{false};
  std::mutex wmu;
  std::condition_variable wcv;
  bool stamps = false;            // WG_PP_CALL_STAMPS=1: per-call stage stamps (wg_pp_last_call), off by default
  uint64_t hold_counter = ~0ull;  // test hook (WG_PP_TEST_HOLD_COUNTER / _US): a call with this counter
  uint32_t hold_us = 0;           // sleeps between claiming its entry and publishing it

  uint8_t* in_slot(uint32_t i) { return host + (size_t)i * wgpp::kInSlot; }
  uint8_t* out_slot(uint32_t i) { return host + (size_t)wgpp::kRing * wgpp::kInSlot + (size_t)i * wgpp::kOutSlot; }
  size_t done_off() const { return (size_t)wgpp::kRing * (wgpp::kInSlot + wgpp::kOutSlot); }
  volatile uint64_t* done(uint32_t i) { return (volatile uint64_t*)(host + done_off()) + i; }
  size_t bell_off() const { return done_off() + (size_t)wgpp::kRing * 8; }
  uint64_t* bell(uint32_t k) { return (uint64_t*)(host + bell_off()) + k; }
  size_t ctl_off() const { return bell_off() + (size_t)wgpp::kBells * 8; }
  volatile wgpp::Ctl* ctl() { return (volatile wgpp::Ctl*)(host + ctl_off()); }
  size_t exit_off() const { return ctl_off() + sizeof(wgpp::Ctl); }
  volatile uint64_t* exit_flag() { return (volatile uint64_t*)(host + exit_off()); }
  size_t svc_off() const { return exit_off() + 64; }
  volatile uint64_t* svc(uint32_t i) { return (volatile uint64_t*)(host + svc_off()) + i; }
  size_t bytes() const { return svc_off() + (size_t)wgpp::kRing * 8; }
};

void pp_free(PPServer* S) {
  if (S->host) {
    memset(S->host, 0, S->bytes());  // keys of entries no server took (orphans) do not outlive the ring
    (void)hipHostFree(S->host);
  }
  if (S->d_ack) (void)hipFree(S->d_ack);
  if (S->d_exited) (void)hipFree(S->d_exited);
  if (S->stream) (void)hipStreamDestroy(S->stream);
}

int pp_get(wg_ctx* c, PPServer** out) {
  // the server exists after the context's first per-packet call: no lock after that (a mutex taken by
  // every call of 16 callers made them queue on it)
  if (PPServer* S = c->pp.load(std::memory_order_acquire)) {
    *out = S;
    return WG_OK;
  }
  std::lock_guard<std::mutex> lk(c->pp_mu);
  if (PPServer* S = c->pp.load(std::memory_order_relaxed)) {
    *out = S;
    return WG_OK;
  }
  DeviceGuard g(c->device);
  PPServer* S = new PPServer();
  S->c = c;
  S->state.reset(new std::atomic<uint32_t>[wgpp::kRing]);
  S->pub.reset(new std::atomic<uint64_t>[wgpp::kRing]);
  for (uint32_t i = 0; i < wgpp::kRing; ++i) {
    S->state[i].store(kFree);
    S->pub[i].store(0);
  }
  if (const char* e = getenv("WG_PP_TEST_FAIL_LAUNCHES")) S->fail_launches = atoi(e);
  if (const char* e = getenv("WG_PP_TEST_HOLD_COUNTER")) S->hold_counter = strtoull(e, nullptr, 0);
  if (const char* e = getenv("WG_PP_TEST_HOLD_US")) S->hold_us = (uint32_t)atoi(e);
  if (const char* e = getenv("WG_PP_SPIN")) S->spin_limit = (uint32_t)std::max(1, atoi(e));
  if (const char* e = getenv("WG_PP_CALL_STAMPS")) S->stamps = atoi(e) != 0;
  S->n_wakers = std::min(4u, std::max(1u, host_cpus() / 4u));
  if (const char* e = getenv("WG_PP_WAKERS")) S->n_wakers = (uint32_t)std::min(16, std::max(1, atoi(e)));
  S->spin_callers = host_cpus();
  if (const char* e = getenv("WG_PP_SPIN_CALLERS")) S->spin_callers = (uint32_t)std::max(0, atoi(e));
  S->wake.reset(new std::atomic<uint32_t>[wgpp::kRing]);
  S->waiting.reset(new std::atomic<uint32_t>[wgpp::kRing]);
  for (uint32_t i = 0; i < wgpp::kRing; ++i) {
    S->wake[i].store(0);
    S->waiting[i].store(0);
  }
  bool ok = hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking) == hipSuccess &&
            hipHostMalloc((void**)&S->host, S->bytes(), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer((void**)&S->dev, S->host, 0) == hipSuccess &&
            hipMalloc((void**)&S->d_ack, wgpp::kRing) == hipSuccess &&
            hipMalloc((void**)&S->d_exited, 16) == hipSuccess;
  if (ok) {
    memset(S->host, 0, S->bytes());
    ok = hipMemsetAsync(S->d_ack, 0, wgpp::kRing, S->stream) == hipSuccess &&
         hipStreamSynchronize(S->stream) == hipSuccess;  // not the null stream (see wg_ctx_create)
  }
  if (!ok) {
    pp_free(S);
    delete S;
    return fail(WG_ENOMEM, "per-packet server: pinned ring or device state could not be allocated");
  }
  c->pp.store(S, std::memory_order_release);
  *out = S;
  return WG_OK;
}

// (re)launch k_pp unless a launched kernel is still serving (its exit flag != its gen)
int pp_ensure(PPServer* S) {
  const uint64_t g = S->running.load(std::memory_order_acquire);
  if (g && *S->exit_flag() != g) return WG_OK;
  std::lock_guard<std::mutex> lk(S->launch_mu);
  const uint64_t g2 = S->running.load(std::memory_order_relaxed);
  if (g2 && *S->exit_flag() != g2) return WG_OK;
  DeviceGuard dg(S->c->device);
  wgpp::PPParams P{};
  P.in = S->dev;
  P.out = S->dev + (size_t)wgpp::kRing * wgpp::kInSlot;
  P.done = (uint64_t*)(S->dev + S->done_off());
  P.bell = (const uint64_t*)(S->dev + S->bell_off());
  P.ctl = (const wgpp::Ctl*)(S->dev + S->ctl_off());
  P.exit_flag = (uint64_t*)(S->dev + S->exit_off());
  P.svc = S->stamps ? (uint64_t*)(S->dev + S->svc_off()) : nullptr;
  P.ack = S->d_ack;
  P.exited = S->d_exited;
  P.quit = S->d_exited + 1;
  P.last = (uint64_t*)(S->d_exited + 2);
  P.waves = S->waves;
  P.gen = (uint32_t)(S->gen + 1);
  P.idle_ticks = (uint64_t)S->idle_us * 100u;
  P.life_ticks = (uint64_t)S->life_ms * 100000u;
  if (S->fail_launches > 0) {
    --S->fail_launches;
    return fail(WG_EDEVICE, "k_pp launch refused (WG_PP_TEST_FAIL_LAUNCHES test hook)");
  }
  HIPTRY(hipMemsetAsync(S->d_exited, 0, 16, S->stream));
  hipLaunchKernelGGL(wgpp::k_pp, dim3(S->waves), dim3(wgpp::kUnitThreads), 0, S->stream, P);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_pp launch: %s", hipGetErrorString(e));
  S->gen += 1;
  S->running.store(S->gen, std::memory_order_release);
  S->launches.fetch_add(1, std::memory_order_relaxed);
  return WG_OK;
}

void pp_stop(wg_ctx* c) {
  PPServer* S = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->pp_mu);
    S = c->pp.load(std::memory_order_relaxed);
    c->pp.store(nullptr, std::memory_order_relaxed);
  }
  if (!S) return;
  DeviceGuard g(c->device);
  {
    std::lock_guard<std::mutex> lk(S->wmu);
    S->waker_quit.store(true);
    S->wcv.notify_all();
  }
  for (std::thread& w : S->wakers)
    if (w.joinable()) w.join();
  S->ctl()->stop = 1;  // every wave sees it at its next poll and exits
  (void)hipStreamSynchronize(S->stream);
  pp_free(S);
  delete S;
}

// Stages of the calling thread's last per-packet call (wg_pp_last_call): host steady-clock
// nanoseconds, the device's service time from the entry's svc word, whether the caller slept on its
// futex, and whether this call relaunched the server.
struct PPCallStamps {
  uint64_t t_enter = 0, t_claimed = 0, t_published = 0, t_complete = 0, t_exit = 0;
  uint64_t svc_ticks = 0;
  uint32_t slept = 0, relaunched = 0;
};
thread_local PPCallStamps g_pp_last;

inline uint64_t pp_now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// The calling thread's place among the waves: a thread takes the next wave on its first call to a
// server and then claims that wave's entries in turn, so up to W concurrent callers never queue
// behind each other on one wave (a per-call hint, call k -> wave k mod W, put two of 16 callers on
// one wave about as often as not: 16 callers p50 13.5-14.4 us against 9.1-10.0 for one caller).
struct PPThread {
  const void* server = nullptr;
  uint32_t wave = 0, n = 0;
};
thread_local PPThread t_pp;

// Claim a free ring entry, starting at `start`; any free entry will do, since every wave serves
// whatever is published in its range. An ORPHAN entry (its caller failed after publishing) is
// taken over once the device has completed it.
uint32_t pp_claim(PPServer* S, uint32_t start, uint64_t k) {
  for (uint32_t spin = 0;; ++spin) {
    for (uint32_t d = 0; d < wgpp::kRing; ++d) {
      const uint32_t i = (start + d) % wgpp::kRing;
      // acquire: an ORPHAN entry's pub[i] (stored before the release that made it ORPHAN) is read below
      uint32_t st = S->state[i].load(std::memory_order_acquire);
      if (st == kOrphan && (__atomic_load_n((const uint64_t*)S->done(i), __ATOMIC_ACQUIRE) >> 8) ==
                               S->pub[i].load(std::memory_order_relaxed)) {
        if (S->state[i].compare_exchange_strong(st, kBusy, std::memory_order_acquire)) return i;
      } else if (st == kFree) {
        if (S->state[i].compare_exchange_strong(st, kBusy, std::memory_order_acquire)) return i;
      }
    }
    if (spin == 20000u && getenv("WG_PP_DEBUG")) {
      uint32_t nf = 0, nb = 0, no = 0;
      for (uint32_t i = 0; i < wgpp::kRing; ++i) {
        const uint32_t st = S->state[i].load();
        nf += st == kFree;
        nb += st == kBusy;
        no += st == kOrphan;
      }
      fprintf(stderr, "[wg_pp] call %llu of this thread finds no free entry: free %u busy %u orphan %u\n",
              (unsigned long long)k, nf, nb, no);
    }
    // more calls in flight than entries: wait for one to finish
    if (spin > 16u) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else std::this_thread::yield();
  }
}

// A packet longer than a slot: the host batch path with one descriptor (pageable copy
// pipeline, device key table).
int pp_big(wg_ctx* c, bool open, uint32_t key_slot, uint64_t counter, const uint8_t* src, uint32_t len, uint8_t* dst) {
  wg_pkt d{0, 0, counter, len, key_slot};
  if (!open) return host_transport(c, false, &d, 1, src, len, dst, (uint64_t)len + 16u, nullptr, len, 0);
  std::vector<uint8_t> pt(len);
  uint32_t st = 0;
  const int rc = host_transport(c, true, &d, 1, src, (uint64_t)len + 16u, pt.data(), len, &st, len, 0);
  if (rc != WG_OK) return rc;
  if (st != WG_PKT_OK) return 1;
  if (len) memcpy(dst, pt.data(), len);
  return WG_OK;
}

long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const struct timespec* t) {
  return syscall(SYS_futex, (uint32_t*)w, op, val, t, nullptr, 0);
}

// The wakers: while callers sleep (pp_sleep), n_wakers host threads poll their completion words (waker
// k the entries i with i % n_wakers == k) and wake each caller whose result has landed (a futex per
// entry); waker 0 also relaunches the server if it left.
// Sleeping callers burn no CPU: 64 or 128 callers spinning on 16 cores exhaust a CPU quota early in
// its period and are then all throttled until the next one (p999 ~70-90 ms).
void pp_waker(PPServer* S, uint32_t k0) {
  uint32_t iter = 0;
  const uint32_t nw = S->n_wakers;
  while (!S->waker_quit.load(std::memory_order_acquire)) {
    if (S->sleepers.load(std::memory_order_acquire) == 0) {
      std::unique_lock<std::mutex> lk(S->wmu);
      S->wcv.wait_for(lk, std::chrono::milliseconds(10), [S] {
        return S->sleepers.load() > 0 || S->waker_quit.load();
      });
      continue;
    }
    for (uint32_t i = k0; i < wgpp::kRing; i += nw) {
      if (!S->waiting[i].load(std::memory_order_acquire)) continue;
      const uint64_t d = __atomic_load_n((const uint64_t*)S->done(i), __ATOMIC_ACQUIRE);
      if ((d >> 8) == S->pub[i].load(std::memory_order_relaxed) && !S->wake[i].exchange(1))
        futex(&S->wake[i], FUTEX_WAKE_PRIVATE, 1, nullptr);
    }
    if ((++iter & 63u) == 0 && k0 == 0) (void)pp_ensure(S);  // a server that left while callers sleep
    for (int k = 0; k < 32; ++k) __builtin_ia32_pause();
  }
}

// A caller whose completion has not landed within spin_limit polls sleeps on its entry's futex; the
// waker (started with the first sleeper) wakes it. A 2-ms timeout re-checks the server on its own.
int pp_sleep(PPServer* S, uint32_t i, uint64_t seq, uint64_t* d_out) {
  // the mutex only to start the waker and to wake it from its idle wait (the first sleeper): with
  // 128 callers taking it for every sleep, the lock itself burnt the CPU quota
  if (!S->waker_started.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(S->wmu);
    if (S->wakers.empty())
      for (uint32_t k = 0; k < S->n_wakers; ++k) S->wakers.emplace_back(pp_waker, S, k);
    S->waker_started.store(true, std::memory_order_release);
  }
  S->waiting[i].store(1, std::memory_order_seq_cst);
  if (S->sleepers.fetch_add(1, std::memory_order_seq_cst) == 0) {
    std::lock_guard<std::mutex> lk(S->wmu);
    S->wcv.notify_all();
  }
  int rc = WG_OK;
  const struct timespec to = {0, 2 * 1000 * 1000};
  for (uint32_t naps = 0;; ++naps) {
    S->wake[i].store(0, std::memory_order_seq_cst);
    const uint64_t d = __atomic_load_n((const uint64_t*)S->done(i), __ATOMIC_ACQUIRE);
    if ((d >> 8) == seq) {
      *d_out = d;
      break;
    }
    if ((naps & 255u) == 255u) {  // about half a second without a completion: is the device alive?
      if ((rc = pp_ensure(S)) != WG_OK) break;
      const hipError_t e = hipStreamQuery(S->stream);
      if (e != hipSuccess && e != hipErrorNotReady) {
        rc = fail(WG_EDEVICE, "per-packet server: %s", hipGetErrorString(e));
        break;
      }
    }
    futex(&S->wake[i], FUTEX_WAIT_PRIVATE, 0, &to);
  }
  S->waiting[i].store(0, std::memory_order_release);
  S->sleepers.fetch_sub(1, std::memory_order_release);
  return rc;
}


int pp_submit(wg_ctx* c, bool open, uint32_t key_slot, uint64_t counter, const uint8_t* src, uint32_t len,
              uint8_t* dst) {
  // a slot without a key (never set, or zeroed by wg_keys_zero = clean()): refused, not sealed or opened
  // under the all-zero key (the reference's cipher() / decipher() throw once clean() closed the arena)
  if (!key_is_live(c, key_slot)) return fail(WG_ENOKEY, "key slot %u holds no key (zeroed or never set)", key_slot);
  if (len > wgpp::kPPMaxLen) return pp_big(c, open, key_slot, counter, src, len, dst);
  PPServer* S;
  int rc;
  if ((rc = pp_get(c, &S)) != WG_OK) return rc;
  // per-call stage stamps only with WG_PP_CALL_STAMPS (a stamped call writes into a dummy otherwise)
  PPCallStamps dummy;
  PPCallStamps& st = S->stamps ? g_pp_last : dummy;
  const bool stamp = S->stamps;
  st = PPCallStamps{};
  if (stamp) st.t_enter = pp_now_ns();
  uint32_t key[8];
  if (!key_snapshot(c, key_slot, key))  // zeroed since the check above
    return fail(WG_ENOKEY, "key slot %u holds no key (zeroed or never set)", key_slot);
  if (t_pp.server != (const void*)S) {
    t_pp.server = S;
    t_pp.wave = S->threads.fetch_add(1, std::memory_order_relaxed);
    t_pp.n = 0;
  }
  const uint32_t W = S->waves, E = wgpp::kRing / W;
  const uint32_t i = pp_claim(S, (t_pp.wave % W) * E + (t_pp.n++ % E), t_pp.n);
  // the completion word echoes seq: it must differ from every earlier publication of this entry, so the
  // entry's own count will do and callers share no counter (one shared line that 16 callers increment per
  // call cost each of them a cross-core transfer); tools/pp_stamps indexes its stamps by call number
#ifdef WG_PP_STAMPS
  const uint64_t seq = S->calls.fetch_add(1, std::memory_order_relaxed) + 1;
#else
  const uint64_t seq = S->pub[i].load(std::memory_order_relaxed) + 1;
#endif
  if (stamp) st.t_claimed = pp_now_ns();
  const uint64_t launches0 = S->launches.load(std::memory_order_relaxed);
  wgpp::Hdr* h = (wgpp::Hdr*)S->in_slot(i);
  h->seq = seq;
  h->counter = counter;
  h->mode = open ? WG_MODE_OPEN : WG_MODE_SEAL;
  h->len = len;
  memcpy(h->key, key, 32);
  memset(key, 0, sizeof key);
  if (len || open) memcpy(S->in_slot(i) + wgpp::kHdr, src, (size_t)len + (open ? 16u : 0u));
  if (counter == S->hold_counter && S->hold_us)  // test hook: a caller descheduled before publishing
    std::this_thread::sleep_for(std::chrono::microseconds(S->hold_us));
  S->pub[i].store(seq, std::memory_order_relaxed);
  // publish: toggle the entry's doorbell bit (a locked RMW, ordered after every byte above)
  __atomic_fetch_xor(S->bell(i >> 6), 1ull << (i & 63u), __ATOMIC_SEQ_CST);
  rc = pp_ensure(S);
  if (stamp) st.t_published = pp_now_ns();
  uint64_t d = 0;
  // with more calls in flight than spin_callers, a caller that polls for its whole round trip burns a
  // core the host does not have (and under a CPU quota every thread of the process then stalls until
  // the next quota period): it polls briefly and sleeps
  const uint32_t in_flight = S->active.fetch_add(1, std::memory_order_relaxed) + 1u;
  const uint32_t spin_limit = in_flight <= S->spin_callers ? S->spin_limit : 64u;
  for (uint64_t spin = 1; rc == WG_OK; ++spin) {
    d = __atomic_load_n((const uint64_t*)S->done(i), __ATOMIC_ACQUIRE);
    if ((d >> 8) == seq) break;
    if (spin > spin_limit) {  // past the usual round trip: sleep until the waker sees the completion
      st.slept = 1;
      rc = pp_sleep(S, i, seq, &d);
      break;
    }
    if ((spin & 255u) == 0) rc = pp_ensure(S);  // the server may have left (idle / lifetime) before it saw this entry
    __builtin_ia32_pause();
  }
  S->active.fetch_sub(1, std::memory_order_relaxed);
  if (stamp) {
    st.t_complete = pp_now_ns();
    st.relaunched = S->launches.load(std::memory_order_relaxed) != launches0 ? 1u : 0u;
  }
  int result = rc;
  if (rc == WG_OK) {
    if (stamp) st.svc_ticks = *S->svc(i);
    const uint32_t status = (uint32_t)(d & 0xffu);
    if (status == WG_PKT_OK) {
      if (open) {
        if (len) memcpy(dst, S->out_slot(i), len);
      } else {
        memcpy(dst, S->out_slot(i), (size_t)len + 16u);
      }
    } else {
      result = status == WG_PKT_BADTAG ? 1 : fail(WG_EDEVICE, "per-packet server refused the packet");
    }
    S->served[t_pp.wave % PPServer::kShards].n.fetch_add(1, std::memory_order_relaxed);
    memset(h->key, 0, 32);  // no key material left in the ring
    S->state[i].store(kFree, std::memory_order_release);
  } else {
    // published but not served (a refused launch, a stream error): the next server serves the
    // entry like any other (the key stays until then), and pp_claim takes it over once its
    // completion word has landed, so the entry is never lost
    S->state[i].store(kOrphan, std::memory_order_release);
  }
  if (stamp) st.t_exit = pp_now_ns();
  return result;
}

}  // namespace

extern "C" {

int wg_seal1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint8_t* out) {
  if (!c || (!pt && len) || !out) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  return pp_submit(c, false, key_slot, counter, pt, len, out);
}

int wg_open1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* in, uint32_t len, uint8_t* pt) {
  if (!c || !in || (!pt && len)) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  return pp_submit(c, true, key_slot, counter, in, len, pt);
}

// Stages of the calling thread's last wg_seal1 / wg_open1 (a diagnostic for latency outliers,
// tools/batcher_bench stamps=1), in nanoseconds: out[0] total, [1] claim (key snapshot + ring entry),
// [2] publish (header and payload copy + doorbell + server check), [3] wait (published -> completion
// observed by the caller, spinning or woken), [4] device service (the wave's doorbell sighting ->
// completion store), [5] copy-out and release, [6] slept on the futex (0/1), [7] this call relaunched
// the server (0/1). Packets past a ring slot (the host batch path) leave zeros.
int wg_pp_last_call(uint64_t* out, uint32_t n) {
  if (!out && n) return fail(WG_EINVAL, "NULL argument");
  const PPCallStamps& s = g_pp_last;
  const uint64_t v[8] = {s.t_exit - s.t_enter, s.t_claimed - s.t_enter, s.t_published - s.t_claimed,
                         s.t_complete - s.t_published, s.svc_ticks * 10u, s.t_exit - s.t_complete, s.slept,
                         s.relaunched};
  for (uint32_t k = 0; k < n && k < 8u; ++k) out[k] = s.t_enter ? v[k] : 0u;
  return WG_OK;
}

int wg_pp_config(wg_ctx* c, uint32_t waves, uint32_t idle_us) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (waves == 0 || waves > wgpp::kMaxWaves || (waves & (waves - 1u)))
    return fail(WG_EINVAL, "waves must be a power of two in 1..%u", wgpp::kMaxWaves);
  PPServer* S;
  int rc;
  if ((rc = pp_get(c, &S)) != WG_OK) return rc;
  std::lock_guard<std::mutex> lk(S->launch_mu);
  // the wave count fixes which wave serves which entries: change it only between kernels (the
  // served parity is kept per entry, so no call in flight is lost across the change)
  const uint64_t g = S->running.load();
  if (g && *S->exit_flag() != g) {
    S->ctl()->stop = 1;
    (void)hipStreamSynchronize(S->stream);
    S->ctl()->stop = 0;
  }
  S->waves = waves;
  S->idle_us = idle_us ? idle_us : 20000;
  return WG_OK;
}

// round-2 name and arguments (max_batch, window_us of the launch-per-batch batcher, which the
// persistent server replaced): accepted and ignored
int wg_batcher_config(wg_ctx* c, uint32_t max_batch, uint32_t window_us) {
  (void)max_batch;
  (void)window_us;
  if (!c) return fail(WG_EINVAL, "NULL context");
  return WG_OK;
}

int wg_batcher_stats(wg_ctx* c, uint64_t* launches, uint64_t* packets) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  uint64_t l = 0, p = 0;
  {
    std::lock_guard<std::mutex> lk(c->pp_mu);
    if (PPServer* S = c->pp.load()) {
      l = S->launches.load();
      p = S->packets();
    }
  }
  if (launches) *launches = l;
  if (packets) *packets = p;
  return WG_OK;
}

}  // extern "C"
