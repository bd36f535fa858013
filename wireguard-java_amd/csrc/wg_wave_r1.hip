// wg_wave_r1.hip — round-1 transport kernel k_wave<MODE, 5, 1>, kept only as the A/B
// baseline for k_transport (wg_ctx_set_kernel(ctx, "wave1", ...)); not the product default.
#pragma once
#include "wg_tile.hip"

namespace wgk {
#define WG_PH_STORE_WAVE(idx) do {} while (0)
#define WG_PH_DECL
#define WG_PH_MARK() do {} while (0)
#define WG_PH_ADD(k) do {} while (0)
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
// Progress-based wave priority: a wave drops its issue priority as it completes
// rounds (3, 2, 1, then 0), so the SIMD's oldest-first arbitration no longer lets
// one wave run ahead while the others idle at the end of a launch.
__device__ __forceinline__ void progress_prio(uint32_t done_rounds) {
  if (done_rounds == 0) __builtin_amdgcn_s_setprio(3);
  else if (done_rounds == 1) __builtin_amdgcn_s_setprio(2);
  else if (done_rounds == 2) __builtin_amdgcn_s_setprio(1);
  else if (done_rounds == 3) __builtin_amdgcn_s_setprio(0);
}
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
template __global__ void k_wave<WG_MODE_SEAL, 5, 1>(StreamParams);
template __global__ void k_wave<WG_MODE_OPEN, 5, 1>(StreamParams);
}  // namespace wgk
