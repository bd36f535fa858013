// wg_kernels.h — launch parameters shared by the kernels (wg_tile.hip, wg_wave_r1.hip) and wg_capi.hip.
#pragma once
#include <stdint.h>

#include "../../include/wgaead.h"

#define WG_TPB 256u  // threads per workgroup: 4 waves of 64

namespace wgk {

struct TileParams {
  const void* desc;  // wg_pkt* (transport) or wg_aead_desc* (general)
  uint32_t n;
  uint32_t max_len;  // every valid packet has len <= max_len (== max_len when uniform)
  const uint8_t* in;
  uint64_t in_size;
  uint8_t* out;
  uint64_t out_size;
  const uint8_t* aad;
  uint64_t aad_size;
  const uint32_t* keys;  // key table, 8 words per slot
  uint32_t key_slots;
  uint32_t* status;  // open: per-packet WG_PKT_*
  // tile plan
  uint32_t uniform;     // 1: closed-form tiles of `ppt` packets of `nb_uniform` blocks
  uint32_t ppt;
  uint32_t nb_uniform;
  uint32_t nb_magic;    // ceil(2^32 / nb_uniform): q = umulhi(b, magic)
  const uint32_t* tile_start;  // non-uniform: [ntiles + 1]
  const uint32_t* blk_prefix;  // non-uniform: [n + 1] exclusive block prefix
  const uint32_t* ntiles_dev;  // non-uniform: tile count computed on device
  uint32_t max_tile_pkts;      // LDS sizing of the per-packet records
  uint32_t poly_g;             // lanes per packet in the Poly1305 phase
};

template <int MODE, bool GENERAL>
__global__ void k_tile(TileParams P);
template <int MODE, bool GENERAL>
__global__ void k_plan_count(const void* desc, uint32_t n, uint32_t max_len, uint32_t* nb);
__global__ void k_plan_tiles(const uint32_t* prefix, uint32_t n, uint32_t C, uint32_t* tile_start, uint32_t* ntiles,
                             uint32_t max_tiles);

// LDS bytes of the per-packet records of a tile holding up to `mp` packets
// (128-byte record + 4-byte first-block index each, plus one); the payload
// image follows, 16-byte aligned (see tile_rec in wg_tile.hip).
__host__ __device__ inline uint32_t tile_header_bytes(uint32_t mp) {
  uint32_t b = 128u * mp + 4u * (mp + 1);
  return (b + 15u) & ~15u;
}

}  // namespace wgk
