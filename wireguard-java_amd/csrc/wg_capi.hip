// wg_capi.hip — the C-ABI of libwgaead.so (include/wgaead.h).
//
// Host runtime around the gfx950 kernels: per-device context (stream, device key
// table, plan workspace, staging buffers), launch planning, the device-pointer
// batch API, the host-pointer convenience API and the on-device self test.
// No CPU crypto lives here: every seal/open/cipher/MAC runs in wg_kernels.hip,
// and every entry point fails with WG_EDEVICE when no HIP device is usable.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "wg_kernels.hip"
#include "wg_lane.h"

namespace {

thread_local std::string g_err;
#ifdef WG_DIAG
uint64_t* g_stamps = nullptr;
#endif

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPTRY(expr)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return fail(WG_EDEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                       \
  } while (0)

// grow-only device buffer
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return WG_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&p, want) != hipSuccess) return fail(WG_ENOMEM, "hipMalloc(%zu) failed", want);
    cap = want;
    return WG_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct wg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;      // host path: H2D
  hipStream_t copy_out_stream = nullptr;  // host path: D2H
  hipEvent_t ev_desc = nullptr, ev_in = nullptr, ev_kernel = nullptr;
  uint32_t key_slots = 0;
  uint32_t* keys = nullptr;  // device key table
  const uint32_t* receivers = nullptr;  // device receiver_index per key slot (WG_F_FRAME; caller-owned)
  // non-uniform plan workspace
  DevBuf plan_nb, plan_prefix, plan_tiles, plan_ntiles, plan_tmp;
  DevBuf sink;  // k_coop scratch
  // transport kernel for this context (wg_ctx_set_kernel); kern == 0: the process
  // default from WG_TRANSPORT_KERNEL (tunables())
  int kern = 0;
  uint32_t kern_k = 2, kern_v = 0;
  // host-API staging
  DevBuf h_desc, h_in, h_out, h_aad, h_status, h_keys;
  std::mutex mu;  // serialises host-API calls and plan workspace reuse
  // timing
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  double timed_ms = 0;
  uint64_t timed_launches = 0;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <int MODE>
uint32_t host_pkt_blocks(uint32_t len) {
  uint32_t nb = (len + 63u) / 64u;
  return (MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN) ? nb + 1u : nb;
}

constexpr uint32_t kLdsBudget = 64u * 1024u;  // per workgroup; keeps >= 2 tiles per CU

// Tunables (environment, read once): WG_TILE_PASSES = max workgroup passes per
// uniform tile (1..4, default 2); WG_POLY_WAVES = waves the Poly1305 phase spreads
// a tile's packets over (1..4, default 4); WG_POLY_GMAX = cap on lanes per packet.
struct Tunables {
  uint32_t tile_passes = 2, poly_waves = 4, poly_gmax = 16;
  uint32_t stream_ppw_uniform = 8, stream_ppw_mixed = 16;  // packets per wave in k_stream
  int use_tile_for_transport = 0;                           // 1: route transport batches to k_tile
  int stream_variant = 1;                                   // k_stream<MODE, V> variant bits
  int use_pipe = 0;                                         // k_pipe (software-pipelined) for transport
  int use_lean = 0;                                         // k_lean (state in LDS) for transport
  uint32_t stream_lds_pad = 0;                              // dynamic LDS per wave: caps occupancy
  int use_wave = 1;                                         // k_wave (8 waves/SIMD layout): the default
  int wave_variant = 5;                                     // k_wave<SEAL, V, WPG>: prefetch + progress priority
  int wave_variant_open = 5;                                // k_wave<OPEN, V, WPG>
  int wave_wpg = 1;                                         // k_wave waves per workgroup (1, 4, 8)
  int use_lane = 0;                                         // k_lane (K lanes per packet, contiguous block ranges)
  int lane_k = 2;                                           // k_lane lanes per packet (1, 2, 4, 8)
  int use_ws = 0;                                           // k_ws (warp-specialised producer/consumer waves)
  int use_coop = 0;                                         // k_coop (k_lane ranges + cooperative coalesced IO)
  int use_quad = 0;                                         // k_quad (k_lane K=4 with quad-cooperative IO)
  int quad_variant = 0;                                     // k_quad<MODE, V> variant bits
  int lane_variant = 5;                                     // k_lane<MODE, K, V> variant bits
  Tunables() {
    if (const char* e = getenv("WG_STREAM_LDS_PAD")) stream_lds_pad = (uint32_t)std::min(65536, std::max(0, atoi(e)));
    if (const char* e = getenv("WG_STREAM_PPW")) stream_ppw_uniform = stream_ppw_mixed = std::max(1, atoi(e));
    if (const char* e = getenv("WG_STREAM_PPW_MIXED")) stream_ppw_mixed = std::max(1, atoi(e));
    if (const char* e = getenv("WG_TRANSPORT_KERNEL")) {
      use_tile_for_transport = strcmp(e, "tile") == 0;
      use_pipe = strcmp(e, "pipe") == 0;
      use_lean = strcmp(e, "lean") == 0;
      use_wave = strcmp(e, "wave") == 0 || strcmp(e, "default") == 0;
      use_lane = strcmp(e, "lane") == 0;
      use_quad = strcmp(e, "quad") == 0;
      use_coop = strcmp(e, "coop") == 0;
      use_ws = strcmp(e, "ws") == 0;
    }
    if (const char* e = getenv("WG_WAVE_VARIANT")) wave_variant = wave_variant_open = atoi(e) & 255;
    if (const char* e = getenv("WG_WAVE_VARIANT_OPEN")) wave_variant_open = atoi(e) & 255;
    if (const char* e = getenv("WG_WAVE_WPG")) {
      const int g = atoi(e);
      wave_wpg = (g == 4 || g == 8 || g == 16) ? g : 1;
    }
    if (const char* e = getenv("WG_LANE_K")) {
      const int k = atoi(e);
      lane_k = (k == 1 || k == 2 || k == 4 || k == 8) ? k : 2;
    }
    if (const char* e = getenv("WG_LANE_VARIANT")) lane_variant = atoi(e) & 63;
    if (const char* e = getenv("WG_QUAD_VARIANT")) quad_variant = atoi(e) & 63;
    if (const char* e = getenv("WG_STREAM_VARIANT")) stream_variant = atoi(e) & 127;
    if (const char* e = getenv("WG_TILE_PASSES")) tile_passes = std::min(4u, std::max(1u, (uint32_t)atoi(e)));
    if (const char* e = getenv("WG_POLY_WAVES")) poly_waves = std::min(4u, std::max(1u, (uint32_t)atoi(e)));
    if (const char* e = getenv("WG_POLY_GMAX")) poly_gmax = std::min(64u, std::max(1u, (uint32_t)atoi(e)));
  }
};
const Tunables& tunables() {
  static Tunables t;
  return t;
}

// lanes per packet for the Poly1305 phase: spread the tile's packets over
// `poly_waves` waves (groups never straddle a wave)
uint32_t choose_poly_g(uint32_t ppt) {
  if (ppt == 0) return 1;
  const Tunables& t = tunables();
  uint32_t per_wave = (ppt + t.poly_waves - 1) / t.poly_waves;
  uint32_t g = 64u / per_wave;
  if (g < 1) g = 1;
  if (g > t.poly_gmax) g = t.poly_gmax;
  return g;
}

void record_start(wg_ctx* c, hipStream_t s, hipEvent_t* ev) {
  *ev = nullptr;
  if (!c->timing) return;
  hipEvent_t a;
  if (hipEventCreate(&a) != hipSuccess) return;
  (void)hipEventRecord(a, s);
  *ev = a;
}
void record_end(wg_ctx* c, hipStream_t s, hipEvent_t a) {
  if (!a) return;
  hipEvent_t b;
  if (hipEventCreate(&b) != hipSuccess) return;
  (void)hipEventRecord(b, s);
  c->events.emplace_back(a, b);
}

template <int MODE, bool GENERAL>
int launch_tiles(wg_ctx* c, const void* desc, uint32_t n, const uint8_t* in, uint64_t in_size, const uint8_t* aad,
                 uint64_t aad_size, uint8_t* out, uint64_t out_size, uint32_t* status, uint32_t max_len,
                 uint32_t flags, hipStream_t s) {
  if (n == 0) return WG_OK;
  if (!desc || (((uintptr_t)desc) & 15u)) return fail(WG_EINVAL, "descriptor array must be non-NULL and 16-byte aligned");
  if (!in && MODE != WG_MODE_MAC) return fail(WG_EINVAL, "NULL input buffer");
  if (!out) return fail(WG_EINVAL, "NULL output buffer");
  if (max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", max_len);
  wgk::TileParams P{};
  P.desc = desc;
  P.n = n;
  P.max_len = max_len;
  P.in = in;
  P.in_size = in ? in_size : 0;
  P.out = out;
  P.out_size = out_size;
  P.aad = aad;
  P.aad_size = aad ? aad_size : 0;
  P.keys = c->keys;
  P.key_slots = c->key_slots;
  P.status = status;
  const uint32_t aead_extra = (MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN) ? 1u : 0u;
  uint32_t grid = 0, lds = 0;
  if (flags & WG_F_UNIFORM) {
    const uint32_t nb = host_pkt_blocks<MODE>(max_len);
    uint32_t ppt = 1;
    if (nb == 0) {
      ppt = 64;
    } else if (nb <= WG_TPB) {
      // pick the tile size (1 or 2 passes of the workgroup) that idles fewest lanes
      double best = -1;
      for (uint32_t k = 1; k <= tunables().tile_passes; ++k) {
        uint32_t p = k * WG_TPB / nb;
        uint32_t img = p * (nb - aead_extra) * 64u;
        if (p == 0 || wgk::tile_header_bytes(p) + img > kLdsBudget) continue;
        double util = (double)(p * nb) / (double)(k * WG_TPB);
        if (util > best + 1e-9) { best = util; ppt = p; }
      }
    }
    if (ppt > n) ppt = n;
    P.uniform = 1;
    P.ppt = ppt;
    P.nb_uniform = nb;
    P.nb_magic = nb > 1 ? (uint32_t)((((uint64_t)1 << 32) + nb - 1) / nb) : 0u;
    P.max_tile_pkts = ppt;
    P.poly_g = choose_poly_g(ppt);
    lds = wgk::tile_header_bytes(ppt) + ppt * (nb > aead_extra ? nb - aead_extra : 0u) * 64u;
    grid = (n + ppt - 1) / ppt;
  } else {
    // device plan: block counts -> exclusive scan -> start-owned tiles of C blocks
    const uint32_t C = WG_TPB;
    const uint32_t max_nb = host_pkt_blocks<MODE>(max_len);
    const uint64_t max_tiles64 = ((uint64_t)n * std::max<uint32_t>(max_nb, 1u) + C - 1) / C;
    if (max_tiles64 > 0x7fffffffull) return fail(WG_EINVAL, "batch too large");
    const uint32_t max_tiles = (uint32_t)max_tiles64;
    int rc;
    if ((rc = c->plan_nb.ensure(sizeof(uint32_t) * (n + 1))) != WG_OK) return rc;
    if ((rc = c->plan_prefix.ensure(sizeof(uint32_t) * (n + 1))) != WG_OK) return rc;
    if ((rc = c->plan_tiles.ensure(sizeof(uint32_t) * (max_tiles + 2))) != WG_OK) return rc;
    if ((rc = c->plan_ntiles.ensure(sizeof(uint32_t))) != WG_OK) return rc;
    size_t tmp = 0;
    HIPTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (uint32_t*)c->plan_nb.p, (uint32_t*)c->plan_prefix.p,
                                            (int)(n + 1), s));
    if ((rc = c->plan_tmp.ensure(tmp)) != WG_OK) return rc;
    hipLaunchKernelGGL((wgk::k_plan_count<MODE, GENERAL>), dim3((n + 1 + 255) / 256), dim3(256), 0, s, desc, n,
                       max_len, (uint32_t*)c->plan_nb.p);
    HIPTRY(hipGetLastError());
    HIPTRY(hipcub::DeviceScan::ExclusiveSum(c->plan_tmp.p, tmp, (uint32_t*)c->plan_nb.p, (uint32_t*)c->plan_prefix.p,
                                            (int)(n + 1), s));
    hipLaunchKernelGGL(wgk::k_plan_tiles, dim3((max_tiles + 1 + 255) / 256), dim3(256), 0, s,
                       (const uint32_t*)c->plan_prefix.p, n, C, (uint32_t*)c->plan_tiles.p,
                       (uint32_t*)c->plan_ntiles.p, max_tiles);
    HIPTRY(hipGetLastError());
    P.uniform = 0;
    P.tile_start = (const uint32_t*)c->plan_tiles.p;
    P.blk_prefix = (const uint32_t*)c->plan_prefix.p;
    P.ntiles_dev = (const uint32_t*)c->plan_ntiles.p;
    P.max_tile_pkts = C;
    P.poly_g = 8;
    lds = wgk::tile_header_bytes(C) + (C + max_nb) * 64u;
    grid = max_tiles;
  }
  if (lds > 160u * 1024u) return fail(WG_E2BIG, "tile needs %u bytes of LDS", lds);
#ifdef WG_DIAG
  P.stamps = g_stamps;
#endif
  hipEvent_t ev;
  record_start(c, s, &ev);
  hipLaunchKernelGGL((wgk::k_tile<MODE, GENERAL>), dim3(grid), dim3(WG_TPB), lds, s, P);
  hipError_t e = hipGetLastError();
  record_end(c, s, ev);
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_tile launch: %s", hipGetErrorString(e));
  return WG_OK;
}

// k_wave<MODE, V, G> for the variant bits V (see wg_kernels.hip) and G waves per workgroup
template <int MODE, int G>
void launch_wave(int V, uint32_t wgrid, hipStream_t s, const wgk::StreamParams& P) {
  switch (V) {
#define WG_WV(VV) \
  case VV: hipLaunchKernelGGL((wgk::k_wave<MODE, VV, G>), dim3(wgrid), dim3(64 * G), 0, s, P); break;
    WG_WV(0) WG_WV(1) WG_WV(3) WG_WV(7) WG_WV(13) WG_WV(15) WG_WV(65) WG_WV(67) WG_WV(69) WG_WV(71)
    WG_WV(132) WG_WV(133) WG_WV(134) WG_WV(135)
#undef WG_WV
    default: hipLaunchKernelGGL((wgk::k_wave<MODE, 5, G>), dim3(wgrid), dim3(64 * G), 0, s, P); break;
  }
}

// k_lane<MODE, K, V>: K lanes per packet, 256-thread workgroups
template <int MODE, int K>
void launch_lane_k(int V, uint32_t n, hipStream_t s, const wgk::StreamParams& P) {
  switch (V) {
#define WG_LV(VV)                                                                                        \
  case VV: {                                                                                             \
    constexpr uint32_t T = wgk::lane_wg_threads<VV>();                                                  \
    const uint32_t grid = (uint32_t)(((uint64_t)n * K + T - 1u) / T);                                   \
    hipLaunchKernelGGL((wgk::k_lane<MODE, K, VV>), dim3(grid), dim3(T), 0, s, P);                        \
  } break;
    WG_LV(1) WG_LV(3) WG_LV(7)
#undef WG_LV
#define WG_LA(VV)                                                                                        \
  case VV:                                                                                               \
    if constexpr (K == 2) {                                                                              \
      const uint32_t grid = (uint32_t)(((uint64_t)n * K + 63u) / 64u);                                   \
      hipLaunchKernelGGL((wgk::k_lane<MODE, K, VV>), dim3(grid), dim3(64), 0, s, P);                     \
    }                                                                                                    \
    break;
    WG_LA(13) WG_LA(21) WG_LA(29) WG_LA(53)
#undef WG_LA
    default: {
      const uint32_t grid = (uint32_t)(((uint64_t)n * K + 63u) / 64u);
      hipLaunchKernelGGL((wgk::k_lane<MODE, K, 5>), dim3(grid), dim3(64), 0, s, P);
    } break;
  }
}
template <int MODE>
void launch_lane(int K, int V, uint32_t n, hipStream_t s, const wgk::StreamParams& P) {
  switch (K) {
    case 1: launch_lane_k<MODE, 1>(V, n, s, P); break;
    case 4: launch_lane_k<MODE, 4>(V, n, s, P); break;
    case 8: launch_lane_k<MODE, 8>(V, n, s, P); break;
    default: launch_lane_k<MODE, 2>(V, n, s, P); break;
  }
}

// transport kernels selectable per context (wg_ctx_set_kernel) or per process
// (WG_TRANSPORT_KERNEL); k_wave is the default
enum Kern { KERN_DEFAULT = 0, KERN_WAVE, KERN_STREAM, KERN_TILE, KERN_LANE, KERN_QUAD, KERN_COOP, KERN_WS, KERN_PIPE, KERN_LEAN };
struct KernChoice {
  int kind;
  uint32_t k;     // lanes per packet (lane, coop, ws)
  int v_seal;     // variant bits (wave: per mode)
  int v_open;
};
int kern_from_name(const char* e) {
  if (!e || !strcmp(e, "default") || !strcmp(e, "wave")) return KERN_WAVE;
  if (!strcmp(e, "stream")) return KERN_STREAM;
  if (!strcmp(e, "tile")) return KERN_TILE;
  if (!strcmp(e, "lane")) return KERN_LANE;
  if (!strcmp(e, "quad")) return KERN_QUAD;
  if (!strcmp(e, "coop")) return KERN_COOP;
  if (!strcmp(e, "ws")) return KERN_WS;
  if (!strcmp(e, "pipe")) return KERN_PIPE;
  if (!strcmp(e, "lean")) return KERN_LEAN;
  return -1;
}
KernChoice kern_choice(const wg_ctx* c) {
  const Tunables& T = tunables();
  if (c->kern != KERN_DEFAULT) {
    const int v = (int)c->kern_v;
    return {c->kern, c->kern_k, v, v};
  }
  int kind = KERN_STREAM;
  if (T.use_tile_for_transport) kind = KERN_TILE;
  else if (T.use_ws) kind = KERN_WS;
  else if (T.use_coop) kind = KERN_COOP;
  else if (T.use_quad) kind = KERN_QUAD;
  else if (T.use_lane) kind = KERN_LANE;
  else if (T.use_wave) kind = KERN_WAVE;
  else if (T.use_lean) kind = KERN_LEAN;
  else if (T.use_pipe) kind = KERN_PIPE;
  if (kind == KERN_WAVE) return {kind, 1u, T.wave_variant, T.wave_variant_open};
  if (kind == KERN_QUAD) return {kind, 4u, T.quad_variant, T.quad_variant};
  if (kind == KERN_STREAM) return {kind, 8u, T.stream_variant, T.stream_variant};
  return {kind, (uint32_t)T.lane_k, T.lane_variant, T.lane_variant};
}

// the caller's stream as-is: NULL is HIP's default (null) stream, like every HIP API;
// pass wg_ctx_stream(ctx) to use the context's own non-blocking stream
// Transport seal/open through k_stream (one wave per workgroup, 8 packet slots).
template <int MODE>
int launch_stream(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                  uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, hipStream_t s) {
  if (n == 0) return WG_OK;
  if (!desc || (((uintptr_t)desc) & 15u)) return fail(WG_EINVAL, "descriptor array must be non-NULL and 16-byte aligned");
  if (!in || !out) return fail(WG_EINVAL, "NULL buffer");
  if (max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", max_len);
  wgk::StreamParams P{};
  P.desc = desc;
  P.n = n;
  P.ppw = (flags & WG_F_UNIFORM) ? tunables().stream_ppw_uniform : tunables().stream_ppw_mixed;
  P.max_len = max_len;
  P.key_slots = c->key_slots;
  P.in = in;
  P.in_size = in_size;
  P.out = out;
  P.out_size = out_size;
  P.keys = c->keys;
  P.status = status;
#ifdef WG_DIAG
  P.stamps = g_stamps;
#endif
  const KernChoice ch = kern_choice(c);
  const int CV = MODE == WG_MODE_OPEN ? ch.v_open : ch.v_seal;
  const uint32_t K = ch.k == 1 ? 1u : (ch.k == 4 ? 4u : (ch.k == 8 ? 8u : 2u));
  if (ch.kind == KERN_COOP || ch.kind == KERN_WS) {
    int rc;
    if ((rc = c->sink.ensure(wgk::kCoopSinkBytes)) != WG_OK) return rc;
    P.sink = (uint8_t*)c->sink.p;
  }
  const uint32_t grid = (n + P.ppw - 1) / P.ppw;
  const uint32_t pad = tunables().stream_lds_pad;
  hipEvent_t ev;
  record_start(c, s, &ev);
  if (ch.kind == KERN_WS && (flags & WG_F_UNIFORM) && K <= 4u) {
    const uint32_t wgrid = (uint32_t)(((uint64_t)n * K + 511u) / 512u);
    if (K == 1) hipLaunchKernelGGL((wgk::k_ws<MODE, 1>), dim3(wgrid), dim3(640), 0, s, P);
    else if (K == 4) hipLaunchKernelGGL((wgk::k_ws<MODE, 4>), dim3(wgrid), dim3(640), 0, s, P);
    else hipLaunchKernelGGL((wgk::k_ws<MODE, 2>), dim3(wgrid), dim3(640), 0, s, P);
    if (MODE == WG_MODE_OPEN && status)
      hipLaunchKernelGGL(wgk::k_ws_scrub, dim3((uint32_t)(((uint64_t)n * 16u + 255u) / 256u)), dim3(256), 0, s, P);
  } else if (ch.kind == KERN_COOP && K <= 4u) {
    const uint32_t cgrid = (uint32_t)(((uint64_t)n * K + 63u) / 64u);
    if (K == 2 && CV == 8) hipLaunchKernelGGL((wgk::k_coop<MODE, 2, 8>), dim3(cgrid), dim3(64), 0, s, P);
    else if (K == 2 && CV == 48) hipLaunchKernelGGL((wgk::k_coop<MODE, 2, 48>), dim3(cgrid), dim3(64), 0, s, P);
    else if (K == 2 && CV == 16) hipLaunchKernelGGL((wgk::k_coop<MODE, 2, 16>), dim3(cgrid), dim3(64), 0, s, P);
    else if (K == 1) hipLaunchKernelGGL((wgk::k_coop<MODE, 1, 0>), dim3(cgrid), dim3(64), 0, s, P);
    else if (K == 4) hipLaunchKernelGGL((wgk::k_coop<MODE, 4, 0>), dim3(cgrid), dim3(64), 0, s, P);
    else hipLaunchKernelGGL((wgk::k_coop<MODE, 2, 0>), dim3(cgrid), dim3(64), 0, s, P);
  } else if (ch.kind == KERN_QUAD) {
    const uint32_t qgrid = (uint32_t)(((uint64_t)n * 4u + 63u) / 64u);
    switch (CV) {
      case 2: hipLaunchKernelGGL((wgk::k_quad<MODE, 2>), dim3(qgrid), dim3(64), 0, s, P); break;
      case 16: hipLaunchKernelGGL((wgk::k_quad<MODE, 16>), dim3(qgrid), dim3(64), 0, s, P); break;
      case 48: hipLaunchKernelGGL((wgk::k_quad<MODE, 48>), dim3(qgrid), dim3(64), 0, s, P); break;
      default: hipLaunchKernelGGL((wgk::k_quad<MODE, 0>), dim3(qgrid), dim3(64), 0, s, P); break;
    }
  } else if (ch.kind == KERN_LANE) {
    launch_lane<MODE>((int)K, CV, n, s, P);
  } else if (ch.kind == KERN_WAVE) {
    const int G = tunables().wave_wpg;
    const int V = CV;
    const uint32_t wgrid = (grid + G - 1) / G;
    switch (G) {
      case 4: launch_wave<MODE, 4>(V, wgrid, s, P); break;
      case 8: launch_wave<MODE, 8>(V, wgrid, s, P); break;
      case 16: launch_wave<MODE, 16>(V, wgrid, s, P); break;
      default: launch_wave<MODE, 1>(V, wgrid, s, P); break;
    }
  } else if (ch.kind == KERN_LEAN) {
    hipLaunchKernelGGL((wgk::k_lean<MODE>), dim3(grid), dim3(64), 0, s, P);
  } else if (ch.kind == KERN_PIPE) {
    hipLaunchKernelGGL((wgk::k_pipe<MODE, 0>), dim3(grid), dim3(64), 0, s, P);
  } else switch (ch.kind == KERN_STREAM ? CV : tunables().stream_variant) {
#define WG_CASE(V) \
  case V: hipLaunchKernelGGL((wgk::k_stream<MODE, V>), dim3(grid), dim3(64), pad, s, P); break;
    WG_CASE(0) WG_CASE(1) WG_CASE(2) WG_CASE(3) WG_CASE(4) WG_CASE(5) WG_CASE(6) WG_CASE(7)
    WG_CASE(9) WG_CASE(11) WG_CASE(15) WG_CASE(17) WG_CASE(33) WG_CASE(49) WG_CASE(65) WG_CASE(73)
    default: return fail(WG_EINVAL, "k_stream variant %d not built", ch.kind == KERN_STREAM ? CV : tunables().stream_variant);
#undef WG_CASE
  }
  hipError_t e = hipGetLastError();
  record_end(c, s, ev);
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_stream launch: %s", hipGetErrorString(e));
  return WG_OK;
}

template <int MODE>
int launch_transport(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                     uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, hipStream_t s) {
  if (kern_choice(c).kind == KERN_TILE)
    return launch_tiles<MODE, false>(c, desc, n, in, in_size, nullptr, 0, out, out_size, status, max_len, flags, s);
  return launch_stream<MODE>(c, desc, n, in, in_size, out, out_size, status, max_len, flags, s);
}

hipStream_t pick_stream(wg_ctx*, void* stream) { return (hipStream_t)stream; }

// ---- wire framing (TransportPacket.java:18-35) ------------------------------
// One thread per packet: 16 header bytes against ~1.4 KB of AEAD work, so these
// are launch-bound, not bandwidth-bound; bytes are moved with 4-B or 1-B vector
// stores depending on the header's alignment (stride 1452 leaves it 4-aligned).
__global__ void __launch_bounds__(256) k_frame_seal(const wg_pkt* __restrict__ d, uint32_t n,
                                                    const uint32_t* __restrict__ rx, uint32_t slots,
                                                    uint8_t* __restrict__ out, uint64_t out_size) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const wg_pkt p = d[i];
  if (p.out_off < 16 || p.out_off > out_size || p.key_slot >= slots) return;
  wgk::put_header(out + p.out_off - 16, rx[p.key_slot], p.counter);
}

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
  bool ok = wl >= 32 && o <= wire_size && (uint64_t)wl <= wire_size - o &&
            (uint64_t)wl - 32 <= wire_size - o - wl;
  if (ok) {
    const uint8_t* h = wire + o;
    uint32_t w[4];
    if ((((uintptr_t)h) & 3u) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = ((const uint32_t*)h)[k];
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) |
               ((uint32_t)h[4 * k + 3] << 24);
    }
    ok = (w[0] & 0xffu) == 4u;  // only the type byte is checked (UndecryptedIncomingTransport.java:24-26)
    if (ok) {
      p.counter = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
      p.len = wl - 32;
    }
  }
  d[i] = p;
  if (st) st[i] = ok ? WG_PKT_OK : WG_PKT_BADHDR;
}

}  // namespace

extern "C" {

#ifdef WG_DIAG
// diagnostic build only: device buffer of 8 x u64 per workgroup for phase stamps
int wg_diag_stamps(void* dev_buf) {
  g_stamps = (uint64_t*)dev_buf;
  return WG_OK;
}
#endif

const char* wg_last_error(void) { return g_err.c_str(); }
const char* wg_version(void) { return "wgaead 0.1.0 gfx950"; }

int wg_ctx_set_kernel(wg_ctx* c, const char* name, uint32_t lanes, uint32_t variant) {
  if (!c) return fail(WG_EINVAL, "ctx is NULL");
  if (!name || !strcmp(name, "default")) {
    std::lock_guard<std::mutex> lk(c->mu);
    c->kern = KERN_DEFAULT;
    return WG_OK;
  }
  const int k = kern_from_name(name);
  if (k < 0) return fail(WG_EINVAL, "unknown transport kernel '%s'", name);
  if (lanes != 1 && lanes != 2 && lanes != 4 && lanes != 8) return fail(WG_EINVAL, "lanes per packet must be 1, 2, 4 or 8");
  std::lock_guard<std::mutex> lk(c->mu);
  c->kern = k;
  c->kern_k = lanes;
  c->kern_v = variant;
  return WG_OK;
}

int wg_ctx_create(int device, uint32_t key_slots, wg_ctx** out) {
  if (!out) return fail(WG_EINVAL, "out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(WG_EDEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(WG_EINVAL, "device %d out of range (%d devices)", device, ndev);
  if (key_slots == 0) key_slots = 1;
  DeviceGuard g(device);
  wg_ctx* c = new wg_ctx();
  c->device = device;
  c->key_slots = key_slots;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_out_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_desc, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_kernel, hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&c->keys, (size_t)key_slots * 32) != hipSuccess ||
      hipMemset(c->keys, 0, (size_t)key_slots * 32) != hipSuccess) {
    wg_ctx_destroy(c);
    return fail(WG_ENOMEM, "context allocation failed on device %d", device);
  }
  *out = c;
  return WG_OK;
}

int wg_ctx_destroy(wg_ctx* c) {
  if (!c) return WG_OK;
  DeviceGuard g(c->device);
  if (c->keys) {
    (void)hipMemset(c->keys, 0, (size_t)c->key_slots * 32);  // SymmetricKeypair.clean zeroes keys
    (void)hipDeviceSynchronize();
    (void)hipFree(c->keys);
  }
  for (auto& e : c->events) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  for (DevBuf* b : {&c->plan_nb, &c->plan_prefix, &c->plan_tiles, &c->plan_ntiles, &c->plan_tmp, &c->h_desc, &c->h_in,
                    &c->h_out, &c->h_aad, &c->h_status, &c->h_keys, &c->sink})
    b->release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->copy_out_stream) (void)hipStreamDestroy(c->copy_out_stream);
  for (hipEvent_t e : {c->ev_desc, c->ev_in, c->ev_kernel})
    if (e) (void)hipEventDestroy(e);
  delete c;
  return WG_OK;
}

int wg_ctx_device(const wg_ctx* c) { return c ? c->device : -1; }
uint32_t wg_ctx_key_slots(const wg_ctx* c) { return c ? c->key_slots : 0; }
void* wg_ctx_stream(wg_ctx* c) { return c ? (void*)c->stream : nullptr; }

int wg_sync(wg_ctx* c, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  DeviceGuard g(c->device);
  HIPTRY(hipStreamSynchronize(pick_stream(c, stream)));
  return WG_OK;
}

int wg_keys_set(wg_ctx* c, uint32_t first, uint32_t n, const uint8_t* keys_host) {
  if (!c || (!keys_host && n)) return fail(WG_EINVAL, "NULL argument");
  if ((uint64_t)first + n > c->key_slots) return fail(WG_ERANGE, "key slots [%u, %u) exceed table of %u", first, first + n, c->key_slots);
  if (!n) return WG_OK;
  DeviceGuard g(c->device);
  HIPTRY(hipMemcpyAsync((uint8_t*)c->keys + (size_t)first * 32, keys_host, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_keys_zero(wg_ctx* c, uint32_t first, uint32_t n) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if ((uint64_t)first + n > c->key_slots) return fail(WG_ERANGE, "key slots out of range");
  if (!n) return WG_OK;
  DeviceGuard g(c->device);
  HIPTRY(hipMemsetAsync((uint8_t*)c->keys + (size_t)first * 32, 0, (size_t)n * 32, c->stream));
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_seal_batch(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                  uint64_t out_size, uint32_t max_len, uint32_t flags, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  if ((flags & WG_F_FRAME) && !c->receivers) return fail(WG_EINVAL, "WG_F_FRAME without a receiver table (wg_ctx_set_receivers)");
  hipStream_t s = pick_stream(c, stream);
  const int rc = launch_transport<WG_MODE_SEAL>(c, desc, n, in, in_size, out, out_size, nullptr, max_len, flags, s);
  // measured: writing the header inside k_wave cost the seal launch +11% (register
  // pressure at 64 VGPRs), so every kernel gets k_frame_seal after it on the same stream
  if (rc != WG_OK || !(flags & WG_F_FRAME) || n == 0) return rc;
  hipLaunchKernelGGL(k_frame_seal, dim3((n + 255u) / 256u), dim3(256), 0, s, desc, n, c->receivers, c->key_slots, out,
                     out_size);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_frame_seal launch: %s", hipGetErrorString(e));
  return WG_OK;
}

int wg_ctx_set_receivers(wg_ctx* c, const uint32_t* receivers) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  std::lock_guard<std::mutex> lk(c->mu);
  c->receivers = receivers;
  return WG_OK;
}

int wg_open_batch(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                  uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  return launch_transport<WG_MODE_OPEN>(c, desc, n, in, in_size, out, out_size, status, max_len, flags,
                                       pick_stream(c, stream));
}

int wg_frame_seal(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint32_t* receivers, uint8_t* out,
                  uint64_t out_size, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (n == 0) return WG_OK;
  if (!desc || !receivers || !out) return fail(WG_EINVAL, "NULL descriptor, receiver table or output buffer");
  DeviceGuard g(c->device);
  hipStream_t s = pick_stream(c, stream);
  hipLaunchKernelGGL(k_frame_seal, dim3((n + 255u) / 256u), dim3(256), 0, s, desc, n, receivers, c->key_slots, out,
                     out_size);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_frame_seal launch: %s", hipGetErrorString(e));
  return WG_OK;
}

int wg_parse_open(wg_ctx* c, const uint8_t* wire, uint64_t wire_size, const uint64_t* pkt_off, const uint32_t* pkt_len,
                  const uint32_t* key_slot, uint32_t n, wg_pkt* desc_out, uint32_t* parse_status, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (n == 0) return WG_OK;
  if (!wire || !pkt_off || !pkt_len || !key_slot) return fail(WG_EINVAL, "NULL wire buffer or packet table");
  if (!desc_out || (((uintptr_t)desc_out) & 15u)) return fail(WG_EINVAL, "descriptor output must be non-NULL and 16-byte aligned");
  DeviceGuard g(c->device);
  hipStream_t s = pick_stream(c, stream);
  hipLaunchKernelGGL(k_parse_open, dim3((n + 255u) / 256u), dim3(256), 0, s, wire, wire_size, pkt_off, pkt_len,
                     key_slot, n, desc_out, parse_status);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_parse_open launch: %s", hipGetErrorString(e));
  return WG_OK;
}

int wg_aead_batch(wg_ctx* c, int mode, const wg_aead_desc* desc, uint32_t n, const uint8_t* in, uint64_t in_size,
                  const uint8_t* aad, uint64_t aad_size, uint8_t* out, uint64_t out_size, uint32_t* status,
                  uint32_t max_len, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  hipStream_t s = pick_stream(c, stream);
  switch (mode) {
    case WG_MODE_SEAL:
      return launch_tiles<WG_MODE_SEAL, true>(c, desc, n, in, in_size, aad, aad_size, out, out_size, nullptr, max_len, 0, s);
    case WG_MODE_OPEN:
      return launch_tiles<WG_MODE_OPEN, true>(c, desc, n, in, in_size, aad, aad_size, out, out_size, status, max_len, 0, s);
    case WG_MODE_CIPHER:
      return launch_tiles<WG_MODE_CIPHER, true>(c, desc, n, in, in_size, nullptr, 0, out, out_size, nullptr, max_len, 0, s);
    case WG_MODE_MAC:
      return launch_tiles<WG_MODE_MAC, true>(c, desc, n, in, in_size, nullptr, 0, out, out_size, nullptr, max_len, 0, s);
    default:
      return fail(WG_EINVAL, "unknown mode %d", mode);
  }
}

// ---- host-pointer API --------------------------------------------------------
//
// The transport path starts and ends in host memory (tun device in, UDP socket out).
// Two strategies, chosen per call (WG_HOST_PATH=auto|copy|zerocopy overrides):
//  * zero-copy: when `in` and `out` are pinned, device-mapped host memory
//    (wg_host_alloc, wg_host_register, or a pinned torch tensor), the kernel reads
//    the plaintext/ciphertext over PCIe and writes the result straight into the
//    caller's ring — every byte crosses the link once, in both directions at once;
//  * copy pipeline: otherwise the batch is cut into chunks of consecutive packets
//    and H2D(chunk k+1) / kernel(chunk k) / D2H(chunk k-1) overlap on three streams.
//    Chunks whose packets sit at a uniform stride move only their payload bytes
//    (hipMemcpy2DAsync rows), so bytes between packets (wire headers, ring slack)
//    are left untouched; irregular layouts move whole ranges and stage `out` first.
namespace {

// device alias of pinned, mapped host memory, or nullptr for pageable memory
uint8_t* mapped_alias(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  uint8_t* d = (uint8_t*)a.devicePointer;
  if (a.hostPointer) d += (const uint8_t*)p - (const uint8_t*)a.hostPointer;
  return d;
}

int host_path_mode() {  // 0 auto, 1 copy, 2 zerocopy
  static int m = [] {
    const char* e = getenv("WG_HOST_PATH");
    if (!e) return 0;
    if (!strcmp(e, "copy")) return 1;
    if (!strcmp(e, "zerocopy")) return 2;
    return 0;
  }();
  return m;
}

uint64_t host_chunk_bytes() {
  static uint64_t b = [] {
    const char* e = getenv("WG_HOST_CHUNK");
    uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
    return v ? v : (uint64_t)8 << 20;
  }();
  return b;
}

// one chunk's footprint in a buffer: [lo, hi), and whether its packets sit at a
// uniform stride with equal lengths (then only `width` bytes per row are copied)
struct Span {
  uint64_t lo = ~0ull, hi = 0, stride = 0, width = 0;
  bool rows = false;
};

Span chunk_span(const wg_pkt* d, uint32_t a, uint32_t b, bool in_side, uint32_t extra) {
  Span sp;
  const uint64_t first = in_side ? d[a].in_off : d[a].out_off;
  const uint64_t second = (b - a > 1) ? (in_side ? d[a + 1].in_off : d[a + 1].out_off) : first;
  const uint64_t stride = second > first ? second - first : 0;  // descending order: no row copy
  bool uni = b - a == 1 || stride > 0;
  for (uint32_t i = a; i < b; ++i) {
    const uint64_t o = in_side ? d[i].in_off : d[i].out_off;
    const uint64_t e = o + d[i].len + extra;
    sp.lo = std::min(sp.lo, o);
    sp.hi = std::max(sp.hi, e);
    uni = uni && d[i].len == d[a].len && o == first + (uint64_t)(i - a) * stride;
  }
  sp.width = (uint64_t)d[a].len + extra;
  sp.stride = stride;
  sp.rows = uni && (b - a == 1 || stride >= sp.width);
  return sp;
}

int copy_span(uint8_t* dst, const uint8_t* src, const Span& sp, uint32_t rows, hipMemcpyKind k, hipStream_t s) {
  if (sp.hi <= sp.lo) return WG_OK;
  if (sp.rows && rows > 1 && sp.stride != sp.width) {
    HIPTRY(hipMemcpy2DAsync(dst + sp.lo, sp.stride, src + sp.lo, sp.stride, sp.width, rows, k, s));
  } else {
    HIPTRY(hipMemcpyAsync(dst + sp.lo, src + sp.lo, sp.hi - sp.lo, k, s));
  }
  return WG_OK;
}

}  // namespace

static int host_transport(wg_ctx* c, bool open, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size,
                          uint8_t* out, uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags) {
  if (!c || (n && (!desc || !in || !out))) return fail(WG_EINVAL, "NULL argument");
  if (open && n && !status) return fail(WG_EINVAL, "open needs a status array");
  if (!n) return WG_OK;
  if (max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", max_len);
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  int rc;
  if ((rc = c->h_desc.ensure(sizeof(wg_pkt) * (size_t)n)) || (rc = c->h_status.ensure(sizeof(uint32_t) * (size_t)n)))
    return rc;
  hipStream_t s = c->stream, sin = c->copy_stream, sout = c->copy_out_stream;
  HIPTRY(hipMemcpyAsync(c->h_desc.p, desc, sizeof(wg_pkt) * (size_t)n, hipMemcpyHostToDevice, s));
  const wg_pkt* ddesc = (const wg_pkt*)c->h_desc.p;
  uint32_t* dstatus = (uint32_t*)c->h_status.p;

  const int mode = host_path_mode();
  uint8_t* zin = mode == 1 ? nullptr : mapped_alias(in);
  uint8_t* zout = mode == 1 ? nullptr : mapped_alias(out);
  if (mode == 2 && (!zin || !zout)) return fail(WG_EINVAL, "WG_HOST_PATH=zerocopy needs pinned host buffers");
  if (zin && zout) {
    rc = open ? launch_transport<WG_MODE_OPEN>(c, ddesc, n, zin, in_size, zout, out_size, dstatus, max_len, flags, s)
              : launch_transport<WG_MODE_SEAL>(c, ddesc, n, zin, in_size, zout, out_size, nullptr, max_len, flags, s);
    if (rc) return rc;
    if (open) HIPTRY(hipMemcpyAsync(status, dstatus, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    return WG_OK;
  }

  // copy pipeline over full-size device mirrors of the two buffers
  if ((rc = c->h_in.ensure(in_size)) || (rc = c->h_out.ensure(out_size))) return rc;
  uint8_t* din = (uint8_t*)c->h_in.p;
  uint8_t* dout = (uint8_t*)c->h_out.p;
  const uint32_t in_extra = open ? 16u : 0u, out_extra = open ? 0u : 16u;
  uint64_t per = host_chunk_bytes() / ((uint64_t)max_len + 32u);
  uint32_t chunk = (uint32_t)std::min<uint64_t>(n, std::max<uint64_t>(per, 64));
  // the chunks must occupy increasing, disjoint ranges of both buffers, or one chunk's
  // staged copy of `out` could overwrite another's results: otherwise use one chunk
  {
    uint64_t prev_in = 0, prev_out = 0;
    for (uint32_t a = 0; a < n; a += chunk) {
      const uint32_t b = std::min(n, a + chunk);
      const Span si = chunk_span(desc, a, b, true, in_extra), so = chunk_span(desc, a, b, false, out_extra);
      if (a && (si.lo < prev_in || so.lo < prev_out)) { chunk = n; break; }
      prev_in = si.hi;
      prev_out = so.hi;
    }
  }
  HIPTRY(hipEventRecord(c->ev_desc, s));
  HIPTRY(hipStreamWaitEvent(sin, c->ev_desc, 0));
  for (uint32_t a = 0; a < n; a += chunk) {
    const uint32_t b = std::min(n, a + chunk), rows = b - a;
    const Span si = chunk_span(desc, a, b, true, in_extra), so = chunk_span(desc, a, b, false, out_extra);
    if ((rc = copy_span(din, in, si, rows, hipMemcpyHostToDevice, sin))) return rc;
    // a range (not row) copy back would overwrite the bytes between packets: stage them
    if (!(so.rows && rows > 1 && so.stride != so.width) && (so.hi - so.lo) != (uint64_t)rows * so.width)
      HIPTRY(hipMemcpyAsync(dout + so.lo, out + so.lo, so.hi - so.lo, hipMemcpyHostToDevice, sin));
    HIPTRY(hipEventRecord(c->ev_in, sin));
    HIPTRY(hipStreamWaitEvent(s, c->ev_in, 0));
    rc = open ? launch_transport<WG_MODE_OPEN>(c, ddesc + a, rows, din, in_size, dout, out_size, dstatus + a, max_len,
                                               flags, s)
              : launch_transport<WG_MODE_SEAL>(c, ddesc + a, rows, din, in_size, dout, out_size, nullptr, max_len,
                                               flags, s);
    if (rc) return rc;
    HIPTRY(hipEventRecord(c->ev_kernel, s));
    HIPTRY(hipStreamWaitEvent(sout, c->ev_kernel, 0));
    if ((rc = copy_span(out, dout, so, rows, hipMemcpyDeviceToHost, sout))) return rc;
  }
  if (open) HIPTRY(hipMemcpyAsync(status, dstatus, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, sout));
  HIPTRY(hipStreamSynchronize(sout));
  HIPTRY(hipStreamSynchronize(s));
  return WG_OK;
}

int wg_host_alloc(wg_ctx* c, uint64_t bytes, void** out) {
  if (!c || !out) return fail(WG_EINVAL, "NULL argument");
  *out = nullptr;
  DeviceGuard g(c->device);
  HIPTRY(hipHostMalloc(out, std::max<uint64_t>(bytes, 1), hipHostMallocMapped | hipHostMallocPortable));
  return WG_OK;
}

int wg_host_free(wg_ctx* c, void* p) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (!p) return WG_OK;
  DeviceGuard g(c->device);
  HIPTRY(hipHostFree(p));
  return WG_OK;
}

int wg_host_register(wg_ctx* c, void* p, uint64_t bytes) {
  if (!c || !p || !bytes) return fail(WG_EINVAL, "NULL argument");
  DeviceGuard g(c->device);
  HIPTRY(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  return WG_OK;
}

int wg_host_unregister(wg_ctx* c, void* p) {
  if (!c || !p) return fail(WG_EINVAL, "NULL argument");
  DeviceGuard g(c->device);
  HIPTRY(hipHostUnregister(p));
  return WG_OK;
}

int wg_seal_host(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                 uint64_t out_size, uint32_t max_len, uint32_t flags) {
  return host_transport(c, false, desc, n, in, in_size, out, out_size, nullptr, max_len, flags);
}

int wg_open_host(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                 uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags) {
  return host_transport(c, true, desc, n, in, in_size, out, out_size, status, max_len, flags);
}

int wg_seal1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint8_t* out) {
  if (!c || (!pt && len) || !out) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  wg_pkt d{0, 0, counter, len, key_slot};
  static const uint8_t zero = 0;
  return host_transport(c, false, &d, 1, len ? pt : &zero, len ? len : 1, out, (uint64_t)len + 16, nullptr, len,
                        WG_F_UNIFORM);
}

int wg_open1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* in, uint32_t len, uint8_t* pt) {
  if (!c || !in || (!pt && len)) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  wg_pkt d{0, 0, counter, len, key_slot};
  uint32_t st = WG_PKT_BADTAG;
  std::vector<uint8_t> tmp(len ? len : 1);
  int rc = host_transport(c, true, &d, 1, in, (uint64_t)len + 16, tmp.data(), tmp.size(), &st, len, WG_F_UNIFORM);
  if (rc) return rc;
  if (st != WG_PKT_OK) return 1;  // dst untouched, as ChaCha20Poly1305.java:51-53 throws before decrypting
  if (len) memcpy(pt, tmp.data(), len);
  return WG_OK;
}

int wg_aead_host(wg_ctx* c, int mode, const wg_aead_desc* desc, uint32_t n, const uint8_t* keys_host, uint32_t nkeys,
                 const uint8_t* in, uint64_t in_size, const uint8_t* aad, uint64_t aad_size, uint8_t* out,
                 uint64_t out_size, uint32_t* status) {
  if (!c || (n && (!desc || !keys_host || !out))) return fail(WG_EINVAL, "NULL argument");
  if (mode == WG_MODE_OPEN && n && !status) return fail(WG_EINVAL, "open needs a status array");
  if (!n) return WG_OK;
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (desc[i].key_slot >= nkeys) return fail(WG_ERANGE, "desc %u key_slot %u >= nkeys %u", i, desc[i].key_slot, nkeys);
    max_len = std::max(max_len, desc[i].len);
  }
  if (max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", max_len);
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  int rc;
  const size_t in_b = std::max<uint64_t>(in_size, 1), aad_b = std::max<uint64_t>(aad_size, 1);
  if ((rc = c->h_desc.ensure(sizeof(wg_aead_desc) * (size_t)n)) || (rc = c->h_in.ensure(in_b)) ||
      (rc = c->h_out.ensure(out_size)) || (rc = c->h_aad.ensure(aad_b)) ||
      (rc = c->h_status.ensure(sizeof(uint32_t) * (size_t)n)) || (rc = c->h_keys.ensure((size_t)nkeys * 32)))
    return rc;
  hipStream_t s = c->stream;
  HIPTRY(hipMemcpyAsync(c->h_desc.p, desc, sizeof(wg_aead_desc) * (size_t)n, hipMemcpyHostToDevice, s));
  if (in && in_size) HIPTRY(hipMemcpyAsync(c->h_in.p, in, in_size, hipMemcpyHostToDevice, s));
  if (aad && aad_size) HIPTRY(hipMemcpyAsync(c->h_aad.p, aad, aad_size, hipMemcpyHostToDevice, s));
  HIPTRY(hipMemcpyAsync(c->h_out.p, out, out_size, hipMemcpyHostToDevice, s));
  HIPTRY(hipMemcpyAsync(c->h_keys.p, keys_host, (size_t)nkeys * 32, hipMemcpyHostToDevice, s));
  // swap in the per-call key table
  uint32_t* saved_keys = c->keys;
  uint32_t saved_slots = c->key_slots;
  c->keys = (uint32_t*)c->h_keys.p;
  c->key_slots = nkeys;
  const uint8_t* din = (const uint8_t*)c->h_in.p;
  const uint8_t* dad = (const uint8_t*)c->h_aad.p;
  uint8_t* dout = (uint8_t*)c->h_out.p;
  uint32_t* dst = (uint32_t*)c->h_status.p;
  switch (mode) {
    case WG_MODE_SEAL:
      rc = launch_tiles<WG_MODE_SEAL, true>(c, c->h_desc.p, n, din, in_size, dad, aad_size, dout, out_size, nullptr, max_len, 0, s);
      break;
    case WG_MODE_OPEN:
      rc = launch_tiles<WG_MODE_OPEN, true>(c, c->h_desc.p, n, din, in_size, dad, aad_size, dout, out_size, dst, max_len, 0, s);
      break;
    case WG_MODE_CIPHER:
      rc = launch_tiles<WG_MODE_CIPHER, true>(c, c->h_desc.p, n, din, in_size, nullptr, 0, dout, out_size, nullptr, max_len, 0, s);
      break;
    case WG_MODE_MAC:
      rc = launch_tiles<WG_MODE_MAC, true>(c, c->h_desc.p, n, din, in_size, nullptr, 0, dout, out_size, nullptr, max_len, 0, s);
      break;
    default:
      rc = fail(WG_EINVAL, "unknown mode %d", mode);
  }
  c->keys = saved_keys;
  c->key_slots = saved_slots;
  if (rc) return rc;
  if (mode == WG_MODE_OPEN) HIPTRY(hipMemcpyAsync(status, dst, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemcpyAsync(out, dout, out_size, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemsetAsync(c->h_keys.p, 0, (size_t)nkeys * 32, s));  // do not leave key material behind
  HIPTRY(hipStreamSynchronize(s));
  return WG_OK;
}

// ---- instrumentation -----------------------------------------------------------

int wg_timing_enable(wg_ctx* c, int on) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  std::lock_guard<std::mutex> lk(c->mu);
  c->timing = on != 0;
  return WG_OK;
}

int wg_timing_read(wg_ctx* c, double* total_ms, uint64_t* launches) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  for (auto& e : c->events) {
    float ms = 0;
    HIPTRY(hipEventSynchronize(e.second));
    HIPTRY(hipEventElapsedTime(&ms, e.first, e.second));
    c->timed_ms += ms;
    c->timed_launches += 1;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  c->events.clear();
  if (total_ms) *total_ms = c->timed_ms;
  if (launches) *launches = c->timed_launches;
  c->timed_ms = 0;
  c->timed_launches = 0;
  return WG_OK;
}

// ---- self test: the reference's own known-answer vectors, run on the device ----

int wg_aead_selftest(int device) {
  wg_ctx* c = nullptr;
  if (wg_ctx_create(device, 1, &c) != WG_OK) return 0;
  int ok = 1;
  // RFC 8439 2.8.2 (Poly1305Test.java:151-199)
  static const uint8_t key[32] = {0x80, 0x81, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a,
                                  0x8b, 0x8c, 0x8d, 0x8e, 0x8f, 0x90, 0x91, 0x92, 0x93, 0x94, 0x95,
                                  0x96, 0x97, 0x98, 0x99, 0x9a, 0x9b, 0x9c, 0x9d, 0x9e, 0x9f};
  static const uint8_t aad[12] = {0x50, 0x51, 0x52, 0x53, 0xc0, 0xc1, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7};
  static const char* pt = "Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, sunscreen would be it.";
  static const uint8_t tag_expect[16] = {0x1a, 0xe1, 0x0b, 0x59, 0x4f, 0x09, 0xe2, 0x6a,
                                         0x7e, 0x90, 0x2e, 0xcb, 0xd0, 0x60, 0x06, 0x91};
  static const uint8_t ct_head[8] = {0xd3, 0x1a, 0x8d, 0x34, 0x64, 0x8e, 0x60, 0xdb};
  const uint32_t L = (uint32_t)strlen(pt);
  wg_aead_desc d{};
  d.len = L;
  d.aad_len = 12;
  d.nonce[0] = 0x00000007u;  // 07 00 00 00 | 40 41 42 43 | 44 45 46 47
  d.nonce[1] = 0x43424140u;
  d.nonce[2] = 0x47464544u;
  std::vector<uint8_t> out(L + 16, 0);
  if (wg_aead_host(c, WG_MODE_SEAL, &d, 1, key, 1, (const uint8_t*)pt, L, aad, 12, out.data(), out.size(), nullptr) != WG_OK ||
      memcmp(out.data() + L, tag_expect, 16) != 0 || memcmp(out.data(), ct_head, 8) != 0)
    ok = 0;
  // RFC 8439 2.5.2 Poly1305 (Poly1305Test.java:49-61)
  static const uint8_t pkey[32] = {0x85, 0xd6, 0xbe, 0x78, 0x57, 0x55, 0x6d, 0x33, 0x7f, 0x44, 0x52,
                                   0xfe, 0x42, 0xd5, 0x06, 0xa8, 0x01, 0x03, 0x80, 0x8a, 0xfb, 0x0d,
                                   0xb2, 0xfd, 0x4a, 0xbf, 0xf6, 0xaf, 0x41, 0x49, 0xf5, 0x1b};
  static const char* msg = "Cryptographic Forum Research Group";
  static const uint8_t mac_expect[16] = {0xa8, 0x06, 0x1d, 0xc1, 0x30, 0x51, 0x36, 0xc6,
                                         0xc2, 0x2b, 0x8b, 0xaf, 0x0c, 0x01, 0x27, 0xa9};
  wg_aead_desc m{};
  m.len = (uint32_t)strlen(msg);
  uint8_t mac[16] = {0};
  if (wg_aead_host(c, WG_MODE_MAC, &m, 1, pkey, 1, (const uint8_t*)msg, m.len, nullptr, 0, mac, 16, nullptr) != WG_OK ||
      memcmp(mac, mac_expect, 16) != 0)
    ok = 0;
  // donna wrap vector: a final value of 2^130 - 2 (poly1305-donna.c:118-134)
  uint8_t wkey[32] = {2};
  uint8_t wmsg[16];
  memset(wmsg, 0xff, 16);
  static const uint8_t wmac[16] = {3};
  wg_aead_desc w{};
  w.len = 16;
  if (wg_aead_host(c, WG_MODE_MAC, &w, 1, wkey, 1, wmsg, 16, nullptr, 0, mac, 16, nullptr) != WG_OK ||
      memcmp(mac, wmac, 16) != 0)
    ok = 0;
  wg_ctx_destroy(c);
  return ok;
}

}  // extern "C"
