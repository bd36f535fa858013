// wg_capi.hip — the C-ABI of libwgaead.so (include/wgaead.h).
//
// Host runtime around the gfx950 kernels: per-device context (stream, device key
// table, plan workspace, staging buffers), launch planning, the device-pointer
// batch API, the host-pointer API, the per-packet batcher (wg_batcher.hip) and the
// on-device self test. No CPU crypto lives here: every seal/open/cipher/MAC runs in
// a HIP kernel, and every entry point fails with WG_EDEVICE when no HIP device is usable.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>
#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "wg_tile.hip"
#include "wg_transport.hip"
#include "wg_wave_r1.hip"

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
  // a histogram workspace used by k_lpt_one: its two counter sets (zeroed = both are zero or hold this
  // buffer's counts), the set the next call counts into, the set the last call counted into
  bool zeroed = false;
  uint32_t par = 0;
  uint32_t* last_cnt = nullptr;
  int ensure(size_t bytes) {
    if (bytes <= cap) return WG_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    zeroed = false;
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

// transport kernels selectable per context (wg_ctx_set_kernel)
enum Kern { KERN_TRANSPORT = 0, KERN_WAVE1 = 1, KERN_TILE = 2 };

struct PPServer;  // wg_pp.hip
void pp_stop(wg_ctx* c);
int rx_tables(wg_ctx* c, const wgt::RxTables** out);  // wg_rx.hip
struct RxState;  // wg_rx.hip

}  // namespace

struct wg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;      // host path: H2D
  hipStream_t copy_out_stream = nullptr;  // host path: D2H
  hipEvent_t ev_desc = nullptr, ev_in = nullptr, ev_kernel = nullptr;
  hipEvent_t ev_ws = nullptr;             // last use of the plan workspace
  hipStream_t ws_stream = nullptr;        // stream of that use
  uint32_t key_slots = 0;
  uint32_t* keys = nullptr;               // device key table
  const uint32_t* receivers = nullptr;    // device receiver_index per key slot (WG_F_FRAME; caller-owned)
  // waves resident at once (occupancy) of k_transport<SEAL>, <OPEN> and k_step, with 8-lane [0],
  // 16-lane [1] and 4-lane [2] slots (rw_row)
  uint32_t resident_waves[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  int slot16 = -1;                        // mixed batches: -1 planned (slot_plan), 0 / 1 force 8- / 16-lane slots (WG_SLOT16)
  // mixed batches of short packets (WG_SLOT4): -1 planned (16-lane slots for the long packets, 4-lane for the
  // rest), 0 never, 1 always 4-lane slots for every packet, 2 always the 16 / 4 split
  int slot4 = -1;
  bool slot4_pairs = false;               // 4-lane slots in longest-first pairs even when one packet per slot fits (A/B)
  bool slot4_snake = true;                // 4-lane slots: odd workgroup generations reversed (WG_SLOT4_SNAKE=0: not; A/B)
  uint32_t cus = 0;                       // compute units
  int prio_mode = -1;                     // progress-based issue priority: -1 mixed batches only, 0 off, 1 on (WG_PRIO)
  uint32_t uniform16 = 8;                 // uniform batches of n <= S8 / k packets in 16-lane slots (WG_UNIFORM16=k; 0 never)
  uint32_t mixed_split = 0;               // > 0: mixed batches one packet per slot, packets of more than this
                                          // many 8-block rounds in 16-lane slots (WG_MIXED_SPLIT)
  bool step_two_launches = false;         // wg_ctx_set_kernel variant 1: WG_F_AFTER_SEAL as seal + open launches
  // half-occupancy k_step grids (C2's longest-first pairs) take the build allocated for 4 waves per
  // SIMD: no SGPR spills, C2 +0.7% in 3 alternations (profiles/r04_wpe_ab.txt); WG_STEP_WPE4=0: not
  bool step_wpe4 = true;
  // mixed-length WG_F_AFTER_SEAL steps through k_step_claim (dynamic claims over the longest-first
  // order) instead of the static snake (WG_CLAIM=1; A/B)
  bool claim = false;
  // WG_F_AFTER_SEAL steps with the stitched Horner (transport_body ST: a round's Horner steps interleaved
  // into the next round's ChaCha20 rounds; WG_STITCH=0|1, A/B)
  bool stitch = false;
  // the short-packet split plan's order in one launch (k_lpt_one; WG_LPT_ONE=0: k_lpt_hist + k_lpt_scatter)
  bool lpt_one = true;
  // ... and for the 8-lane longest-first pairs of other mixed steps (C2; WG_LPT_WIDE=1, A/B): planning 9.9 ->
  // 6.5 us per C2 step, but k_step 411.8 -> 416.5 us (19 round keys order less finely than the two launches'
  // 130 bins, and the sparse lookups): C2 -0.3% (profiles/r06_lpt_wide_ab.jsonl); off
  bool lpt_wide = false;
  // WG_LPT_FUSED=1 (A/B, off): in a k_step_mixed step, planned by the step launch's first workgroups
  // (k_step_mixed_fused) instead of k_lpt_one's own launch. IMIX 66-70 us per step against 59: the planners
  // take 6-8 us while every other workgroup waits, more than the launch gap they remove
  // (profiles/r06_fused_ab.jsonl). plan_err: a pinned word the fused kernel sets when a workgroup's wait for
  // the plan ran out (a later step then fails with WG_EDEVICE)
  bool lpt_fused = false;
  // the short-packet split plan's tiny packets (keys <= slot2, i.e. at most 8 x slot2 blocks: 448 B for 1) in
  // 2-lane slots (k_step_mixed<4, false, 2>; WG_SLOT2=k, 0: none). IMIX +2.3% (715 -> 731 GiB/s, three
  // alternations); 65,536 x 40 B 37.0 -> 27.1 us per step; 2 (576-B packets too) measured +-0
  // (profiles/r06_slot2_ab.jsonl)
  uint32_t slot2 = 1;
  uint32_t fused_poll = 0, fused_np = 0;  // WG_FUSED_POLL (k_step_mixed_fused's poll kind), WG_FUSED_NP (planners)
  uint32_t* plan_err = nullptr;
  // test hook WG_TEST_STEP_FLIP=N (power of two): the k_step launch's seal half writes a wrong tag for every
  // packet whose index is a multiple of N (tests/test_gpu_bench.py: the bench must report verified false)
  uint32_t test_flip = 0;
  // plan workspace: k_tile block scan, k_transport longest-first order
  DevBuf plan_nb, plan_prefix, plan_tiles, plan_ntiles, plan_tmp, lpt_hist, lpt_order;
  DevBuf lpt_hist2, lpt_order2;  // the open half of a wg_duplex_batch
  DevBuf lpt_nlong;              // k_lpt_scatter -> k_*_mixed: long packets at the front of lpt_order
  DevBuf lpt_claim, lpt_chain;   // k_step_claim: sub-order counters (64-B lines) and the seal half's per-position log
  // per-stream plan workspaces for the short-packet split plan's WG_F_AFTER_SEAL steps (k_lpt_one's counters
  // and sparse order): calls on different streams then plan and run concurrently instead of waiting for
  // each other's workspace (ws_acquire). Up to kStreamWS streams; each use waits for the workspace's last
  // use (an event: a no-op on its own stream, an order if a stream handle was reused). WG_STREAM_WS=0: off
  struct StreamWS {
    hipStream_t s = nullptr;
    DevBuf hist, order;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  static constexpr size_t kStreamWS = 8;
  std::vector<std::unique_ptr<StreamWS>> stream_ws;
  bool stream_ws_on = true;
  bool ws_ext = true;  // WG_WS_EXT=0: the workspace event as a hipEventRecord after the step launch (A/B)
  uint32_t wsev = 3;  // WG_WSEV (A/B): bit 0 record an event after each use, bit 1 wait on it before the next

  int kern = KERN_TRANSPORT;
  // host-API staging
  DevBuf h_desc, h_in, h_out, h_aad, h_status, h_keys;
  std::mutex mu;  // serialises host-API calls and plan workspace reuse
  std::atomic<PPServer*> pp{nullptr};  // persistent per-packet server (wg_seal1 / wg_open1), made once
  std::mutex pp_mu;
  // Host mirror of the key table, read by the paths that send a key WITH the packet (the per-packet
  // server, the asynchronous queue): 4 words per slot behind a per-slot sequence lock, so readers
  // (every submit) take no lock and share no written cache line; writers (wg_keys_set / wg_keys_zero)
  // serialise on keys_mu. key_snapshot() reads a consistent key.
  std::unique_ptr<std::atomic<uint64_t>[]> key_words;
  std::unique_ptr<std::atomic<uint32_t>[]> key_seq;  // even: stable, odd: being written
  // per slot: 1 once wg_keys_set wrote a key, 0 when never set or zeroed by wg_keys_zero (clean()): the
  // paths that carry a key with the packet refuse a packet for a slot without a key (WG_ENOKEY /
  // WG_PKT_NOKEY) instead of sealing it under the all-zero key, as the reference's cipher() / decipher()
  // throw once clean() has closed the key arena (SymmetricKeypair.java:85-93)
  std::unique_ptr<std::atomic<uint32_t>[]> key_live;
  std::mutex keys_mu;
  RxState* rx = nullptr;  // receive-side checks (wg_rx.hip)
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

// The key of `slot` as the host mirror holds it now (sequence-lock read: retried while a writer is
// inside wg_keys_set / wg_keys_zero for that slot, so the 32 bytes are never a mix of two keys).
// Returns whether the slot holds a key (false: never set, or zeroed; `key` is then all zero).
bool key_snapshot(const wg_ctx* c, uint32_t slot, uint32_t key[8]) {
  std::atomic<uint32_t>& sq = c->key_seq[slot];
  for (;;) {
    const uint32_t s1 = sq.load(std::memory_order_acquire);
    if (s1 & 1u) {
      __builtin_ia32_pause();
      continue;
    }
    uint64_t w[4];
    for (int i = 0; i < 4; ++i) w[i] = c->key_words[4u * slot + i].load(std::memory_order_relaxed);
    const uint32_t live = c->key_live[slot].load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (sq.load(std::memory_order_relaxed) == s1) {
      memcpy(key, w, 32);
      return live != 0;
    }
  }
}

// Whether `slot` holds a key now (the up-front check of a per-packet call or a queue submit).
bool key_is_live(const wg_ctx* c, uint32_t slot) { return c->key_live[slot].load(std::memory_order_acquire) != 0; }

// Writes slots [first, first + n) of the host mirror (keys: n x 32 B, or NULL for zeros). Caller holds
// c->keys_mu.
void key_mirror_write(wg_ctx* c, uint32_t first, uint32_t n, const uint8_t* keys) {
  for (uint32_t k = 0; k < n; ++k) {
    std::atomic<uint32_t>& sq = c->key_seq[first + k];
    const uint32_t s0 = sq.load(std::memory_order_relaxed);
    sq.store(s0 + 1u, std::memory_order_relaxed);  // odd: readers retry
    std::atomic_thread_fence(std::memory_order_release);
    uint64_t w[4] = {0, 0, 0, 0};
    if (keys) memcpy(w, keys + 32ull * k, 32);
    for (int i = 0; i < 4; ++i) c->key_words[4ull * (first + k) + i].store(w[i], std::memory_order_relaxed);
    c->key_live[first + k].store(keys ? 1u : 0u, std::memory_order_relaxed);
    sq.store(s0 + 2u, std::memory_order_release);
  }
}

template <int MODE>
uint32_t host_pkt_blocks(uint32_t len) {
  uint32_t nb = (len + 63u) / 64u;
  return (MODE == WG_MODE_SEAL || MODE == WG_MODE_OPEN) ? nb + 1u : nb;
}

constexpr uint32_t kLdsBudget = 64u * 1024u;  // k_tile: per workgroup; keeps >= 2 tiles per CU
constexpr uint32_t kTilePasses = 2;           // k_tile: max workgroup passes per uniform tile
constexpr uint32_t kPolyWaves = 4;            // k_tile: waves the Poly1305 phase spreads a tile's packets over
constexpr uint32_t kPolyGmax = 16;            // k_tile: cap on lanes per packet
constexpr uint32_t kFlagsKnown = WG_F_UNIFORM | WG_F_FRAME;

// lanes per packet for the Poly1305 phase of k_tile: spread the tile's packets over
// kPolyWaves waves (groups never straddle a wave)
uint32_t choose_poly_g(uint32_t ppt) {
  if (ppt == 0) return 1;
  uint32_t per_wave = (ppt + kPolyWaves - 1) / kPolyWaves;
  uint32_t g = 64u / per_wave;
  if (g < 1) g = 1;
  if (g > kPolyGmax) g = kPolyGmax;
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

// The plan workspace is reused by every launch on the context: a launch on another
// stream first waits for the previous user (stream-ordered reuse).
int ws_acquire(wg_ctx* c, hipStream_t s) {
  if (c->ws_stream != s && c->ws_stream != (hipStream_t)-1) HIPTRY(hipStreamWaitEvent(s, c->ev_ws, 0));
  return WG_OK;
}
int ws_release(wg_ctx* c, hipStream_t s) {
  HIPTRY(hipEventRecord(c->ev_ws, s));
  c->ws_stream = s;
  return WG_OK;
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
      for (uint32_t k = 1; k <= kTilePasses; ++k) {
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
    if (lds > 160u * 1024u) return fail(WG_E2BIG, "tile needs %u bytes of LDS", lds);
    hipEvent_t ev;
    record_start(c, s, &ev);
    hipLaunchKernelGGL((wgk::k_tile<MODE, GENERAL>), dim3(grid), dim3(WG_TPB), lds, s, P);
    hipError_t e = hipGetLastError();
    record_end(c, s, ev);
    if (e != hipSuccess) return fail(WG_EDEVICE, "k_tile launch: %s", hipGetErrorString(e));
    return WG_OK;
  }
  // device plan: block counts -> exclusive scan -> start-owned tiles of C blocks
  const uint32_t C = WG_TPB;
  const uint32_t max_nb = host_pkt_blocks<MODE>(max_len);
  const uint64_t max_tiles64 = ((uint64_t)n * std::max<uint32_t>(max_nb, 1u) + C - 1) / C;
  if (max_tiles64 > 0x7fffffffull) return fail(WG_EINVAL, "batch too large");
  const uint32_t max_tiles = (uint32_t)max_tiles64;
  lds = wgk::tile_header_bytes(C) + (C + max_nb) * 64u;
  if (lds > 160u * 1024u) return fail(WG_E2BIG, "tile needs %u bytes of LDS", lds);
  int rc;
  if ((rc = c->plan_nb.ensure(sizeof(uint32_t) * (n + 1))) != WG_OK) return rc;
  if ((rc = c->plan_prefix.ensure(sizeof(uint32_t) * (n + 1))) != WG_OK) return rc;
  if ((rc = c->plan_tiles.ensure(sizeof(uint32_t) * (max_tiles + 2))) != WG_OK) return rc;
  if ((rc = c->plan_ntiles.ensure(sizeof(uint32_t))) != WG_OK) return rc;
  size_t tmp = 0;
  HIPTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (uint32_t*)c->plan_nb.p, (uint32_t*)c->plan_prefix.p,
                                          (int)(n + 1), s));
  if ((rc = c->plan_tmp.ensure(tmp)) != WG_OK) return rc;
  if ((rc = ws_acquire(c, s)) != WG_OK) return rc;
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
  grid = max_tiles;
  hipEvent_t ev;
  record_start(c, s, &ev);
  hipLaunchKernelGGL((wgk::k_tile<MODE, GENERAL>), dim3(grid), dim3(WG_TPB), lds, s, P);
  hipError_t e = hipGetLastError();
  record_end(c, s, ev);
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_tile launch: %s", hipGetErrorString(e));
  return ws_release(c, s);
}

// Parameters and grid of one k_transport direction (shared by k_transport, k_step and k_duplex):
// persistent slots for mixed lengths (longest-first order in lpt_order), one packet per
// slot for uniform batches. cap_waves: the waves resident at once for this direction; G: lanes
// per slot (64 / G slots per wave).
template <int MODE>
int plan_transport(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                   uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, hipStream_t s,
                   uint64_t cap_waves, uint32_t G, DevBuf& lpt_hist, DevBuf& lpt_order, wgt::TransportParams* Pout,
                   uint32_t* grid_out, bool* ordered_out, const wgt::RxTables* rx = nullptr,
                   bool private_ws = false, bool reuse_order = false, uint32_t split = 0,
                   uint32_t* claim = nullptr, uint32_t claim_nc = 0, bool* defer_one = nullptr,
                   bool wide_ok = false) {
  bool ordered = false;
  const bool may_defer = defer_one && *defer_one;
  if (defer_one) *defer_one = false;
  wgt::TransportParams P{};
  P.desc = desc;
  P.n = n;
  P.max_len = max_len;
  P.key_slots = c->key_slots;
  P.in = in;
  P.in_size = in_size;
  P.out = out;
  P.out_size = out_size;
  P.keys = c->keys;
  P.status = status;
  P.rx = MODE == WG_MODE_OPEN ? rx : nullptr;
#ifdef WG_DIAG
  P.stamps = g_stamps;
#endif
  // mixed lengths with a split (WG_MIXED_SPLIT): one packet per slot, the long ones in 16-lane
  // slots (k_transport_mixed / k_step_mixed); the grid is an upper bound, the kernel sizes both
  // parts from the device count of long packets
  const bool mixed = !(flags & WG_F_UNIFORM) && split > 0;
  const uint32_t spw = 64u / G;  // slots per wave
  const uint64_t cap_slots = spw * cap_waves;
  uint64_t per_slot = (n + cap_slots - 1) / cap_slots;
  // mixed lengths: a slot holding one packet runs as long as the longest packet, so once a
  // one-packet-per-slot grid would fill more than half the machine, pair packets longest-first
  // (an even number per slot, k_lpt_*, so the snake deals each slot long and short packets in
  // turn): about 4 waves per SIMD, every slot with a similar share. Measured on 131072 C2-shaped
  // packets: 4 per slot (4096 waves) 1,322 GiB/s, 2 per slot (8192 waves) 1,208, 3 per slot 1,148.
  if (!(flags & WG_F_UNIFORM) && 2ull * n > cap_slots) per_slot = 2 * ((n + cap_slots - 1) / cap_slots);
  // 4-lane slots (16 per wave) hold a 65,536-packet batch one packet per slot at 4 waves per SIMD; pairs
  // would halve the waves (WG_SLOT4_PAIRS=1: pairs as for 8-lane slots, A/B)
  if (G == 4 && !c->slot4_pairs && n <= cap_slots) per_slot = 1;
#ifndef WG_PERSISTENT_UNIFORM
  // uniform lengths: one packet per slot and as many waves as that takes; the hardware
  // dispatcher starts each new wave as an old one retires, so a wave's packet-start
  // latency overlaps the other waves' work and the launch walks the rings in order
  // (C3: 8M packets, +8% over persistent slots; mixed batches stay persistent: one packet
  // per slot with longest-first order measured 13% slower on C2)
  if (flags & WG_F_UNIFORM) per_slot = 1;
#endif
  if (mixed) per_slot = 1;
  const uint32_t waves = (uint32_t)((n + spw * per_slot - 1) / (spw * per_slot));
  const uint32_t grid = mixed ? (n + 4u * wgt::TW - 1u) / (4u * wgt::TW) + 2u : (waves + wgt::TW - 1) / wgt::TW;
  P.slots = grid * wgt::TW * spw;
  // 4-lane slots, one packet each, longest first: all waves are resident at once, and wave w shares its
  // SIMD with waves w + 4 x CUs k; reversing every other generation of 4 x CUs waves deals each SIMD long
  // and short packets in turn (without it a SIMD holding the longest packets ran alone at the end)
  if (G == 4 && per_slot == 1 && c->slot4_snake) P.wave_gen = wgt::TW * c->cus;
  if (claim) {  // k_step_claim: the largest power of two <= claim_nc that divides the grid (every sub-order
                // then has the same number of workgroups, and its static first positions end at claim_base)
    uint32_t nc = claim_nc;
    while (nc > 1 && grid % nc) nc >>= 1;
    P.claim = claim;
    P.claim_nc = nc;
    P.claim_base = P.slots / nc;
  }
  // mixed lengths: the rounds a slot runs, spread over the 4 issue-priority levels (k_transport),
  // so the waves that have done the least work issue first (C2 +2%); uniform batches keep the
  // default oldest-first arbitration (the same schedule cost C1 2%)
  const uint32_t max_rounds = (host_pkt_blocks<WG_MODE_SEAL>(max_len) + G - 1u) / G;
  const uint32_t pstep = std::max<uint32_t>(1u, (uint32_t)((per_slot * max_rounds + 3u) / 4u));
  P.prio_step = (flags & WG_F_UNIFORM) ? 0u : pstep;
  if (c->prio_mode == 0) P.prio_step = 0;  // WG_PRIO=0 / 1: issue priority off / on for every batch (A/B)
  else if (c->prio_mode == 1) P.prio_step = pstep;
  if (mixed && c->prio_mode != 1) P.prio_step = 0;
  // longest-first order (LPT); 4-lane slots always (one packet per slot: a wave then holds 16 packets of
  // about one length instead of running as long as the longest of 16 random ones)
  if (!(flags & WG_F_UNIFORM) && (per_slot > 1 || mixed || G == 4)) {
    // reuse_order: the order already in lpt_order (the seal of the same packets, WG_F_AFTER_SEAL);
    // private_ws: buffers owned by the caller's stream (no shared-workspace ordering)
    // one: the short-packet split plan orders in ONE launch (k_lpt_one: sparse order, double-buffered
    // counters, no memset) instead of k_lpt_hist + k_lpt_scatter (WG_LPT_ONE=0: the two launches, A/B)
    // wide: the same one-launch plan over up to kWideBins keys for a k_step<8, 4> step of a mixed batch on
    // the 8-lane longest-first pairs (C2; WG_LPT_WIDE=0: the two launches); wide_ok from launch_after_seal,
    // and exactly the condition under which it launches k_step<8, 4> (the kernel that reads this order)
    const uint32_t key_max = (((max_len + 63u) >> 6) + 1u + 7u) >> 3;
    const bool wide = wide_ok && !mixed && !claim && c->lpt_one && c->lpt_wide && key_max < wgt::kWideBins &&
                      G == 8 && c->step_wpe4 && 2ull * grid * wgt::TW <= cap_waves && !c->stitch && !c->test_flip;
    const bool one = (mixed && max_len <= 2048u && !claim && c->lpt_one) || wide;
    if (!reuse_order && one) {
      int rc;
      if ((rc = lpt_hist.ensure(2 * wgt::kPlanSet * sizeof(uint32_t))) != WG_OK) return rc;
      if ((rc = lpt_order.ensure(sizeof(uint32_t) * (wide ? wgt::kWideBins : wgt::kFastBins) * (size_t)n)) != WG_OK)
        return rc;
      if (!private_ws && (rc = ws_acquire(c, s)) != WG_OK) return rc;
      if (!lpt_hist.zeroed) {  // a new buffer, or one the two-launch planner wrote histograms into
        HIPTRY(hipMemsetAsync(lpt_hist.p, 0, 2 * wgt::kPlanSet * sizeof(uint32_t), s));
        lpt_hist.zeroed = true;
        lpt_hist.par = 0;
      }
      uint32_t* cnt = (uint32_t*)lpt_hist.p + wgt::kPlanSet * lpt_hist.par;
      uint32_t* nxt = (uint32_t*)lpt_hist.p + wgt::kPlanSet * (lpt_hist.par ^ 1u);
      const uint32_t lgrid = std::max<uint32_t>(1u, std::min<uint32_t>(wgt::LPT_MAX_BLOCKS, (n + 1023u) / 1024u));
      if (may_defer && !wide) {  // the caller's k_step_mixed_fused launch plans (into cnt / nxt, as below)
        *defer_one = true;
      } else if (wide) {
        hipLaunchKernelGGL((wgt::k_lpt_one<MODE, wgt::LPT_THREADS, 1, wgt::kWideBins>), dim3(lgrid),
                           dim3(wgt::LPT_THREADS), 0, s, desc, n, max_len, cnt, nxt, (uint32_t*)lpt_order.p);
        HIPTRY(hipGetLastError());
      } else {
        // (block shapes of 256 / 512 threads or 4 packets per thread measured the same or slower: 5.0-8.3 us,
        // profiles/r06_lpt_shape_ab.jsonl)
        hipLaunchKernelGGL((wgt::k_lpt_one<MODE>), dim3(lgrid), dim3(wgt::LPT_THREADS), 0, s, desc, n, max_len, cnt,
                           nxt, (uint32_t*)lpt_order.p);
        HIPTRY(hipGetLastError());
      }
      lpt_hist.last_cnt = cnt;
      lpt_hist.par ^= 1u;
    } else if (!reuse_order) {
      int rc;
      lpt_hist.zeroed = false;
      const uint32_t lgrid = std::max<uint32_t>(1u, std::min<uint32_t>(wgt::LPT_MAX_BLOCKS, (n + 1023u) / 1024u));
      if ((rc = lpt_hist.ensure(sizeof(uint32_t) * wgt::LPT_MAX_BLOCKS * wgt::LPT_BINS)) != WG_OK) return rc;
      if ((rc = lpt_order.ensure(sizeof(uint32_t) * (size_t)n)) != WG_OK) return rc;
      if (mixed && (rc = c->lpt_nlong.ensure(sizeof(uint32_t))) != WG_OK) return rc;
      if (!private_ws && (rc = ws_acquire(c, s)) != WG_OK) return rc;
      uint32_t* bh = (uint32_t*)lpt_hist.p;
      hipLaunchKernelGGL((wgt::k_lpt_hist<MODE>), dim3(lgrid), dim3(wgt::LPT_THREADS), 0, s, desc, n, max_len, bh);
      hipLaunchKernelGGL((wgt::k_lpt_scatter<MODE>), dim3(lgrid), dim3(wgt::LPT_THREADS), 0, s, desc, n, max_len,
                         (const uint32_t*)bh, (uint32_t*)lpt_order.p, split,
                         mixed ? (uint32_t*)c->lpt_nlong.p : nullptr, claim, P.claim_nc, P.claim_base);
      HIPTRY(hipGetLastError());
    }
    P.order = (const uint32_t*)lpt_order.p;
    if (one) {
      P.bin_cnt = lpt_hist.last_cnt;
      P.bin_cap = n;
      P.split = split;
      if (mixed) P.n_long = lpt_hist.last_cnt;  // (marks the launch as mixed; a wide plan's k_step is not)
    } else if (mixed) {
      P.n_long = (const uint32_t*)c->lpt_nlong.p;
    }
    ordered = !private_ws;
  }
  *Pout = P;
  *grid_out = grid;
  *ordered_out = ordered;
  return WG_OK;
}

// An open whose input and output buffers overlap may hold packets whose plaintext overlaps their
// own ciphertext || tag: it runs the verify-first kernel variant (include/wgaead.h, wg_pkt).
bool open_overlaps(const uint8_t* in, uint64_t in_size, const uint8_t* out, uint64_t out_size) {
  const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out;
  return a < b + out_size && b < a + in_size;
}

// How a batch runs (round-3 measurements; S8 = 8-lane slots resident at once,
// 65536 on MI355X):
//   uniform lengths: one packet per slot, as many waves as that takes; 8-lane slots, 16-lane ones for
//     n <= S8 / 8 (8192 x 1420 B: 665 -> 750 GiB/s; 16384: 1085 -> 948, so not above);
//   mixed, n >= 3/4 S8: 8-lane slots, longest-first pairs (2+ packets per slot, ~4 waves per SIMD);
//   mixed, n >= 3/8 S8: 16-lane slots, longest-first pairs (the same wave count for half the packets);
//   mixed, smaller: one packet per slot, every packet of more than one 8-block round in a 16-lane
//     slot, longest first (k_transport_mixed / k_step_mixed).
// C2-shaped batches (64..9000 B): 16384 packets 722 -> 1152 GiB/s, 32768 909 -> 1321 against the
// 8-lane pairs; 65536 stays on them. WG_SLOT16 / WG_MIXED_SPLIT force a plan (A/B).
//   mixed, n >= 3/8 S8 and max_len <= kSlot4MaxLen: one packet per slot, packets of more than two 8-block
//     rounds in 16-lane slots and the rest in 4-lane slots (k_*_mixed<4>). Short packets waste most of an
//     8-block round (a 40-B packet is 2 blocks) and pay the per-packet work (r-power scan, finish, slot
//     sum) once per 8 packets of a wave instead of 16; the long ones in 16 lanes keep the slowest wave
//     short (IMIX 40 / 576 / 1500 B, bench.py --workload imix: 32,768 packets 340 -> 428 GiB/s, 65,536
//     517 -> 660, 131,072 607 -> 820; at 16,384 and below the other plans stay 10-13% ahead: DESIGN.md §4.1).
struct SlotPlan {
  uint32_t G;      // lanes per slot
  uint32_t split;  // > 0: one packet per slot, packets of more than `split` 8-block rounds in 16-lane slots
  uint32_t gs = 8;  // with a split: lanes of the other packets' slots (8 or 4)
};
constexpr uint32_t kSlot4MaxLen = 2048;
inline int rw_row(uint32_t G) { return G == 16 ? 1 : G == 4 ? 2 : 0; }
SlotPlan slot_plan(const wg_ctx* c, uint32_t flags, uint32_t n, uint32_t max_len) {
  if (flags & WG_F_UNIFORM)  // small uniform batches: twice the waves in 16-lane slots (8192 x 1420 B: 665 -> 750 GiB/s)
    return {c->uniform16 > 0 && (uint64_t)n * c->uniform16 <= 8ull * c->resident_waves[0][0] ? 16u : 8u, 0u};
  if (c->mixed_split > 0) return {8u, c->mixed_split, c->slot4 == 2 ? 4u : 8u};
  if (c->slot4 == 1) return {4u, 0u};
  if (c->slot4 == 2) return {8u, 2u, 4u};
  if (c->slot16 >= 0) return {c->slot16 ? 16u : 8u, 0u};
  const uint64_t s8 = 8ull * c->resident_waves[0][0];
  if (8ull * n >= 3ull * s8 && c->slot4 != 0 && max_len <= kSlot4MaxLen) return {8u, 2u, 4u};
  if (4ull * n >= 3ull * s8) return {8u, 0u};
  if (8ull * n >= 3ull * s8) return {16u, 0u};
  return {8u, 1u};
}

// Transport seal/open through k_transport: persistent slots, 64 / G per wave. Each slot takes
// ceil(n / resident slots) packets; mixed-length batches are ordered longest-first on
// the device first (k_lpt_*), so the slots' snake over the order balances their rounds.
// A launch that brings its own key table (the asynchronous queue: one key per ring slot, copied at
// submit time) runs the transport kernel whatever kernel the context selects, touches no state shared
// with the context's other callers (no plan workspace, no timing events) and so needs no c->mu.
struct OwnKeys {
  const uint32_t* keys;  // device-readable table, 8 words per entry
  uint32_t slots;
};

template <int MODE>
int launch_transport(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                     uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, hipStream_t s,
                     const wgt::RxTables* rx = nullptr, DevBuf* own_hist = nullptr, DevBuf* own_order = nullptr,
                     bool reuse_order = false, const OwnKeys* own_keys = nullptr) {
  if (n == 0) return WG_OK;
  if (!desc || (((uintptr_t)desc) & 15u)) return fail(WG_EINVAL, "descriptor array must be non-NULL and 16-byte aligned");
  if (!in || !out) return fail(WG_EINVAL, "NULL buffer");
  if (max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", max_len);
  // an open whose buffers overlap runs the transport kernel whatever kernel is selected: only its
  // verify-first variant leaves a forged in-place packet's bytes untouched (ChaCha20Poly1305.java:40-56),
  // and every selectable kernel must write identical bytes (include/wgaead.h)
  int kern = own_keys ? (int)KERN_TRANSPORT : c->kern;
  if (MODE == WG_MODE_OPEN && kern != KERN_TRANSPORT && open_overlaps(in, in_size, out, out_size)) kern = KERN_TRANSPORT;
  if (rx && kern != KERN_TRANSPORT) return fail(WG_EINVAL, "WG_F_RX_FILTER needs the transport kernel");
  // k_tile's uniform plan sizes every tile for max_len-long packets; WG_F_UNIFORM is only a
  // scheduling hint of the transport API, so the tile kernel always plans from the lengths
  if (kern == KERN_TILE)
    return launch_tiles<MODE, false>(c, desc, n, in, in_size, nullptr, 0, out, out_size, status, max_len,
                                     flags & ~WG_F_UNIFORM, s);
  if (kern == KERN_WAVE1) {
    wgk::StreamParams P{};
    P.desc = desc;
    P.n = n;
    P.ppw = (flags & WG_F_UNIFORM) ? 8u : 16u;
    P.max_len = max_len;
    P.key_slots = c->key_slots;
    P.in = in;
    P.in_size = in_size;
    P.out = out;
    P.out_size = out_size;
    P.keys = c->keys;
    P.status = status;
    hipEvent_t ev;
    record_start(c, s, &ev);
    hipLaunchKernelGGL((wgk::k_wave<MODE, 5, 1>), dim3((n + P.ppw - 1) / P.ppw), dim3(64), 0, s, P);
    const hipError_t e = hipGetLastError();
    record_end(c, s, ev);
    if (e != hipSuccess) return fail(WG_EDEVICE, "k_wave launch: %s", hipGetErrorString(e));
    return WG_OK;
  }
  wgt::TransportParams P{};
  uint32_t grid = 0;
  bool ordered = false;
  const SlotPlan sp = slot_plan(c, flags, n, max_len);
  const uint32_t G = sp.G;
  const uint64_t cap_waves = std::max<uint32_t>(c->resident_waves[rw_row(G)][MODE == WG_MODE_OPEN], wgt::TW);
  const bool own = own_hist && own_order;  // the caller holds the plan workspace (launch_after_seal)
  int rc = plan_transport<MODE>(c, desc, n, in, in_size, out, out_size, status, max_len, flags, s, cap_waves, G,
                                own ? *own_hist : c->lpt_hist, own ? *own_order : c->lpt_order, &P, &grid, &ordered,
                                rx, own, reuse_order, sp.split);
  if (rc != WG_OK) return rc;
  if (own_keys) {
    if (!(flags & WG_F_UNIFORM) && !own) return fail(WG_EINVAL, "own-key launches plan without the shared workspace");
    P.keys = own_keys->keys;
    P.key_slots = own_keys->slots;
  }
  hipEvent_t ev = nullptr;
  if (!own_keys) record_start(c, s, &ev);
  if constexpr (MODE == WG_MODE_OPEN) {
    if (open_overlaps(in, in_size, out, out_size)) {  // in-place opens verify first (k_transport<OPEN, G, true>)
      if (P.n_long && sp.gs == 4)
        hipLaunchKernelGGL((wgt::k_transport_mixed<MODE, true, 4>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
      else if (P.n_long) hipLaunchKernelGGL((wgt::k_transport_mixed<MODE, true>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
      else if (G == 16) hipLaunchKernelGGL((wgt::k_transport<MODE, 16, true>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
      else if (G == 4) hipLaunchKernelGGL((wgt::k_transport<MODE, 4, true>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
      else hipLaunchKernelGGL((wgt::k_transport<MODE, 8, true>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
      const hipError_t e = hipGetLastError();
      record_end(c, s, ev);
      if (e != hipSuccess) return fail(WG_EDEVICE, "k_transport launch: %s", hipGetErrorString(e));
      return ordered ? ws_release(c, s) : WG_OK;
    }
  }
  if (P.n_long && sp.gs == 4)
    hipLaunchKernelGGL((wgt::k_transport_mixed<MODE, false, 4>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
  else if (P.n_long) hipLaunchKernelGGL((wgt::k_transport_mixed<MODE>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
  else if (G == 16) hipLaunchKernelGGL((wgt::k_transport<MODE, 16>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
  else if (G == 4) hipLaunchKernelGGL((wgt::k_transport<MODE, 4>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
  else hipLaunchKernelGGL((wgt::k_transport<MODE, 8>), dim3(grid), dim3(64 * wgt::TW), 0, s, P);
  const hipError_t e = hipGetLastError();
  record_end(c, s, ev);
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_transport launch: %s", hipGetErrorString(e));
  return ordered ? ws_release(c, s) : WG_OK;
}

hipStream_t pick_stream(wg_ctx*, void* stream) { return (hipStream_t)stream; }

// wg_duplex_batch(seal, open | WG_F_AFTER_SEAL): the seal launch, then the open launch of what it
// wrote, on `s`. A mixed-length batch is ordered longest-first once: the open's packets have the
// seal's lengths, so it reuses the seal's order (one k_lpt_* pair per step instead of two). The
// plan workspace is held from the seal's order to the open. Caller holds c->mu.
// The stream's own plan workspace (created on first use), or nullptr when kStreamWS streams have one already.
wg_ctx::StreamWS* stream_ws(wg_ctx* c, hipStream_t s) {
  // a stream being captured into a graph takes the shared workspace, as before: it cannot allocate one, and
  // its workspace's event would be recorded inside the graph
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  for (auto& w : c->stream_ws)
    if (w->s == s) return w.get();
  if (c->stream_ws.size() >= wg_ctx::kStreamWS) return nullptr;
  auto w = std::make_unique<wg_ctx::StreamWS>();
  w->s = s;
  if (hipEventCreateWithFlags(&w->ev, hipEventDisableTiming) != hipSuccess) return nullptr;
  c->stream_ws.push_back(std::move(w));
  return c->stream_ws.back().get();
}

int launch_after_seal(wg_ctx* c, const wg_batch* sb, const wg_batch* ob, hipStream_t s) {
  const bool same_plan = sb->max_len == ob->max_len && (sb->flags & WG_F_UNIFORM) == (ob->flags & WG_F_UNIFORM) &&
                         c->resident_waves[0][0] == c->resident_waves[0][1] &&
                         c->resident_waves[1][0] == c->resident_waves[1][1] &&
                         c->resident_waves[2][0] == c->resident_waves[2][1];
  // a uniform batch is not ordered (one packet per slot): no workspace, and no event record
  // between one step's open and the next step's seal
  const bool ordered = !(sb->flags & WG_F_UNIFORM) || !(ob->flags & WG_F_UNIFORM);
  // one k_step launch: both halves on one grid and one order, so every slot opens what it sealed
  const bool fused = c->kern == KERN_TRANSPORT && !c->step_two_launches && sb->max_len == ob->max_len &&
                     !open_overlaps(ob->in, ob->in_size, ob->out, ob->out_size) &&
                     (sb->flags & WG_F_UNIFORM) == (ob->flags & WG_F_UNIFORM) && !(sb->flags & WG_F_FRAME);
  if (fused) {
    if (sb->n == 0) return WG_OK;
    for (const wg_batch* b : {sb, ob}) {
      if (!b->desc || (((uintptr_t)b->desc) & 15u))
        return fail(WG_EINVAL, "descriptor array must be non-NULL and 16-byte aligned");
      if (!b->in || !b->out) return fail(WG_EINVAL, "NULL buffer");
      if (b->max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", b->max_len);
    }
  }
  int rc;
  // the short-packet split plan in one launch (plan_transport's `one`) on the stream's own workspace
  wg_ctx::StreamWS* pws = nullptr;
  if (fused && c->stream_ws_on && !(sb->flags & WG_F_UNIFORM) && sb->max_len <= 2048u && c->lpt_one &&
      !(c->lpt_fused && !c->stitch) && slot_plan(c, sb->flags, sb->n, sb->max_len).split > 0) {
    pws = stream_ws(c, s);
    if (pws && pws->used && (c->wsev & 2u)) HIPTRY(hipStreamWaitEvent(s, pws->ev, 0));
    // the shared workspace sized too: a later call on a stream being captured into a graph (no workspace of
    // its own, and no allocation possible) plans there
    if (pws && (c->lpt_hist.ensure(2 * wgt::kPlanSet * sizeof(uint32_t)) != WG_OK ||
                c->lpt_order.ensure(sizeof(uint32_t) * wgt::kFastBins * (size_t)sb->n) != WG_OK))
      return WG_ENOMEM;
  }
  hipEvent_t stop_ev = nullptr;  // set when the step kernel's launch records the workspace event itself
  DevBuf& plan_hist = pws ? pws->hist : c->lpt_hist;
  DevBuf& plan_order = pws ? pws->order : c->lpt_order;
  if (ordered && !pws && (rc = ws_acquire(c, s)) != WG_OK) return rc;
  if (fused) {
    const SlotPlan sp = slot_plan(c, sb->flags, sb->n, sb->max_len);
    const uint32_t G = sp.G;
    const uint64_t cap = std::max<uint32_t>(c->resident_waves[rw_row(G)][2], wgt::TW);
    wgt::TransportParams PS{}, PO{};
    uint32_t gs = 0, go = 0;
    bool os = false, oo = false;
    // dynamic claims (WG_CLAIM): mixed lengths on the persistent 8-lane plan with at least two packets
    // per slot (the same test plan_transport makes for its longest-first pairs); up to 64 sub-orders,
    // plan_transport picks how many divide its grid
    uint32_t claim_nc = 0;
    if (c->plan_err && __atomic_load_n(c->plan_err, __ATOMIC_ACQUIRE))
      return fail(WG_EDEVICE, "a k_step_mixed_fused workgroup timed out waiting for its plan");
    // the short-packet plan folded into the step launch (k_step_mixed_fused): a pinned error word first
    bool defer = c->lpt_fused && !c->stitch;
    if (defer && !c->plan_err) {
      void* p = nullptr;
      if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !p) defer = false;
      else {
        memset(p, 0, 64);
        c->plan_err = (uint32_t*)p;
      }
    }
    if (c->claim && !(sb->flags & WG_F_UNIFORM) && sp.split == 0 && G == 8 && 2ull * sb->n > 8ull * cap &&
        c->lpt_claim.ensure(64u * 64u) == WG_OK && c->lpt_chain.ensure(sizeof(uint2) * (size_t)sb->n) == WG_OK)
      claim_nc = 64;
    rc = plan_transport<WG_MODE_SEAL>(c, sb->desc, sb->n, sb->in, sb->in_size, sb->out, sb->out_size, nullptr,
                                      sb->max_len, sb->flags, s, cap, G, plan_hist, plan_order, &PS, &gs, &os,
                                      nullptr, true, false, sp.split, claim_nc ? (uint32_t*)c->lpt_claim.p : nullptr,
                                      claim_nc, &defer, true);
    if (rc == WG_OK)
      rc = plan_transport<WG_MODE_OPEN>(c, ob->desc, ob->n, ob->in, ob->in_size, ob->out, ob->out_size, ob->status,
                                        ob->max_len, ob->flags & ~WG_F_AFTER_SEAL, s, cap, G, plan_hist,
                                        plan_order, &PO, &go, &oo, nullptr, true, true, sp.split, nullptr, 0,
                                        nullptr, true);
    // one issue-priority schedule over the seal and open halves (the rounds of both)
    if (PS.prio_step) PS.prio_step = PO.prio_step = 2u * PS.prio_step;
    if (claim_nc) {
      PS.chain_out = (uint2*)c->lpt_chain.p;
      PO.claim_nc = PS.claim_nc;  // the open half replays the seal's log from the same first positions
      PO.chain_in = (const uint2*)c->lpt_chain.p;
    }
    if (rc == WG_OK && (gs != go || PS.slots != PO.slots || PS.order != PO.order || PS.bin_cnt != PO.bin_cnt))
      rc = fail(WG_EINVAL, "k_step: seal and open plans differ (%u / %u workgroups)", gs, go);
    // a sparse (one-launch) order is read only by k_step_mixed* and k_step<8, 4, ..., kWideBins>
    if (rc == WG_OK && PS.bin_cnt && !PS.n_long && !defer &&
        !(G == 8 && c->step_wpe4 && 2ull * gs * wgt::TW <= cap && !c->stitch && !c->test_flip && !claim_nc))
      rc = fail(WG_EINVAL, "k_step: a sparse plan without the kernel that reads it");
#ifdef WG_DIAG
    if (PO.stamps) PO.stamps += 10ull * gs * wgt::TW;  // the open half's stamps after the seal half's
#endif
    if (rc == WG_OK) {
      hipEvent_t ev;
      record_start(c, s, &ev);
      // the workspace's last-use event rides on the step kernel's own completion signal (hipExtLaunchKernel's
      // stop event): a separate hipEventRecord after the launch costs a 3-us gap between steps (IMIX 6%,
      // profiles/r06_ws_event_ab.jsonl). Not while the stream is being captured into a graph.
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (c->ws_ext && hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone && !ev)
        stop_ev = pws ? pws->ev : (ordered ? c->ev_ws : nullptr);
#define WG_XLAUNCH(kern, grid, block, shm, strm, ...) \
  hipExtLaunchKernelGGL(kern, grid, block, shm, strm, nullptr, stop_ev, 0u, __VA_ARGS__)
      if (defer) {  // the planner's blocks first (as k_lpt_one's grid, with 64 x TW threads each), then the step's
        uint32_t np = std::max<uint32_t>(1u, std::min<uint32_t>(wgt::LPT_MAX_BLOCKS, (sb->n + 1023u) / 1024u));
        if (c->fused_np) np = std::min<uint32_t>(c->fused_np, std::max<uint32_t>(1u, sb->n / 256u));
        uint32_t* cnt = const_cast<uint32_t*>(PS.bin_cnt);
        uint32_t* nxt = (uint32_t*)c->lpt_hist.p + wgt::kPlanSet * c->lpt_hist.par;  // plan_transport flipped par
        uint32_t* err = nullptr;
        HIPTRY(hipHostGetDevicePointer((void**)&err, c->plan_err, 0));
        if (sp.gs == 4)
          WG_XLAUNCH(wgt::k_step_mixed_fused<4>, dim3(np + gs), dim3(64 * wgt::TW), 0, s, PS, PO, np, cnt, nxt, err,
                             c->fused_poll);
        else
          WG_XLAUNCH(wgt::k_step_mixed_fused<8>, dim3(np + gs), dim3(64 * wgt::TW), 0, s, PS, PO, np, cnt, nxt, err,
                             c->fused_poll);
      } else if (claim_nc) WG_XLAUNCH((wgt::k_step_claim<8, 4>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO);
      else if (PS.n_long && sp.gs == 4 && c->stitch)
        WG_XLAUNCH((wgt::k_step_mixed<4, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO);
      else if (PS.n_long && sp.gs == 4 && PS.bin_cnt && c->slot2 && c->slot2 < sp.split && c->key_slots < (1u << 24)) {
        PS.split2 = PO.split2 = c->slot2;  // a third part: the grid's upper bound grows by one workgroup
        WG_XLAUNCH((wgt::k_step_mixed<4, false, 2>), dim3(gs + 1), dim3(64 * wgt::TW), 0, s, PS, PO);
      } else if (PS.n_long && sp.gs == 4) WG_XLAUNCH(wgt::k_step_mixed<4>, dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO);
      else if (PS.n_long && c->stitch)
        WG_XLAUNCH((wgt::k_step_mixed<8, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO);
      else if (PS.n_long) WG_XLAUNCH(wgt::k_step_mixed<8>, dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO);
#ifdef WG_TEST_HOOKS
      else if (c->test_flip && G == 8)  // test hook build: the same body with the tag flip between the halves
        WG_XLAUNCH((wgt::k_step<8, 4, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, c->test_flip);
#endif
      else if (G == 16 && c->stitch)
        WG_XLAUNCH((wgt::k_step<16, WG_STITCH_WPE, false, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (G == 16) WG_XLAUNCH(wgt::k_step<16>, dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (G == 4 && c->stitch)
        WG_XLAUNCH((wgt::k_step<4, WG_STITCH_WPE, false, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (G == 4) WG_XLAUNCH(wgt::k_step<4>, dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (c->step_wpe4 && 2ull * gs * wgt::TW <= cap && c->stitch)
        WG_XLAUNCH((wgt::k_step<8, WG_STITCH_WPE, false, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (c->step_wpe4 && 2ull * gs * wgt::TW <= cap && PS.bin_cnt)  // the wide one-launch plan (sparse order)
        WG_XLAUNCH((wgt::k_step<8, 4, false, false, (int)wgt::kWideBins>), dim3(gs), dim3(64 * wgt::TW), 0, s,
                           PS, PO, 0u);
      else if (c->step_wpe4 && 2ull * gs * wgt::TW <= cap)
        WG_XLAUNCH((wgt::k_step<8, 4>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else if (c->stitch)
        WG_XLAUNCH((wgt::k_step<8, WG_STITCH_WPE, false, true>), dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
      else WG_XLAUNCH(wgt::k_step<8>, dim3(gs), dim3(64 * wgt::TW), 0, s, PS, PO, 0u);
#undef WG_XLAUNCH
      const hipError_t e = hipGetLastError();
      record_end(c, s, ev);
      if (e != hipSuccess) rc = fail(WG_EDEVICE, "k_step launch: %s", hipGetErrorString(e));
    }
  } else {
    rc = launch_transport<WG_MODE_SEAL>(c, sb->desc, sb->n, sb->in, sb->in_size, sb->out, sb->out_size, nullptr,
                                        sb->max_len, sb->flags, s, nullptr, &c->lpt_hist, &c->lpt_order);
    if (rc == WG_OK)
      rc = launch_transport<WG_MODE_OPEN>(c, ob->desc, ob->n, ob->in, ob->in_size, ob->out, ob->out_size, ob->status,
                                          ob->max_len, ob->flags & ~WG_F_AFTER_SEAL, s, nullptr, &c->lpt_hist,
                                          &c->lpt_order, same_plan);
  }
  if (pws) {  // the workspace's last use, for the next call that takes it
    if (stop_ev && rc == WG_OK) {
      pws->used = true;
    } else if (c->wsev & 1u) {
      if (hipEventRecord(pws->ev, s) != hipSuccess) return fail(WG_EDEVICE, "hipEventRecord failed");
      pws->used = true;
    }
    return rc;
  }
  if (ordered && stop_ev && rc == WG_OK) {  // ws_release's record done by the step kernel's completion
    c->ws_stream = s;
    return rc;
  }
  const int rr = ordered ? ws_release(c, s) : WG_OK;
  return rc != WG_OK ? rc : rr;
}

}  // namespace

#include "wg_rx.hip"

extern "C" {

#ifdef WG_DIAG
// diagnostic build only: device buffer of 8 x u64 per wave for k_transport phase cycles
int wg_diag_stamps(void* dev_buf) {
  g_stamps = (uint64_t*)dev_buf;
  return WG_OK;
}
#endif

const char* wg_last_error(void) { return g_err.c_str(); }
const char* wg_version(void) { return "wgaead 0.3.0 gfx950"; }

int wg_ctx_set_kernel(wg_ctx* c, const char* name, uint32_t lanes, uint32_t variant) {
  (void)lanes;
  if (!c) return fail(WG_EINVAL, "ctx is NULL");
  int k;
  if (!name || !strcmp(name, "default") || !strcmp(name, "transport")) k = KERN_TRANSPORT;
  else if (!strcmp(name, "wave1")) k = KERN_WAVE1;
  else if (!strcmp(name, "tile")) k = KERN_TILE;
  else return fail(WG_EINVAL, "unknown transport kernel '%s'", name);
  if (variant > 1u) return fail(WG_EINVAL, "unknown kernel variant %u", variant);
  std::lock_guard<std::mutex> lk(c->mu);
  c->kern = k;
  c->step_two_launches = variant == 1u;
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
  c->ws_stream = (hipStream_t)-1;
  hipDeviceProp_t prop;
  int bl[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  // workgroups per CU of each transport kernel
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_out_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_desc, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_kernel, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_ws, hipEventDisableTiming) != hipSuccess ||
      hipGetDeviceProperties(&prop, device) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[0][0], wgt::k_transport<WG_MODE_SEAL, 8>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[0][1], wgt::k_transport<WG_MODE_OPEN, 8>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[0][2], wgt::k_step<8>, 64 * wgt::TW, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[1][0], wgt::k_transport<WG_MODE_SEAL, 16>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[1][1], wgt::k_transport<WG_MODE_OPEN, 16>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[1][2], wgt::k_step<16>, 64 * wgt::TW, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[2][0], wgt::k_transport<WG_MODE_SEAL, 4>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[2][1], wgt::k_transport<WG_MODE_OPEN, 4>, 64 * wgt::TW, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&bl[2][2], wgt::k_step<4>, 64 * wgt::TW, 0) != hipSuccess ||
      hipMalloc(&c->keys, (size_t)key_slots * 32) != hipSuccess ||
      // on the context's stream, like every later key write: a memset on the null stream can sit
      // behind another context's per-packet server in a shared hardware queue and land AFTER the
      // first wg_keys_set (which runs on this non-blocking stream), zeroing the keys it wrote
      hipMemsetAsync(c->keys, 0, (size_t)key_slots * 32, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    wg_ctx_destroy(c);
    return fail(WG_ENOMEM, "context allocation failed on device %d", device);
  }
  c->key_words.reset(new std::atomic<uint64_t>[(size_t)key_slots * 4]());
  c->key_seq.reset(new std::atomic<uint32_t>[key_slots]());
  c->key_live.reset(new std::atomic<uint32_t>[key_slots]());
  c->cus = (uint32_t)prop.multiProcessorCount;
  for (int w = 0; w < 3; ++w)
    for (int k = 0; k < 3; ++k)
      c->resident_waves[w][k] = (uint32_t)std::max(bl[w][k], 1) * wgt::TW * (uint32_t)prop.multiProcessorCount;
  // Scheduling overrides for A/B measurements (tools/ab_args.sh), read once per context; none
  // changes a byte of output (the parity suite runs each): WG_SLOT16=0|1 (mixed batches in 8- or
  // 16-lane slots), WG_SLOT4=0|1|2 (mixed batches never / always in 4-lane slots /
  // always long ones in 16-lane and the rest in 4-lane slots), WG_MIXED_SPLIT=R (mixed batches one packet per slot, packets of more than R
  // 8-block rounds in 16-lane slots), WG_UNIFORM16=k (uniform batches of at most S8/k packets in
  // 16-lane slots, 0 never), WG_PRIO=0|1 (issue-priority schedule off / on for every batch).
  if (const char* e = getenv("WG_SLOT16")) c->slot16 = atoi(e);
  if (const char* e = getenv("WG_SLOT4")) c->slot4 = atoi(e);
  if (const char* e = getenv("WG_SLOT4_PAIRS")) c->slot4_pairs = atoi(e) != 0;
  if (const char* e = getenv("WG_SLOT4_SNAKE")) c->slot4_snake = atoi(e) != 0;
  if (const char* e = getenv("WG_MIXED_SPLIT")) c->mixed_split = (uint32_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_UNIFORM16")) c->uniform16 = (uint32_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_PRIO")) c->prio_mode = atoi(e);
  if (const char* e = getenv("WG_STEP_WPE4")) c->step_wpe4 = atoi(e) != 0;
  if (const char* e = getenv("WG_CLAIM")) c->claim = atoi(e) != 0;
  if (const char* e = getenv("WG_STITCH")) c->stitch = atoi(e) != 0;
  if (const char* e = getenv("WG_LPT_ONE")) c->lpt_one = atoi(e) != 0;
  if (const char* e = getenv("WG_LPT_WIDE")) c->lpt_wide = atoi(e) != 0;
  if (const char* e = getenv("WG_LPT_FUSED")) c->lpt_fused = atoi(e) != 0;
  if (const char* e = getenv("WG_SLOT2")) c->slot2 = (uint32_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_STREAM_WS")) c->stream_ws_on = atoi(e) != 0;
  if (const char* e = getenv("WG_WSEV")) c->wsev = (uint32_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_WS_EXT")) c->ws_ext = atoi(e) != 0;
  if (const char* e = getenv("WG_FUSED_POLL")) c->fused_poll = (uint32_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_FUSED_NP")) c->fused_np = (uint32_t)std::max(0, atoi(e));
#ifdef WG_TEST_HOOKS
  // fault-injection hooks exist only in the test library (make test: libwgaead_test.so); the product
  // library never reads these variables, so no environment can make it write wrong tags
  if (const char* e = getenv("WG_TEST_STEP_FLIP")) {
    const long v = atol(e);
    c->test_flip = (v > 0 && (v & (v - 1)) == 0) ? (uint32_t)v : 0u;
  }
#endif
  *out = c;
  return WG_OK;
}

int wg_ctx_destroy(wg_ctx* c) {
  if (!c) return WG_OK;
  pp_stop(c);
  if (c->key_words) {
    std::lock_guard<std::mutex> lk(c->keys_mu);
    key_mirror_write(c, 0, c->key_slots, nullptr);
  }
  DeviceGuard g(c->device);
  rx_free(c);
  if (c->keys) {
    (void)hipDeviceSynchronize();  // no launch of this context may still read the table
    (void)hipMemsetAsync(c->keys, 0, (size_t)c->key_slots * 32, c->stream);  // SymmetricKeypair.clean zeroes keys
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->keys);
  }
  for (auto& e : c->events) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  for (DevBuf* b : {&c->plan_nb, &c->plan_prefix, &c->plan_tiles, &c->plan_ntiles, &c->plan_tmp, &c->lpt_hist,
                    &c->lpt_order, &c->lpt_hist2, &c->lpt_order2, &c->lpt_nlong, &c->h_desc, &c->h_in, &c->h_out, &c->h_aad, &c->h_status,
                    &c->h_keys})
    b->release();
  if (c->plan_err) (void)hipHostFree(c->plan_err);
  for (auto& w : c->stream_ws) {
    w->hist.release();
    w->order.release();
    if (w->ev) (void)hipEventDestroy(w->ev);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->copy_out_stream) (void)hipStreamDestroy(c->copy_out_stream);
  for (hipEvent_t e : {c->ev_desc, c->ev_in, c->ev_kernel, c->ev_ws})
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
  std::lock_guard<std::mutex> lk(c->mu);  // the replay-window reset is ordered with queued checks under it
  HIPTRY(hipMemcpyAsync((uint8_t*)c->keys + (size_t)first * 32, keys_host, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
  {
    std::lock_guard<std::mutex> lk2(c->keys_mu);
    key_mirror_write(c, first, n, keys_host);
  }
  int rc;
  if ((rc = rx_reset_slots(c, first, n, c->stream)) != WG_OK) return rc;  // new key: new session
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_keys_zero(wg_ctx* c, uint32_t first, uint32_t n) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if ((uint64_t)first + n > c->key_slots) return fail(WG_ERANGE, "key slots out of range");
  if (!n) return WG_OK;
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  HIPTRY(hipMemsetAsync((uint8_t*)c->keys + (size_t)first * 32, 0, (size_t)n * 32, c->stream));
  {
    std::lock_guard<std::mutex> lk2(c->keys_mu);
    key_mirror_write(c, first, n, nullptr);
  }
  int rc;
  if ((rc = rx_reset_slots(c, first, n, c->stream)) != WG_OK) return rc;
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_seal_batch(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                  uint64_t out_size, uint32_t max_len, uint32_t flags, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (flags & ~kFlagsKnown) return fail(WG_EINVAL, "unknown flag bits 0x%x", flags & ~kFlagsKnown);
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  if ((flags & WG_F_FRAME) && !c->receivers) return fail(WG_EINVAL, "WG_F_FRAME without a receiver table (wg_ctx_set_receivers)");
  hipStream_t s = pick_stream(c, stream);
  const int rc = launch_transport<WG_MODE_SEAL>(c, desc, n, in, in_size, out, out_size, nullptr, max_len, flags, s);
  // measured in round 1: writing the header inside the AEAD kernel cost the seal launch
  // +11%, so the header is a separate launch on the same stream
  if (rc != WG_OK || !(flags & WG_F_FRAME) || n == 0) return rc;
  hipLaunchKernelGGL(wgt::k_frame_seal, dim3((n + 255u) / 256u), dim3(256), 0, s, desc, n, c->receivers, max_len,
                     c->key_slots, in_size, out, out_size);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_frame_seal launch: %s", hipGetErrorString(e));
  return WG_OK;
}

int wg_ctx_set_receivers(wg_ctx* c, const uint32_t* receivers, uint32_t n) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (receivers && n < c->key_slots)
    return fail(WG_ERANGE, "receiver table of %u entries for %u key slots", n, c->key_slots);
  if (receivers) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, receivers) != hipSuccess || a.type != hipMemoryTypeDevice || a.device != c->device) {
      (void)hipGetLastError();
      return fail(WG_EINVAL, "receiver table must be device memory on device %d", c->device);
    }
    if (((uintptr_t)receivers) & 3u) return fail(WG_EINVAL, "receiver table must be 4-byte aligned");
  }
  std::lock_guard<std::mutex> lk(c->mu);
  c->receivers = receivers;
  return WG_OK;
}

int wg_open_batch(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* in, uint64_t in_size, uint8_t* out,
                  uint64_t out_size, uint32_t* status, uint32_t max_len, uint32_t flags, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (flags & ~(WG_F_UNIFORM | WG_F_RX_FILTER))
    return fail(WG_EINVAL, "open takes only WG_F_UNIFORM | WG_F_RX_FILTER (flags 0x%x)", flags);
  if (n && !status) return fail(WG_EINVAL, "open needs a status array");
  DeviceGuard g(c->device);
  std::lock_guard<std::mutex> lk(c->mu);
  const wgt::RxTables* rx = nullptr;
  if (flags & WG_F_RX_FILTER) {
    int rc;
    if ((rc = rx_tables(c, &rx)) != WG_OK) return rc;
  }
  return launch_transport<WG_MODE_OPEN>(c, desc, n, in, in_size, out, out_size, status, max_len,
                                       flags & ~WG_F_RX_FILTER, pick_stream(c, stream), rx);
}

// Seal one batch and open another in one k_duplex launch (wg_duplex_batch).
int wg_duplex_batch(wg_ctx* c, const wg_batch* sb, const wg_batch* ob, void* stream) {
  if (!c || !sb || !ob) return fail(WG_EINVAL, "NULL argument");
  if (sb->flags & ~kFlagsKnown) return fail(WG_EINVAL, "unknown seal flag bits 0x%x", sb->flags & ~kFlagsKnown);
  if (ob->flags & ~(WG_F_UNIFORM | WG_F_AFTER_SEAL))
    return fail(WG_EINVAL, "open takes only WG_F_UNIFORM | WG_F_AFTER_SEAL (flags 0x%x)", ob->flags);
  if (ob->n && !ob->status) return fail(WG_EINVAL, "open needs a status array");
  const bool after = (ob->flags & WG_F_AFTER_SEAL) != 0;
  if (after && sb->n != ob->n) return fail(WG_EINVAL, "WG_F_AFTER_SEAL needs equal batch sizes (%u, %u)", sb->n, ob->n);
  DeviceGuard g(c->device);
  hipStream_t s = pick_stream(c, stream);
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if ((sb->flags & WG_F_FRAME) && !c->receivers)
      return fail(WG_EINVAL, "WG_F_FRAME without a receiver table (wg_ctx_set_receivers)");
    const bool fused = !after && c->kern == KERN_TRANSPORT && sb->n && ob->n &&
                       !open_overlaps(ob->in, ob->in_size, ob->out, ob->out_size);
    if (after && c->kern == KERN_TRANSPORT && sb->n) {
      int rc = launch_after_seal(c, sb, ob, s);
      if (rc != WG_OK) return rc;
    } else if (fused) {
      for (const wg_batch* b : {sb, ob}) {
        if (!b->desc || (((uintptr_t)b->desc) & 15u))
          return fail(WG_EINVAL, "descriptor array must be non-NULL and 16-byte aligned");
        if (!b->in || !b->out) return fail(WG_EINVAL, "NULL buffer");
        if (b->max_len > WG_MAX_PACKET) return fail(WG_E2BIG, "max_len %u > WG_MAX_PACKET", b->max_len);
      }
      // the two halves share the machine: each plans with half of the resident slots
      const uint64_t cap = std::max<uint32_t>(std::min(c->resident_waves[0][0], c->resident_waves[0][1]) / 2u, wgt::TW);
      wgt::TransportParams PS{}, PO{};
      uint32_t gs = 0, go = 0;
      bool os = false, oo = false;
      int rc = plan_transport<WG_MODE_SEAL>(c, sb->desc, sb->n, sb->in, sb->in_size, sb->out, sb->out_size, nullptr,
                                            sb->max_len, sb->flags, s, cap, 8u, c->lpt_hist, c->lpt_order, &PS, &gs, &os);
      if (rc != WG_OK) return rc;
      rc = plan_transport<WG_MODE_OPEN>(c, ob->desc, ob->n, ob->in, ob->in_size, ob->out, ob->out_size, ob->status,
                                        ob->max_len, ob->flags, s, cap, 8u, c->lpt_hist2, c->lpt_order2, &PO, &go, &oo);
      if (rc != WG_OK) return rc;
      hipEvent_t ev;
      record_start(c, s, &ev);
      hipLaunchKernelGGL(wgt::k_duplex, dim3(gs + go), dim3(64 * wgt::TW), 0, s, PS, PO, gs, go);
      const hipError_t e = hipGetLastError();
      record_end(c, s, ev);
      if (e != hipSuccess) return fail(WG_EDEVICE, "k_duplex launch: %s", hipGetErrorString(e));
      if ((os || oo) && (rc = ws_release(c, s)) != WG_OK) return rc;
    } else {  // another kernel selected, or one side empty: the two launches in turn
      int rc = launch_transport<WG_MODE_SEAL>(c, sb->desc, sb->n, sb->in, sb->in_size, sb->out, sb->out_size, nullptr,
                                              sb->max_len, sb->flags, s);
      if (rc != WG_OK) return rc;
      rc = launch_transport<WG_MODE_OPEN>(c, ob->desc, ob->n, ob->in, ob->in_size, ob->out, ob->out_size, ob->status,
                                          ob->max_len, ob->flags & ~WG_F_AFTER_SEAL, s);
      if (rc != WG_OK) return rc;
    }
    if (!(sb->flags & WG_F_FRAME) || sb->n == 0) return WG_OK;
    hipLaunchKernelGGL(wgt::k_frame_seal, dim3((sb->n + 255u) / 256u), dim3(256), 0, s, sb->desc, sb->n, c->receivers,
                       sb->max_len, c->key_slots, sb->in_size, sb->out, sb->out_size);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EDEVICE, "k_frame_seal launch: %s", hipGetErrorString(e));
  }
  return WG_OK;
}

int wg_frame_seal(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint32_t* receivers, uint8_t* out,
                  uint64_t out_size, uint64_t in_size, uint32_t max_len, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (n == 0) return WG_OK;
  if (!desc || !receivers || !out) return fail(WG_EINVAL, "NULL descriptor, receiver table or output buffer");
  DeviceGuard g(c->device);
  hipStream_t s = pick_stream(c, stream);
  hipLaunchKernelGGL(wgt::k_frame_seal, dim3((n + 255u) / 256u), dim3(256), 0, s, desc, n, receivers, max_len,
                     c->key_slots, in_size, out, out_size);
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
  hipLaunchKernelGGL(wgt::k_parse_open, dim3((n + 255u) / 256u), dim3(256), 0, s, wire, wire_size, pkt_off, pkt_len,
                     key_slot, n, desc_out, parse_status);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(WG_EDEVICE, "k_parse_open launch: %s", hipGetErrorString(e));
  return WG_OK;
}

int wg_aead_batch(wg_ctx* c, int mode, const wg_aead_desc* desc, uint32_t n, const uint8_t* in, uint64_t in_size,
                  const uint8_t* aad, uint64_t aad_size, uint8_t* out, uint64_t out_size, uint32_t* status,
                  uint32_t max_len, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (mode == WG_MODE_OPEN && n && !status) return fail(WG_EINVAL, "open needs a status array");
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

}  // extern "C"

#include "wg_host.hip"
#include "wg_pp.hip"
#include "wg_queue.hip"

extern "C" {

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
  // the transport kernel itself: one 1420-B seal + open through k_transport (RFC 8439
  // vectors above pin k_tile; this pins the product transport path against the same key)
  {
    uint8_t* dbuf = nullptr;
    const uint32_t TL = 1420, S = 1440;
    if (wg_keys_set(c, 0, 1, key) != WG_OK || hipMalloc(&dbuf, 3 * S + 128) != hipSuccess) {
      ok = 0;
    } else {
      std::vector<uint8_t> h(3 * S + 128, 0);
      for (uint32_t i = 0; i < TL; ++i) h[i] = (uint8_t)(i * 7 + 3);
      wg_pkt* dd = (wg_pkt*)(dbuf + 3 * S);
      wg_pkt hd[2] = {{0, S, 5, TL, 0}, {S, 2 * S, 5, TL, 0}};
      uint32_t* st = (uint32_t*)(dbuf + 3 * S + 64);
      if (hipMemcpy(dbuf, h.data(), 3 * S, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(dd, hd, sizeof hd, hipMemcpyHostToDevice) != hipSuccess ||
          wg_seal_batch(c, dd, 1, dbuf, 3 * S, dbuf, 3 * S, TL, WG_F_UNIFORM, c->stream) != WG_OK ||
          wg_open_batch(c, dd + 1, 1, dbuf, 3 * S, dbuf, 3 * S, st, TL, WG_F_UNIFORM, c->stream) != WG_OK ||
          hipStreamSynchronize(c->stream) != hipSuccess ||
          hipMemcpy(h.data(), dbuf, 3 * S + 128, hipMemcpyDeviceToHost) != hipSuccess)
        ok = 0;
      else if (memcmp(h.data(), h.data() + 2 * S, TL) != 0 || *(uint32_t*)(h.data() + 3 * S + 64) != WG_PKT_OK)
        ok = 0;
      (void)hipFree(dbuf);
    }
  }
  wg_ctx_destroy(c);
  return ok;
}

}  // extern "C"
