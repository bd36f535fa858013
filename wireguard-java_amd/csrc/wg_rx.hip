// wg_rx.hip — receive-side checks after open, on the device (included by wg_capi.hip).
//
// The reference hands every opened packet to TransportManager.processDecryptedTransport
// (TransportManager.java:98-119): a zero-length plaintext is a keepalive and is not
// forwarded (:103-105); otherwise the destination address (destinationIPOf, :124-130:
// bytes 16..19 of an IPv4 header, 24..39 of an IPv6 header, anything else throws) must
// be inside the peer's AllowedIPs (IPFilter.search, util/IPFilter.java:49-61) or the
// packet is dropped (:106-108). wg_rx_check does the same for a whole opened batch and
// reports the outcome in the status array, after an optional anti-replay window
// (WG_RX_REPLAY) that the reference does not have.
//
// AllowedIPs on the device. IPFilter is a binary trie walked one bit per step; search()
// reports a match if any node it passes at depths 0 .. nbits-1 ends a subnet, and it
// stops at the first missing child. Note the depth-nbits node is never tested, so a /32
// (or /128) entry never matches; IPFilter.allowingAll() inserts exactly such entries
// (0.0.0.0/32, ::/128) and so matches nothing. The device keeps that behaviour: the
// binary trie is compiled on the host into stride-8 tables (one 256-entry node per trie
// node at a depth that is a multiple of 8; entry = next node | "a subnet ended on the
// way", bit 31), so a lookup is 4 (IPv4) or 16 (IPv6) dependent table reads instead of
// 32 or 128.
//
// Replay window (WG_RX_REPLAY, WireGuard whitepaper §5.4.6 / RFC 6479 style): per key
// slot, `top` = highest accepted counter + 1 and a ring bitmap of the last W counters.
// A batch is checked against the window as it stood before the batch:
//   - counters >= 2^64 - 2^13 - 1 (Reject-After-Messages) are rejected;
//   - of several authenticated packets with the same (slot, counter) in one batch only
//     the first (lowest index) can be accepted;
//   - counter >= top is accepted; top - counter > W is too old; otherwise it is accepted
//     iff its bit is clear.
// Then the window advances to the largest accepted counter and records every accepted
// counter still inside it. The window thus slides between batches: a packet older than
// W behind an EARLIER packet of the same batch (but not behind the window at the batch's
// start) is accepted, where a one-packet-at-a-time window would reject it. No counter is
// ever accepted twice. oracle/rx.py restates these rules one packet at a time.
// Kernels: k_rp_order flags a batch whose (slot, counter) pairs do not strictly increase with
// the index (only then can a pair repeat); k_rp_insert claims one entry per (slot, counter) pair in an open-addressing table
// (lowest index by atomicMin). By default k_rp_judge raises the flag and judges every packet against
// the old window as if no pair repeated (its last block then moves each slot's window; a separate
// k_rp_advance for tables of more than 512 slots), k_rp_insert fills the table only for a flagged
// batch, and k_rp_fixmark turns every copy of a repeated pair but the lowest into REPLAY, sets the
// ring bits and empties the table again. Atomics on a shared address (a
// slot's new top, a window word) are aggregated per workgroup first; new tops are spread over 8
// copies per slot.
#pragma once

namespace {

constexpr uint32_t kRxNoFilter = 0xFFFFFFFFu;
constexpr uint64_t kRejectAfter = ~0ull - 8191ull - 1ull;  // 2^64 - 2^13 - 1
constexpr uint64_t kEmptyKey = ~0ull;                      // counters that large are rejected first
constexpr uint32_t kTopWays = 8;         // copies of each slot's new top (spread same-address atomics)
constexpr size_t kFlagBytes = 64 * (2 + kTopWays);  // order flags (2) | done count | kTopWays group counts
// key slots the last block of k_rp_judge advances: one peer's 64K packets in order 25 us per
// check against 31 as separate launches, but 1024 interleaved slots 65 against 60 (the last block
// walks every slot), so larger tables launch the advance (profiles/r04_rx_launches.txt)
constexpr uint32_t kAdvanceInline = 512;

struct RxState {
  // AllowedIPs: host copies of each filter's compiled tables; device image rebuilt on change
  std::vector<std::vector<uint32_t>> filt_entries;  // per filter: nodes x 256 entries (node 0 = none)
  std::vector<std::pair<uint32_t, uint32_t>> filt_roots;  // per filter: (root4, root6) node index in its own table
  DevBuf d_entries, d_hdr, d_slot_filter;
  bool slot_filter_init = false;
  // replay window
  uint32_t window = 0;      // W bits (0: disabled)
  DevBuf d_top, d_bits;     // per slot: u64 top; W/64 u64 words
  DevBuf d_newtop;          // per slot, kTopWays copies: the window's new top while a batch is checked (== top between calls)
  DevBuf d_tab;             // (slot, counter) -> lowest batch index, open addressing; all empty between calls
  uint32_t tab_size = 0;    // entries (a power of two >= 2n)
  DevBuf d_pos;             // per packet: its (slot, counter) entry in d_tab, or ~0
  DevBuf d_flag;            // the order flag, k_rp_judge's finished blocks and groups, 64 B apart (0 between calls)
  bool five = false;        // WG_RX_LAUNCHES=5: decide and advance as two launches (A/B)
  // test hooks (tests/test_gpu_rx.py::test_replay_flag_protocol_under_block_skew), never set in production:
  // WG_RX_TEST_SKEW=us delays every block but block 0 of each replay launch by `us` before it reads
  // the order flag, the done counts or the new tops; WG_RX_TEST_MUTANT=1 restores round 4's flag
  // clearing (k_rp_fixmark clears the word its own later blocks read) so the test can show it fails
  uint32_t test_skew_ticks = 0;  // s_memrealtime ticks (100 MHz)
  bool test_mutant = false;
  uint64_t checks = 0;      // replay checks queued: the order flag alternates between two words
  hipEvent_t ev = nullptr;  // last use of the replay scratch, and its stream (stream-ordered reuse)
  hipStream_t ev_stream = (hipStream_t)-1;
  DevBuf d_tables;          // wgt::RxTables for the fused open (WG_F_RX_FILTER)
  bool tables_valid = false;
};

// ---- host: IPFilter.insert as a binary trie, then stride-8 tables -------------------------
struct BinTrie {
  std::vector<std::array<int32_t, 2>> child{{{-1, -1}}};
  std::vector<uint8_t> end{0};
  void insert(const uint8_t* addr, uint32_t prefix_len) {  // IPFilter.insert (:30-42)
    int32_t node = 0;
    for (uint32_t i = 0; i < prefix_len; ++i) {
      const int bit = (addr[i / 8] >> (7 - i % 8)) & 1;
      if (child[node][bit] < 0) {
        child[node][bit] = (int32_t)child.size();
        child.push_back({-1, -1});
        end.push_back(0);
      }
      node = child[node][bit];
    }
    end[node] = 1;
  }
};

// node at depth 8L -> 256 entries; returns its index in `out` (>= 1)
uint32_t compile_level(const BinTrie& t, int32_t bnode, uint32_t depth, uint32_t nbits, std::vector<uint32_t>& out) {
  const uint32_t me = (uint32_t)(out.size() / 256);
  out.resize(out.size() + 256, 0u);
  for (uint32_t v = 0; v < 256; ++v) {
    bool found = false, reached = true;
    int32_t cur = bnode;
    for (uint32_t k = 0; k < 8; ++k) {  // IPFilter.search (:52-59): test, then descend
      if (t.end[cur]) found = true;
      cur = t.child[cur][(v >> (7 - k)) & 1];
      if (cur < 0) {
        reached = false;
        break;
      }
    }
    uint32_t next = 0;
    if (reached && depth + 8 < nbits) next = compile_level(t, cur, depth + 8, nbits, out);
    out[(size_t)me * 256 + v] = next | (found ? 0x80000000u : 0u);
  }
  return me;
}

int rx_get(wg_ctx* c, RxState** out) {
  if (!c->rx) {
    c->rx = new RxState();
    if (const char* e = getenv("WG_RX_LAUNCHES")) c->rx->five = atoi(e) == 5;
#ifdef WG_TEST_HOOKS  // the test library only (libwgaead_test.so): never read by the product library
    if (const char* e = getenv("WG_RX_TEST_SKEW")) c->rx->test_skew_ticks = 100u * (uint32_t)std::max(0, atoi(e));
    if (const char* e = getenv("WG_RX_TEST_MUTANT")) c->rx->test_mutant = atoi(e) != 0;
#endif
  }
  *out = c->rx;
  return WG_OK;
}

void rx_free(wg_ctx* c) {
  if (!c->rx) return;
  RxState* r = c->rx;
  for (DevBuf* b : {&r->d_entries, &r->d_hdr, &r->d_slot_filter, &r->d_top, &r->d_bits, &r->d_newtop, &r->d_tab,
                    &r->d_pos, &r->d_flag, &r->d_tables})
    b->release();
  if (r->ev) (void)hipEventDestroy(r->ev);
  delete r;
  c->rx = nullptr;
}

// The RxTables struct the fused open reads (wg_open_batch with WG_F_RX_FILTER), rebuilt after
// every filter / slot-map change. Caller holds c->mu.
int rx_tables(wg_ctx* c, const wgt::RxTables** out) {
  RxState* r;
  rx_get(c, &r);
  int rc;
  if ((rc = r->d_tables.ensure(sizeof(wgt::RxTables))) != WG_OK) return rc;
  if (!r->tables_valid) {
    const wgt::RxTables T{r->slot_filter_init ? (const uint32_t*)r->d_slot_filter.p : nullptr,
                          (const uint32_t*)r->d_hdr.p, (const uint32_t*)r->d_entries.p,
                          (uint32_t)r->filt_roots.size(), c->key_slots};
    DeviceGuard g(c->device);
    HIPTRY(hipMemcpyAsync(r->d_tables.p, &T, sizeof T, hipMemcpyHostToDevice, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    r->tables_valid = true;
  }
  *out = (const wgt::RxTables*)r->d_tables.p;
  return WG_OK;
}

// Orders stream s behind the last replay check (which may sit on another stream): the window
// state is read and written by the check's kernels, so a reset or a state read must not overtake
// them. Caller holds c->mu.
int rx_after_last_check(RxState* r, hipStream_t s) {
  if (r->ev && r->ev_stream != s && r->ev_stream != (hipStream_t)-1) HIPTRY(hipStreamWaitEvent(s, r->ev, 0));
  return WG_OK;
}

// zero the replay window of key slots [first, first + n) (a new key = a new session), in stream
// order after every replay check queued before it; later checks (any stream) wait for the reset.
// Caller holds c->mu.
int rx_reset_slots(wg_ctx* c, uint32_t first, uint32_t n, hipStream_t s) {
  RxState* r = c->rx;
  if (!r || !r->window || !n) return WG_OK;
  int rc;
  if ((rc = rx_after_last_check(r, s)) != WG_OK) return rc;
  HIPTRY(hipMemsetAsync((uint64_t*)r->d_top.p + first, 0, (size_t)n * 8, s));
  HIPTRY(hipMemsetAsync((uint64_t*)r->d_newtop.p + (size_t)first * kTopWays, 0, (size_t)n * 8 * kTopWays, s));
  const size_t words = r->window / 64;
  HIPTRY(hipMemsetAsync((uint64_t*)r->d_bits.p + (size_t)first * words, 0, (size_t)n * words * 8, s));
  if (!r->ev) HIPTRY(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming));
  HIPTRY(hipEventRecord(r->ev, s));
  r->ev_stream = s;
  return WG_OK;
}

}  // namespace

// ---- device -------------------------------------------------------------------------------
namespace wgrx {

struct RxParams {
  const wg_pkt* desc;
  uint32_t n;
  const uint8_t* pt;
  uint64_t pt_size;
  uint32_t* status;
  uint32_t key_slots;
  // filter
  const uint32_t* slot_filter;  // per slot: filter id or kRxNoFilter (NULL: no filters)
  const uint32_t* hdr;          // per filter: root4, root6 (global node indices)
  const uint32_t* entries;      // global nodes x 256
  uint32_t nfilters;
  // replay
  uint32_t window;
  uint64_t* top;
  uint64_t* bits;
  uint64_t* newtop;
  uint32_t* tab;
  uint32_t tab_size;
  uint32_t* pos;
  uint32_t* unsorted;  // 0 while the batch's (slot, counter) pairs strictly increase with the index
  uint32_t* unsorted_next;  // the next check's flag word (checks alternate between two words)
  uint32_t* done_blocks;  // k_rp_judge: blocks finished (0 between calls)
  uint32_t skew_ticks;    // test hook WG_RX_TEST_SKEW (0 in production)
  uint32_t mutant;        // test hook WG_RX_TEST_MUTANT (0 in production)
};

// Test hook: every block but block 0 waits skew_ticks (s_memrealtime, 100 MHz) before it touches the
// check's shared words, so block 0 runs its whole part first. A protocol in which an early block
// clears or consumes a word a later block of the same launch still reads then fails every time.
__device__ __forceinline__ void rx_test_skew(const RxParams& P) {
#ifndef WG_TEST_HOOKS
  return;  // the product library carries no skew code
#endif
  if (P.skew_ticks == 0u || blockIdx.x == 0u) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)P.skew_ticks) __builtin_amdgcn_s_sleep(8);
}

// Words shared between launches are reset with device-scope (agent) atomic stores: they bypass the
// XCD's L2, like the atomics that read and raise them, so no write-back of that L2 is needed for
// another XCD's blocks of the next launch to see the reset.
__device__ __forceinline__ void reset_word(uint32_t* p) {
  __hip_atomic_store(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Many lanes of a batch usually share a key slot (and a window word): one atomic per distinct
// key and wave instead of one per lane (65536 same-address atomics serialise at the L2).
// Reductions over a group use DPP row shifts / broadcasts (no LDS traffic); lane 63 ends
// with the whole wave's result.
template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, BANK_MASK, false);
}
template <bool OR>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {  // max or or over the wave (identity 0)
  auto op = [](uint32_t a, uint32_t b) { return OR ? (a | b) : (a > b ? a : b); };
  uint32_t r = op(v, dpp<0x111, 0xf, 0xf>(v));  // row_shr:1
  r = op(r, dpp<0x112, 0xf, 0xf>(v));           // row_shr:2
  r = op(r, dpp<0x113, 0xf, 0xf>(v));           // row_shr:3
  r = op(r, dpp<0x114, 0xf, 0xe>(r));           // row_shr:4, banks 1-3
  r = op(r, dpp<0x118, 0xf, 0xc>(r));           // row_shr:8, banks 2-3
  r = op(r, dpp<0x142, 0xa, 0xf>(r));           // row_bcast:15 into rows 1, 3
  r = op(r, dpp<0x143, 0xc, 0xf>(r));           // row_bcast:31 into rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)r, 63);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src) << 32);
}
// calls f(key, count, max, or) on the leader lane of every distinct key among active lanes
// (every lane of the wave must reach this call); MAX / OR select the reductions computed
template <bool MAX, bool OR, class F>
__device__ __forceinline__ void wave_group(bool active, uint64_t key, uint64_t val, F f) {
  const int lane = (int)(threadIdx.x & 63u);
  for (;;) {
    const uint64_t act = __ballot(active);
    if (!act) break;
    const int leader = __ffsll((unsigned long long)act) - 1;
    const uint64_t lk = shfl_u64(key, leader);
    const bool mine = active && key == lk;
    const uint64_t m = __ballot(mine);
    if (__popcll(m) == 1) {  // keys mostly distinct in this wave: one atomic per lane (no contention)
      if (active) f(key, 1u, val, val);
      break;
    }
    uint64_t mx = 0, orv = 0;
    if constexpr (MAX) {
      const uint32_t hi = wave_reduce<false>(mine ? (uint32_t)(val >> 32) : 0u);
      const uint32_t lo = wave_reduce<false>(mine && (uint32_t)(val >> 32) == hi ? (uint32_t)val : 0u);
      mx = ((uint64_t)hi << 32) | lo;
    }
    if constexpr (OR) {
      const uint32_t hi = wave_reduce<true>(mine ? (uint32_t)(val >> 32) : 0u);
      const uint32_t lo = wave_reduce<true>(mine ? (uint32_t)val : 0u);
      orv = ((uint64_t)hi << 32) | lo;
    }
    if (lane == leader) f(lk, (uint32_t)__popcll(m), mx, orv);
    if (mine) active = false;
  }
}

__device__ __forceinline__ bool rp_candidate(const RxParams& P, uint32_t i, uint32_t& slot, uint64_t& ctr) {
  if (P.status[i] != WG_PKT_OK) return false;
  const wg_pkt d = P.desc[i];
  if (d.key_slot >= P.key_slots) return false;
  slot = d.key_slot;
  ctr = d.counter;
  return true;
}

// A whole workgroup's atomics per distinct key: every wave groups its lanes by key
// (wave_group), the groups' leaders list (key, max, or) in LDS, and one lane per distinct key
// of the workgroup issues the atomic (a single-slot batch: one atomic per workgroup instead of
// one per wave; same-address atomics serialise). Every thread of the block must call it.
constexpr uint32_t kGroupCap = 64;
template <bool MAX, bool OR, class F>
__device__ __forceinline__ void block_group(bool active, uint64_t key, uint64_t val, F f) {
  __shared__ uint64_t g_key[kGroupCap], g_max[kGroupCap], g_or[kGroupCap];
  __shared__ uint32_t g_n;
  if (threadIdx.x == 0) g_n = 0;
  __syncthreads();
  wave_group<MAX, OR>(active, key, val, [&](uint64_t k, uint32_t, uint64_t mx, uint64_t orv) {
    const uint32_t e = atomicAdd(&g_n, 1u);
    if (e < kGroupCap) {
      g_key[e] = k;
      g_max[e] = mx;
      g_or[e] = orv;
    } else {
      f(k, mx, orv);  // more distinct keys than the list holds: this group's atomic directly
    }
  });
  __syncthreads();
  const uint32_t cnt = min(g_n, kGroupCap);
  if (threadIdx.x < cnt) {
    const uint64_t k = g_key[threadIdx.x];
    bool first = true;
    for (uint32_t e = 0; e < threadIdx.x; ++e) first = first && g_key[e] != k;
    if (first) {
      uint64_t mx = 0, orv = 0;
      for (uint32_t e = threadIdx.x; e < cnt; ++e)
        if (g_key[e] == k) {
          mx = g_max[e] > mx ? g_max[e] : mx;
          orv |= g_or[e];
        }
      f(k, mx, orv);
    }
  }
}

// entry of (slot, counter) in the table of `size` (a power of two) entries (multiply-high)
__device__ __forceinline__ uint32_t rp_hash(uint32_t slot, uint64_t c, uint32_t size) {
  return (uint32_t)__umul64hi(mix64(c ^ ((uint64_t)slot * 0x9E3779B97F4A7C15ull)), (uint64_t)size);
}

// A batch whose (key slot, counter) pairs strictly increase with the batch index (one peer's
// in-order stream, or streams sorted by slot) holds no pair twice: the table is skipped. Only
// a wave that finds an out-of-order neighbour raises the flag (no atomics in the common case).
__device__ __forceinline__ void rp_order_at(const RxParams& P, uint32_t i) {
  bool bad = false;
  if (i > 0 && i < P.n) {
    const wg_pkt a = P.desc[i - 1], b = P.desc[i];
    bad = !(a.key_slot < b.key_slot || (a.key_slot == b.key_slot && a.counter < b.counter));
  }
  if (__any(bad) && (threadIdx.x & 63u) == 0) atomicOr(P.unsorted, 1u);
}

// every candidate claims the entry of its (slot, counter): the first claim stores its batch index,
// later claims of the same pair lower it to the smallest index (atomicMin); pos[i] = the entry
__device__ __forceinline__ void rp_insert_at(const RxParams& P, uint32_t i, bool unsorted) {
  if (i >= P.n) return;
  uint32_t slot, pos = ~0u;
  uint64_t c;
  if (unsorted && rp_candidate(P, i, slot, c) && c < kRejectAfter) {
    const uint32_t mask = P.tab_size - 1u;
    uint32_t h = rp_hash(slot, c, P.tab_size);
    for (uint32_t probe = 0; probe < P.tab_size; ++probe, h = (h + 1u) & mask) {
      const uint32_t old = atomicCAS(&P.tab[h], ~0u, i);
      if (old == ~0u) {
        pos = h;
        break;
      }
      const wg_pkt o = P.desc[old];  // an index of the same pair, or of another pair on this entry
      if (o.key_slot == slot && o.counter == c) {
        atomicMin(&P.tab[h], i);
        pos = h;
        break;
      }
    }
  }
  P.pos[i] = pos;
}

__device__ __forceinline__ bool bit_test(const uint64_t* bits, uint32_t W, uint32_t slot, uint64_t c) {
  const uint64_t pos = c % W;
  return (bits[(uint64_t)slot * (W / 64) + pos / 64] >> (pos % 64)) & 1ull;
}

// a candidate passes if it is the lowest index of its (slot, counter) and the window as it stood
// before the batch takes it; newtop[slot] = max(top, passing counter + 1). Every thread of the
// block calls it (block_group).
__device__ __forceinline__ void rp_decide_at(const RxParams& P, uint32_t i, bool unsorted) {
  uint32_t slot = 0;
  uint64_t c = 0;
  const bool cand = i < P.n && rp_candidate(P, i, slot, c);
  bool ok = cand && c < kRejectAfter;
  if (ok && unsorted) ok = P.tab[P.pos[i]] == i;
  if (ok) {
    const uint64_t top = P.top[slot];
    if (c < top) ok = top - c <= P.window && !bit_test(P.bits, P.window, slot, c);
  }
  // newtop has kTopWays copies per slot (block b raises copy b mod kTopWays): a batch of one slot
  // raises one address from every block, and same-address atomics serialise at memory
  const uint32_t way = blockIdx.x % kTopWays;
  block_group<true, false>(ok, slot, c + 1, [&](uint64_t k, uint64_t mx, uint64_t) {
    atomicMax((unsigned long long*)&P.newtop[k * kTopWays + way], (unsigned long long)mx);
  });
  if (cand && !ok) P.status[i] = WG_PKT_REPLAY;
}

// per slot: the window moves to newtop (the largest of its kTopWays copies, read as device-scope
// atomics: in k_rp_judge the last block reads what every block raised); ring positions of the
// counters it passed are cleared and every copy is set to the new top again
__device__ __forceinline__ void rp_advance_to(const RxParams& P, uint32_t slot, uint64_t top, uint64_t nt) {
  const uint32_t W = P.window, words = W / 64;
  uint64_t* b = P.bits + (uint64_t)slot * words;
  if (nt - top >= W) {
    for (uint32_t k = 0; k < words; ++k) b[k] = 0;
  } else {  // ring positions [top mod W, +len), as at most two linear ranges, word by word
    const uint32_t a = (uint32_t)(top % W), len = (uint32_t)(nt - top);
    const uint32_t r0e = min(a + len, W);
    const uint32_t ranges[2][2] = {{a, r0e}, {0u, a + len > W ? a + len - W : 0u}};
    for (int r = 0; r < 2; ++r) {
      for (uint32_t x = ranges[r][0]; x < ranges[r][1];) {
        const uint32_t w = x / 64, lo = x % 64, hi = min(64u, ranges[r][1] - w * 64);
        const uint64_t m = (hi - lo == 64 ? ~0ull : (((1ull << (hi - lo)) - 1ull) << lo));
        b[w] &= ~m;
        x = w * 64 + hi;
      }
    }
  }
  P.top[slot] = nt;
#pragma unroll
  for (uint32_t w = 0; w < kTopWays; ++w) P.newtop[slot * kTopWays + w] = nt;
}
__device__ __forceinline__ void rp_advance_at(const RxParams& P, uint32_t slot) {
  if (slot >= P.key_slots) return;
  const uint64_t top = P.top[slot];
  uint64_t nt = top;
#pragma unroll
  for (uint32_t w = 0; w < kTopWays; ++w) {
    const uint64_t v = __hip_atomic_load(&P.newtop[slot * kTopWays + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nt = v > nt ? v : nt;
  }
  if (nt > top) rp_advance_to(P, slot, top, nt);
}

// accepted counters still inside the advanced window get their ring bit; the table entries this
// batch used are emptied again (nothing reads the table in this phase). Every thread of the block
// calls it (block_group).
__device__ __forceinline__ void rp_mark_at(const RxParams& P, uint32_t i, bool clean = true) {
  uint32_t slot = 0;
  uint64_t c = 0;
  bool act = i < P.n && rp_candidate(P, i, slot, c);  // accepted packets are still OK
  if (act) act = P.top[slot] - c <= P.window;          // top advanced; c < top here
  const uint64_t pos = act ? c % P.window : 0ull;
  const uint64_t word = (uint64_t)slot * (P.window / 64) + pos / 64;
  block_group<false, true>(act, word, 1ull << (pos % 64), [&](uint64_t k, uint64_t, uint64_t orv) {
    atomicOr((unsigned long long*)&P.bits[k], (unsigned long long)orv);
  });
  if (clean && i < P.n && P.pos[i] != ~0u) P.tab[P.pos[i]] = ~0u;
}

// The last block of a launch advances every slot's window (tables of at most kAdvanceInline slots).
__device__ __forceinline__ void rp_advance_all(const RxParams& P) {
  __shared__ uint32_t nfull, full[64];
  if (threadIdx.x == 0) nfull = 0;
  __syncthreads();
  // a slot whose window moves by W or more has every word cleared: by the whole block (a batch of
  // one peer's 64K packets clears 128 words), listed here; every other advance runs per thread
  const uint32_t words = P.window / 64;
  constexpr uint32_t U = 4;  // slots per thread whose loads are in flight together (one latency, not U)
  for (uint32_t base = 0; base < P.key_slots; base += 256u * U) {
    uint64_t tops[U], nts[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t slot = base + threadIdx.x + 256u * u;
      tops[u] = nts[u] = 0;
      if (slot < P.key_slots) {
        tops[u] = nts[u] = P.top[slot];
#pragma unroll
        for (uint32_t w = 0; w < kTopWays; ++w) {
          const uint64_t v =
              __hip_atomic_load(&P.newtop[slot * kTopWays + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          nts[u] = v > nts[u] ? v : nts[u];
        }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
    const uint32_t slot = base + threadIdx.x + 256u * u;
    const uint64_t top = tops[u], nt = nts[u];
    if (slot >= P.key_slots || nt <= top) continue;
    if (nt - top >= P.window && words > 8u) {
      const uint32_t e = atomicAdd(&nfull, 1u);
      if (e < 64u) {
        full[e] = slot;
        P.top[slot] = nt;
#pragma unroll
        for (uint32_t w = 0; w < kTopWays; ++w) P.newtop[slot * kTopWays + w] = nt;
        continue;
      }
    }
    rp_advance_to(P, slot, top, nt);
    }
  }
  __syncthreads();
  const uint32_t nf = min(nfull, 64u);
  for (uint32_t f = 0; f < nf; ++f) {
    uint64_t* b = P.bits + (uint64_t)full[f] * words;
    for (uint32_t k = threadIdx.x; k < words; k += 256u) b[k] = 0;
  }
}

// Counts the calling block done once every atomic it issued has completed; true in the last block
// of the grid (whose device-scope loads then see every block's new tops; no cache flush needed).
// Ordering, per the LLVM AMDGPU memory model for GFX942/GFX950: the blocks exchange data only through
// agent-scope atomics (atomicMax on the new tops, atomicAdd on the counters, relaxed agent-scope
// atomic loads of the new tops), which the hardware performs past the XCD's non-coherent L2. An
// agent-scope release before the counter add is `buffer_wbl2 sc1; s_waitcnt vmcnt(0)`; the write-back
// is for plain stores held in that L2, and this protocol has none, so `s_waitcnt vmcnt(0)` (every
// atomic of this thread acknowledged) + the barrier is the release, and the acquire side needs no L2
// invalidate because the last block reads the new tops with atomic loads. (Round 4 measured the
// agent-scope fences that a grid barrier needs at 156 us per check: DESIGN.md §8.)
// Two levels (kTopWays groups of blocks, then the groups): a counter that every block of a 256-block
// grid raises serialises 256 same-address atomics; each counter sits on its own 64-B line.
__device__ __forceinline__ bool rp_last_block(const RxParams& P) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
    const uint32_t groups = min(gridDim.x, kTopWays), g = blockIdx.x % groups;
    const uint32_t members = (gridDim.x - g + groups - 1u) / groups;  // blocks b < grid with b % groups == g
    uint32_t* gc = P.done_blocks + 16u * (1u + g);
    last = false;
    if (atomicAdd(gc, 1u) == members - 1u) {
      reset_word(gc);  // every member has arrived: ready for the next check (the kernel boundary orders it)
      last = atomicAdd(P.done_blocks, 1u) == groups - 1u;
    }
  }
  __syncthreads();
  return last;
}

// The phases as launches. Default: k_rp_judge (order flag + decisions without the table; its last
// block advances the windows for tables of at most kAdvanceInline slots, else k_rp_advance follows)
// | k_rp_insert (a no-op for a strictly increasing batch) | k_rp_fixmark. WG_RX_LAUNCHES=5 (A/B):
// k_rp_order | k_rp_insert | k_rp_decide | k_rp_advance | k_rp_mark. (Inserting every pair to drop
// the order check made the insert 21 us instead of 3: the table's CAS-with-return round trips cost
// more than a launch.)
__global__ void __launch_bounds__(256) k_rp_order(RxParams P) { rp_order_at(P, blockIdx.x * 256u + threadIdx.x); }
__global__ void __launch_bounds__(256) k_rp_insert(RxParams P) {
  rx_test_skew(P);
  rp_insert_at(P, blockIdx.x * 256u + threadIdx.x, *P.unsorted != 0);
}
__global__ void __launch_bounds__(256) k_rp_decide(RxParams P) {
  rp_decide_at(P, blockIdx.x * 256u + threadIdx.x, *P.unsorted != 0);
}
__global__ void __launch_bounds__(256) k_rp_advance(RxParams P) { rp_advance_at(P, blockIdx.x * 256u + threadIdx.x); }
// The default path's first launch: the order flag, and the decisions as if no (slot, counter) pair
// repeated (a repeated pair's copies all get the same verdict against the old window, and the
// same new top); k_rp_fixmark turns every copy but the lowest into REPLAY when the flag is up.
// With `advance` its last block moves every slot's window.
__global__ void __launch_bounds__(256) k_rp_judge(RxParams P, uint32_t advance) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  rx_test_skew(P);
  rp_order_at(P, i);
  rp_decide_at(P, i, false);
  if (!advance || !rp_last_block(P)) return;
  rp_advance_all(P);
  if (threadIdx.x == 0) reset_word(P.done_blocks);
}
// After k_rp_insert (a no-op for a strictly increasing batch): copies of a pair other than its
// lowest index become REPLAY, then the ring bits of the accepted counters; each used table entry is
// emptied by its lowest index only, after that thread has read it (another copy reading it emptied
// still finds an index other than its own)
__global__ void __launch_bounds__(256) k_rp_fixmark(RxParams P) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  bool own_entry = false;
  rx_test_skew(P);
  if (*P.unsorted && i < P.n && P.pos[i] != ~0u) {
    own_entry = P.tab[P.pos[i]] == i;
    if (!own_entry && P.status[i] == WG_PKT_OK) P.status[i] = WG_PKT_REPLAY;
  }
  rp_mark_at(P, i, false);
  if (own_entry) P.tab[P.pos[i]] = ~0u;
  // the next check's flag, not this one's: every thread of this launch reads this check's flag, and
  // a block that starts after thread 0 has cleared it would skip its fix-ups
#ifdef WG_TEST_HOOKS
  if (i == 0) reset_word(P.mutant ? P.unsorted : P.unsorted_next);
#else
  if (i == 0) reset_word(P.unsorted_next);
#endif
}
__global__ void __launch_bounds__(256) k_rp_mark(RxParams P) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  rp_mark_at(P, i);
  if (i == 0) reset_word(P.unsorted);  // k_rp_decide was its last reader: 0 again for the next batch
}

// keepalive / IP version / AllowedIPs, one thread per packet (wgt::rx_verdict, shared with the
// fused open of wg_open_batch(..., WG_F_RX_FILTER))
__global__ void __launch_bounds__(256) k_rx_filter(RxParams P) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= P.n || P.status[i] != WG_PKT_OK) return;
  const wg_pkt d = P.desc[i];
  if (d.len && (d.out_off >= P.pt_size || P.pt_size - d.out_off < d.len)) {
    P.status[i] = WG_PKT_BADIP;  // not readable here (open would have rejected it already)
    return;
  }
  const wgt::RxTables T{P.slot_filter, P.hdr, P.entries, P.nfilters, P.key_slots};
  P.status[i] = wgt::rx_verdict(T, P.pt + d.out_off, d.len, d.key_slot);
}

}  // namespace wgrx

// ---- C ABI --------------------------------------------------------------------------------
extern "C" {

int wg_filter_set(wg_ctx* c, uint32_t filter_id, const wg_prefix* prefixes, uint32_t n) {
  if (!c || (!prefixes && n)) return fail(WG_EINVAL, "NULL argument");
  if (filter_id >= WG_MAX_FILTERS) return fail(WG_ERANGE, "filter id %u >= %u", filter_id, WG_MAX_FILTERS);
  BinTrie t4, t6;
  for (uint32_t k = 0; k < n; ++k) {
    const wg_prefix& p = prefixes[k];
    if (p.family == 4 && p.prefix_len <= 32) t4.insert(p.addr, p.prefix_len);
    else if (p.family == 6 && p.prefix_len <= 128) t6.insert(p.addr, p.prefix_len);
    else return fail(WG_EINVAL, "prefix %u: family %u / length %u", k, p.family, p.prefix_len);
  }
  std::vector<uint32_t> ent(256, 0u);  // node 0: "none"
  const uint32_t r4 = compile_level(t4, 0, 0, 32, ent);
  const uint32_t r6 = compile_level(t6, 0, 0, 128, ent);
  std::lock_guard<std::mutex> lk(c->mu);
  RxState* r;
  rx_get(c, &r);
  if (r->filt_entries.size() <= filter_id) {
    r->filt_entries.resize(filter_id + 1);
    r->filt_roots.resize(filter_id + 1, {0u, 0u});
  }
  r->filt_entries[filter_id] = std::move(ent);
  r->filt_roots[filter_id] = {r4, r6};
  // device image: every filter's nodes back to back, roots rebased
  std::vector<uint32_t> all, hdr;
  for (size_t f = 0; f < r->filt_entries.size(); ++f) {
    const uint32_t base = (uint32_t)(all.size() / 256);
    const std::vector<uint32_t>& e = r->filt_entries[f];
    if (e.empty()) {
      hdr.push_back(0u);
      hdr.push_back(0u);
      continue;
    }
    for (uint32_t x : e) {
      const uint32_t nx = x & 0x7FFFFFFFu;
      all.push_back((x & 0x80000000u) | (nx ? nx + base : 0u));
    }
    hdr.push_back(r->filt_roots[f].first + base);
    hdr.push_back(r->filt_roots[f].second + base);
  }
  if (all.size() / 256 >= 0x7FFFFFFFu) return fail(WG_E2BIG, "filter tables too large");
  DeviceGuard g(c->device);
  // the tables may be reallocated: no wg_rx_check launched earlier (on any stream) may still read them
  HIPTRY(hipDeviceSynchronize());
  int rc;
  if ((rc = r->d_entries.ensure(all.size() * 4)) != WG_OK || (rc = r->d_hdr.ensure(hdr.size() * 4)) != WG_OK) return rc;
  HIPTRY(hipMemcpyAsync(r->d_entries.p, all.data(), all.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPTRY(hipMemcpyAsync(r->d_hdr.p, hdr.data(), hdr.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPTRY(hipStreamSynchronize(c->stream));
  r->tables_valid = false;  // the tables may have moved
  return WG_OK;
}

int wg_slot_filters_set(wg_ctx* c, uint32_t first_slot, uint32_t n, const uint32_t* filter_ids) {
  if (!c || (!filter_ids && n)) return fail(WG_EINVAL, "NULL argument");
  if ((uint64_t)first_slot + n > c->key_slots) return fail(WG_ERANGE, "key slots out of range");
  std::lock_guard<std::mutex> lk(c->mu);
  RxState* r;
  rx_get(c, &r);
  DeviceGuard g(c->device);
  int rc;
  if (!r->slot_filter_init) HIPTRY(hipDeviceSynchronize());  // first use allocates the table
  if ((rc = r->d_slot_filter.ensure((size_t)c->key_slots * 4)) != WG_OK) return rc;
  if (!r->slot_filter_init) {
    HIPTRY(hipMemsetAsync(r->d_slot_filter.p, 0xFF, (size_t)c->key_slots * 4, c->stream));  // no filter
    r->slot_filter_init = true;
  }
  if (n) HIPTRY(hipMemcpyAsync((uint32_t*)r->d_slot_filter.p + first_slot, filter_ids, (size_t)n * 4,
                               hipMemcpyHostToDevice, c->stream));
  HIPTRY(hipStreamSynchronize(c->stream));
  r->tables_valid = false;
  return WG_OK;
}

int wg_replay_enable(wg_ctx* c, uint32_t window_bits) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (window_bits && (window_bits % 64 || window_bits > 65536))
    return fail(WG_EINVAL, "window_bits must be 0 or a multiple of 64 up to 65536");
  std::lock_guard<std::mutex> lk(c->mu);
  RxState* r;
  rx_get(c, &r);
  DeviceGuard g(c->device);
  HIPTRY(hipDeviceSynchronize());  // window state may be reallocated under earlier wg_rx_check launches
  r->window = window_bits;
  if (!window_bits) return WG_OK;
  int rc;
  if ((rc = r->d_top.ensure((size_t)c->key_slots * 8)) != WG_OK ||
      (rc = r->d_newtop.ensure((size_t)c->key_slots * 8 * kTopWays)) != WG_OK ||
      (rc = r->d_bits.ensure((size_t)c->key_slots * (window_bits / 8))) != WG_OK)
    return rc;
  if ((rc = rx_reset_slots(c, 0, c->key_slots, c->stream)) != WG_OK) return rc;
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_replay_reset(wg_ctx* c, uint32_t first_slot, uint32_t n) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if ((uint64_t)first_slot + n > c->key_slots) return fail(WG_ERANGE, "key slots out of range");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int rc;
  if ((rc = rx_reset_slots(c, first_slot, n, c->stream)) != WG_OK) return rc;
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_replay_state(wg_ctx* c, uint32_t slot, uint64_t* top, uint64_t* bits, uint32_t words) {
  if (!c || !top) return fail(WG_EINVAL, "NULL argument");
  if (slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", slot);
  std::lock_guard<std::mutex> lk(c->mu);
  RxState* r = c->rx;
  if (!r || !r->window) return fail(WG_EINVAL, "replay window not enabled");
  if (bits && words != r->window / 64) return fail(WG_EINVAL, "words must be window_bits / 64");
  DeviceGuard g(c->device);
  int rc;
  if ((rc = rx_after_last_check(r, c->stream)) != WG_OK) return rc;  // the state after every queued check
  HIPTRY(hipMemcpyAsync(top, (uint64_t*)r->d_top.p + slot, 8, hipMemcpyDeviceToHost, c->stream));
  if (bits)
    HIPTRY(hipMemcpyAsync(bits, (uint64_t*)r->d_bits.p + (size_t)slot * words, (size_t)words * 8,
                          hipMemcpyDeviceToHost, c->stream));
  HIPTRY(hipStreamSynchronize(c->stream));
  return WG_OK;
}

int wg_rx_check(wg_ctx* c, const wg_pkt* desc, uint32_t n, const uint8_t* pt, uint64_t pt_size, uint32_t* status,
                uint32_t flags, void* stream) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (flags & ~(WG_RX_FILTER | WG_RX_REPLAY)) return fail(WG_EINVAL, "unknown rx flags 0x%x", flags);
  if (n == 0) return WG_OK;
  if (!desc || !status || (((uintptr_t)desc) & 15u) || (((uintptr_t)status) & 3u))
    return fail(WG_EINVAL, "descriptor / status arrays must be non-NULL and aligned");
  if ((flags & WG_RX_FILTER) && !pt) return fail(WG_EINVAL, "NULL plaintext buffer");
  std::lock_guard<std::mutex> lk(c->mu);
  RxState* r;
  rx_get(c, &r);
  if ((flags & WG_RX_REPLAY) && !r->window) return fail(WG_EINVAL, "WG_RX_REPLAY: call wg_replay_enable first");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard g(c->device);
  wgrx::RxParams P{};
  P.desc = desc;
  P.n = n;
  P.pt = pt;
  P.pt_size = pt ? pt_size : 0;
  P.status = status;
  P.key_slots = c->key_slots;
  const uint32_t grid = (n + 255u) / 256u;
  if (flags & WG_RX_REPLAY) {
    int rc;
    // the scratch (table, positions) is shared by the context's replay checks: a check on
    // another stream first waits for the previous one
    if (!r->ev) HIPTRY(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming));
    if (r->ev_stream != s && r->ev_stream != (hipStream_t)-1) HIPTRY(hipStreamWaitEvent(s, r->ev, 0));
    if (n > (1u << 30)) return fail(WG_EINVAL, "replay check of %u packets: at most 2^30 per batch", n);
    uint32_t T = 1024;
    while (T < 2ull * n) T <<= 1;
    if (T > r->tab_size || (size_t)n * 4 > r->d_pos.cap)
      HIPTRY(hipDeviceSynchronize());  // the scratch is reallocated under earlier checks
    if (T > r->tab_size) {  // (re)allocated, or reset after a failed check: all entries empty
      if ((rc = r->d_tab.ensure((size_t)T * 4)) != WG_OK) return rc;
      if ((rc = r->d_flag.ensure(kFlagBytes)) != WG_OK) return rc;
      HIPTRY(hipMemsetAsync(r->d_tab.p, 0xFF, (size_t)T * 4, s));
      HIPTRY(hipMemsetAsync(r->d_flag.p, 0, kFlagBytes, s));
      r->tab_size = T;
    }
    if ((rc = r->d_pos.ensure((size_t)n * 4)) != WG_OK) return rc;
    P.window = r->window;
    P.top = (uint64_t*)r->d_top.p;
    P.bits = (uint64_t*)r->d_bits.p;
    P.newtop = (uint64_t*)r->d_newtop.p;
    P.tab = (uint32_t*)r->d_tab.p;
    P.tab_size = r->tab_size;
    P.pos = (uint32_t*)r->d_pos.p;
    P.unsorted = (uint32_t*)r->d_flag.p + (r->checks & 1u);
    P.unsorted_next = (uint32_t*)r->d_flag.p + ((r->checks + 1u) & 1u);
    ++r->checks;
    P.done_blocks = (uint32_t*)r->d_flag.p + 16;  // its own line; group counters on the next lines
    P.skew_ticks = r->test_skew_ticks;
    P.mutant = r->test_mutant ? 1u : 0u;
    if (!r->five) {
      const bool inl = c->key_slots <= kAdvanceInline;
      hipLaunchKernelGGL(wgrx::k_rp_judge, dim3(grid), dim3(256), 0, s, P, inl ? 1u : 0u);
      if (!inl)
        hipLaunchKernelGGL(wgrx::k_rp_advance, dim3((c->key_slots + 255u) / 256u), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_insert, dim3(grid), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_fixmark, dim3(grid), dim3(256), 0, s, P);
    } else {
      hipLaunchKernelGGL(wgrx::k_rp_order, dim3(grid), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_insert, dim3(grid), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_decide, dim3(grid), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_advance, dim3((c->key_slots + 255u) / 256u), dim3(256), 0, s, P);
      hipLaunchKernelGGL(wgrx::k_rp_mark, dim3(grid), dim3(256), 0, s, P);
    }
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
      r->tab_size = 0;  // the table / flag may be left dirty: the next check starts from empty ones
      return fail(WG_EDEVICE, "replay kernels: %s", hipGetErrorString(le));
    }
    HIPTRY(hipEventRecord(r->ev, s));
    r->ev_stream = s;
  }
  if (flags & WG_RX_FILTER) {
    P.slot_filter = r->slot_filter_init ? (const uint32_t*)r->d_slot_filter.p : nullptr;
    P.hdr = (const uint32_t*)r->d_hdr.p;
    P.entries = (const uint32_t*)r->d_entries.p;
    P.nfilters = (uint32_t)r->filt_roots.size();
    hipLaunchKernelGGL(wgrx::k_rx_filter, dim3(grid), dim3(256), 0, s, P);
    HIPTRY(hipGetLastError());
  }
  return WG_OK;
}

}  // extern "C"
