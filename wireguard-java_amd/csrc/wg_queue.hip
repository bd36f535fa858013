// wg_queue.hip — asynchronous batch submission, included by wg_capi.hip.
//
// The reference fans every packet out to the ForkJoinPool: a worker calls cipher / decipher
// synchronously and then hands the result to the UDP / tun worker
// (TransportManager.java:41,70-93,137-158; EstablishedSession.java:88-90). A synchronous call per
// packet is bounded by one PCIe round trip (wg_seal1: p50 12 us), so here the producers do not
// wait for the crypto at all:
//   producer (an FJP worker):  wg_submit_seal / wg_submit_open copy the packet into a free slot of a
//       pinned, device-mapped ring and append the slot to its lane's ready ring (per-thread lanes,
//       so producers share no cache line; a lane with no free slot takes one from another lane);
//       they return at once, and block (a futex) only when every slot of the ring is in use;
//   dispatcher (one host thread per queue): pops ready slots into a batch, writes its descriptors
//       into pinned memory and launches k_transport over the ring itself (zero-copy: the kernel
//       reads descriptors and payload and writes the result over PCIe), at most `inflight` batches at a
//       time; when a batch's event has completed it pushes the batch's slots into the completion
//       queue. A batch is launched once min_batch (512) packets wait, or when its first packet has
//       waited 20 us, so batches grow with the load and a light load waits at most 20 us;
//   consumer (the UDP / tun worker): wg_reap takes completions (user tag, status, a pointer to the
//       result in the pinned ring: ct||tag for a seal, the plaintext for an open) and wg_reap_done
//       gives their slots back after it has sent / written them.
// Bit-exactness is that of k_transport (the same kernel as wg_seal_batch / wg_open_batch).
#pragma once

namespace wgq {

// Bounded multi-producer multi-consumer queue of slot ids (Vyukov): a producer preempted inside
// push delays the consumer by the width of one store, not by its packet copy (the copy is done
// before the push).
struct IdQueue {
  struct alignas(16) Cell {
    std::atomic<uint64_t> seq;
    uint32_t v;
  };
  std::unique_ptr<Cell[]> buf;
  uint64_t mask = 0;
  alignas(64) std::atomic<uint64_t> head{0};
  alignas(64) std::atomic<uint64_t> tail{0};

  void init(uint32_t cap) {  // cap: a power of two
    buf.reset(new Cell[cap]);
    mask = cap - 1u;
    for (uint32_t i = 0; i < cap; ++i) buf[i].seq.store(i, std::memory_order_relaxed);
  }
  bool push(uint32_t v) {
    uint64_t pos = tail.load(std::memory_order_relaxed);
    for (;;) {
      Cell& c = buf[pos & mask];
      const uint64_t seq = c.seq.load(std::memory_order_acquire);
      const int64_t dif = (int64_t)seq - (int64_t)pos;
      if (dif == 0) {
        if (tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
          c.v = v;
          c.seq.store(pos + 1, std::memory_order_release);
          return true;
        }
      } else if (dif < 0) {
        return false;  // full
      } else {
        pos = tail.load(std::memory_order_relaxed);
      }
    }
  }
  bool pop(uint32_t* v) {
    uint64_t pos = head.load(std::memory_order_relaxed);
    for (;;) {
      Cell& c = buf[pos & mask];
      const uint64_t seq = c.seq.load(std::memory_order_acquire);
      const int64_t dif = (int64_t)seq - (int64_t)(pos + 1);
      if (dif == 0) {
        if (head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
          *v = c.v;
          c.seq.store(pos + mask + 1, std::memory_order_release);
          return true;
        }
      } else if (dif < 0) {
        return false;  // empty
      } else {
        pos = head.load(std::memory_order_relaxed);
      }
    }
  }
  // Up to max ids at once: one CAS on head for the whole run of ready cells (a consumer popping a
  // burst of completions claims them together instead of one CAS per id). Returns how many.
  uint32_t pop_n(uint32_t* v, uint32_t max) {
    uint64_t pos = head.load(std::memory_order_relaxed);
    for (;;) {
      uint32_t k = 0;
      while (k < max) {
        const uint64_t seq = buf[(pos + k) & mask].seq.load(std::memory_order_acquire);
        if ((int64_t)seq - (int64_t)(pos + k + 1) != 0) break;
        ++k;
      }
      if (k == 0) {
        const uint64_t h = head.load(std::memory_order_relaxed);
        if (h == pos) return 0;  // empty
        pos = h;
        continue;
      }
      if (head.compare_exchange_weak(pos, pos + k, std::memory_order_relaxed)) {
        for (uint32_t i = 0; i < k; ++i) {
          Cell& c = buf[(pos + i) & mask];
          v[i] = c.v;
          c.seq.store(pos + i + mask + 1, std::memory_order_release);
        }
        return k;
      }
    }
  }
  uint64_t size_hint() const {
    const uint64_t t = tail.load(std::memory_order_relaxed), h = head.load(std::memory_order_relaxed);
    return t > h ? t - h : 0;
  }
};

// Producers submit through lanes, so they never share a cache line with each other: a thread takes
// lane (thread number mod lanes) of a queue, and a lane owns the ring slots [lane K, (lane + 1) K)
// (a slot taken by another lane's producer returns to its owner's free ring).
// Its free list (slots the consumers handed back) and its ready list (slots filled and waiting for
// the dispatcher) are single-producer / single-consumer rings; the lane lock is only contended when
// two threads map to one lane, the free lock only among consumer threads.
struct Lane {
  alignas(64) std::atomic<uint32_t> lock{0};  // the lane's producer(s)
  alignas(64) std::atomic<uint64_t> r_tail{0};  // ready ring: pushed under `lock`
  alignas(64) std::atomic<uint64_t> r_head{0};  // popped by the dispatcher alone
  alignas(64) std::atomic<uint32_t> flock{0};   // free ring pushes (consumers)
  std::atomic<uint64_t> f_tail{0};
  alignas(64) std::atomic<uint64_t> f_head{0};  // free ring pops: under `lock`
  // slots this lane's producer took from other lanes (under `lock`): taken kStash at a time, so a
  // producer whose own slots are all in flight scans the other lanes once per kStash packets
  static constexpr uint32_t kStash = 32;
  uint32_t nstash = 0, hint = 0;
  uint32_t stash[kStash];
  std::unique_ptr<uint32_t[]> ready, freel;     // K entries each
};

inline void spin_lock(std::atomic<uint32_t>& l) {
  for (uint32_t k = 0; l.exchange(1, std::memory_order_acquire); ++k)
    if (k > 64) std::this_thread::yield();
    else __builtin_ia32_pause();
}
inline void spin_unlock(std::atomic<uint32_t>& l) { l.store(0, std::memory_order_release); }

inline uint32_t thread_number() {
  static std::atomic<uint32_t> next{0};
  thread_local uint32_t id = next.fetch_add(1, std::memory_order_relaxed);
  return id;
}

struct SlotMeta {  // written by the producer before the slot id is pushed
  uint64_t user;
  uint64_t counter;
  uint64_t t_submit_ns;
  uint32_t len;
  uint32_t key_slot;
  uint32_t status;  // set by the dispatcher when the batch completes
  uint32_t nokey;   // the key slot was zeroed between the submit's check and the copy: never sealed / opened
};

struct Batch {  // one in-flight launch
  wg_pkt* h_desc = nullptr;    // pinned, device-mapped: its descriptors
  wg_pkt* z_desc = nullptr;    // their device alias (the kernel reads them over PCIe)
  uint32_t* h_status = nullptr;  // pinned, device-mapped: open statuses (written by the kernel)
  uint32_t* z_status = nullptr;  // its device alias
  std::vector<uint32_t> slots;   // batch position -> ring slot
  hipEvent_t done = nullptr;
  uint32_t n = 0;
};

// The CPUs of NUMA node `node` (sysfs cpulist "0-63,128-191"); false if unreadable.
inline bool node_cpus(int node, cpu_set_t* set) {
  if (node < 0) return false;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[4096];
  const bool ok = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  if (!ok) return false;
  CPU_ZERO(set);
  int n = 0;
  for (char* p = buf; *p && *p != '\n';) {
    char* e;
    const long a = strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c, ++n) CPU_SET((int)c, set);
    p = *e == ',' ? e + 1 : e;
  }
  return n > 0;
}

inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace wgq

struct wg_queue {
  wg_ctx* c = nullptr;
  int mode = WG_MODE_SEAL;
  uint32_t cap = 0, stride = 0, max_len = 0, max_batch = 0, min_batch = 0, inflight = 0;
  uint64_t window_ns = 0;
  uint8_t* h_in = nullptr;   // pinned ring: slot s at s * stride (plaintext, or ct || tag)
  uint8_t* z_in = nullptr;   // device alias
  uint8_t* h_out = nullptr;  // pinned ring: results (ct || tag, or plaintext)
  uint8_t* z_out = nullptr;
  // pinned, device-mapped: the key of each ring slot, copied from the context's key mirror when the
  // packet is submitted. The kernel reads the key with the packet (its descriptor's key_slot is the
  // ring slot), so wg_keys_zero / wg_keys_set after a submit cannot change what a queued packet is
  // sealed or opened with, exactly as a synchronous cipher() before clean() used the old key.
  uint32_t* h_key = nullptr;
  uint32_t* z_key = nullptr;
  // wg_queue_set_submit_timeout: 0 = a submit waits for a free slot without bound (set from any thread
  // while producers read it)
  std::atomic<uint64_t> submit_timeout_ns{0};
  std::unique_ptr<wgq::SlotMeta[]> meta;
  wgq::IdQueue done_q;                // completions: pushed by the dispatcher, popped by consumers
  uint32_t lanes = 0, per_lane = 0;     // producer lanes and the ring slots each owns
  std::unique_ptr<wgq::Lane[]> lane;
  // producers that found no free slot sleep on `wake_word` until wg_reap_done has handed back
  // wake_batch slots since the last wake (not one wake per freed slot: 16 producers woken for every
  // reap burn the CPU the consumer needs to free slots, and fill the ring one packet at a time)
  alignas(64) std::atomic<uint32_t> wake_word{0};
  std::atomic<uint32_t> free_waiters{0};
  alignas(64) std::atomic<uint32_t> freed_acc{0};
  uint32_t wake_batch = 256;
  bool steal = true;  // a producer whose lane has no free slot takes one from another lane (WG_QUEUE_STEAL=0: no)
  uint32_t prefetch = 2;  // wg_submit_*_n: packets ahead whose bytes are prefetched (WG_QUEUE_PREFETCH)
  std::vector<wgq::Batch> batches;  // `inflight` launch buffers, used round robin
  DevBuf lpt_hist, lpt_order;       // the queue's own longest-first workspace (its own stream)
  hipStream_t stream = nullptr;
  std::thread disp;
  std::atomic<bool> quit{false};
  std::mutex mu;                      // the two condition variables
  std::condition_variable cv_disp, cv_reap;
  std::atomic<int> disp_idle{0}, reapers{0};
  std::atomic<int> err{0};
  std::atomic<uint64_t> n_batches{0}, n_packets{0};
};

namespace {

// One launch per batch: the kernel reads the batch's descriptors straight from pinned memory (no
// copy), one packet per slot (WG_F_UNIFORM is only a scheduling hint: a queue batch is small, so no
// longest-first ordering launches are worth their cost).
// The launch takes the queue's own per-slot key table (OwnKeys): the transport kernel whatever kernel
// the context selects, no plan workspace and no timing events, so the dispatcher needs no c->mu.
int queue_launch(wg_queue* q, wgq::Batch& b, uint32_t lmax) {
  wg_ctx* c = q->c;
  const uint64_t size = (uint64_t)q->cap * q->stride;
  const OwnKeys ok{q->z_key, q->cap};
  int rc;
  if (q->mode == WG_MODE_SEAL)
    rc = launch_transport<WG_MODE_SEAL>(c, b.z_desc, b.n, q->z_in, size, q->z_out, size, nullptr, lmax, WG_F_UNIFORM,
                                        q->stream, nullptr, &q->lpt_hist, &q->lpt_order, false, &ok);
  else
    rc = launch_transport<WG_MODE_OPEN>(c, b.z_desc, b.n, q->z_in, size, q->z_out, size, b.z_status, lmax,
                                        WG_F_UNIFORM, q->stream, nullptr, &q->lpt_hist, &q->lpt_order, false, &ok);
  if (rc != WG_OK) return rc;
  HIPTRY(hipEventRecord(b.done, q->stream));
  return WG_OK;
}

void queue_complete(wg_queue* q, wgq::Batch& b, uint32_t status_override) {
  for (uint32_t j = 0; j < b.n; ++j) {
    const uint32_t s = b.slots[j];
    // the batch's event has completed (or it never ran): no launch reads this slot's key copy any more,
    // so it is wiped now rather than when the queue is freed (SymmetricKeypair.clean zeroes its keys,
    // SymmetricKeypair.java:85-89; the per-packet path wipes its copy after each call the same way)
    memset(q->h_key + 8ull * s, 0, 32);
    q->meta[s].status = q->meta[s].nokey ? (uint32_t)WG_PKT_NOKEY
                        : status_override != 0 ? status_override
                        : q->mode == WG_MODE_OPEN ? b.h_status[j] : (uint32_t)WG_PKT_OK;
    while (!q->done_q.push(s)) std::this_thread::yield();  // cannot stay full: it holds at most cap ids
  }
  q->n_packets.fetch_add(b.n, std::memory_order_relaxed);
  q->n_batches.fetch_add(1, std::memory_order_relaxed);
  b.n = 0;
  if (q->reapers.load(std::memory_order_acquire) > 0) {
    std::lock_guard<std::mutex> lk(q->mu);
    q->cv_reap.notify_all();
  }
}

// Any lane with a submitted packet the dispatcher has not gathered yet (its sleep test).
bool queue_any_ready(wg_queue* q) {
  for (uint32_t l = 0; l < q->lanes; ++l)
    if (q->lane[l].r_tail.load(std::memory_order_acquire) != q->lane[l].r_head.load(std::memory_order_relaxed))
      return true;
  return false;
}

void queue_dispatch(wg_queue* q) {
  DeviceGuard g(q->c->device);
  // short naps below (a few us) must not be stretched to the default 50-us timer slack
  (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
  uint32_t idle = 0;  // loop turns without a completion, a gathered packet or a launch
  uint32_t next = 0, oldest = 0, live = 0;  // batch ring: `live` in flight from `oldest`
  uint32_t rr = 0;                          // lane the next gather starts at
  wgq::Batch* fill = &q->batches[next];
  uint32_t lmax = 0;
  uint64_t first_ns = 0;  // when the batch being filled took its first packet
  while (true) {
    // completions, oldest first
    while (live > 0) {
      wgq::Batch& b = q->batches[oldest];
      const hipError_t e = hipEventQuery(b.done);
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess) {
        q->err.store(WG_EDEVICE);
        fail(WG_EDEVICE, "queue batch: %s", hipGetErrorString(e));
      }
      queue_complete(q, b, e == hipSuccess ? 0u : (uint32_t)WG_PKT_FAILED);
      oldest = (oldest + 1u) % q->inflight;
      --live;
      idle = 0;
    }
    // gather ready packets into the batch being filled
    if (live < q->inflight) {
      uint32_t taken = 0;
      for (uint32_t li = 0; li < q->lanes && fill->n < q->max_batch; ++li) {
        wgq::Lane& ln = q->lane[(rr + li) % q->lanes];
        const uint64_t t = ln.r_tail.load(std::memory_order_acquire);
        uint64_t h = ln.r_head.load(std::memory_order_relaxed);
        for (; h < t && fill->n < q->max_batch; ++h, ++taken) {
          const uint32_t s = ln.ready[h % q->per_lane];
          const wgq::SlotMeta& m = q->meta[s];
          wg_pkt& d = fill->h_desc[fill->n];
          d.in_off = (uint64_t)s * q->stride;
          d.out_off = (uint64_t)s * q->stride;
          d.counter = m.counter;
          d.len = m.nokey ? WG_LEN_INVALID : m.len;  // no key: the kernel skips the packet (out of range)
          d.key_slot = s;  // the key copied into the ring slot at submit time
          if (fill->n == 0) first_ns = wgq::now_ns();
          fill->slots[fill->n++] = s;
          if (!m.nokey) lmax = std::max(lmax, m.len);
        }
        ln.r_head.store(h, std::memory_order_relaxed);
      }
      rr = (rr + 1) % q->lanes;
      if (taken) idle = 0;
      // launch once min_batch packets wait, or when the first of them has waited window_ns (a light
      // load: one packet waits at most that long; a heavy one fills batches of min_batch and more)
      if (fill->n > 0 && (fill->n >= q->min_batch || wgq::now_ns() - first_ns >= q->window_ns)) {
        const int rc = queue_launch(q, *fill, lmax);
        if (rc != WG_OK) {
          q->err.store(rc);
          queue_complete(q, *fill, WG_PKT_FAILED);
        } else {
          ++live;
          next = (next + 1u) % q->inflight;
        }
        fill = &q->batches[next];
        lmax = 0;
        continue;
      }
    }
    if (q->quit.load(std::memory_order_acquire) && live == 0 && fill->n == 0) break;
    if (live > 0 || fill->n > 0) {
      // a batch runs or one is filling: poll the events and the ready lanes; after 32 idle turns in a
      // row nap 4 us between polls (a dispatcher that only yields keeps a core busy for the whole
      // time a batch runs, and on a CPU quota that core is one the producers and consumers lack)
      if (++idle > 32u) std::this_thread::sleep_for(std::chrono::microseconds(4));
      else std::this_thread::yield();
      continue;
    }
    // nothing in flight and nothing ready: sleep until a producer pushes (or 1 ms)
    std::unique_lock<std::mutex> lk(q->mu);
    // Dekker with queue_submit: idle flag, full fence, then the lanes; a producer publishes, fences and
    // then reads the flag, so either this scan sees its packet or it sees the flag and notifies
    q->disp_idle.store(1, std::memory_order_seq_cst);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (!queue_any_ready(q) && !q->quit.load())
      q->cv_disp.wait_for(lk, std::chrono::milliseconds(1));
    q->disp_idle.store(0, std::memory_order_relaxed);
  }
}

void queue_free(wg_queue* q) {
  for (auto& b : q->batches) {
    if (b.h_desc) (void)hipHostFree(b.h_desc);
    if (b.h_status) (void)hipHostFree(b.h_status);
    if (b.done) (void)hipEventDestroy(b.done);
  }
  if (q->h_in) (void)hipHostFree(q->h_in);
  if (q->h_out) (void)hipHostFree(q->h_out);
  if (q->h_key) {
    memset(q->h_key, 0, (size_t)q->cap * 32);  // no session key outlives the queue in pinned memory
    (void)hipHostFree(q->h_key);
  }
  q->lpt_hist.release();
  q->lpt_order.release();
  if (q->stream) (void)hipStreamDestroy(q->stream);
}

// A free slot for a producer of lane `own` (its lock held): its own free ring first, then any other
// lane's (try-lock only, so two producers taking from each other's lanes cannot deadlock). One
// producer thread can so use the whole ring, not only its lane's share of it.
bool queue_take_slot(wg_queue* q, wgq::Lane& own, uint32_t* s) {
  uint64_t fh = own.f_head.load(std::memory_order_relaxed);
  if (fh != own.f_tail.load(std::memory_order_acquire)) {
    *s = own.freel[fh % q->per_lane];
    own.f_head.store(fh + 1, std::memory_order_relaxed);
    return true;
  }
  if (own.nstash) {
    *s = own.stash[--own.nstash];
    return true;
  }
  if (!q->steal) return false;
  const uint32_t me = (uint32_t)(&own - q->lane.get());
  for (uint32_t k = 0; k < q->lanes; ++k) {
    const uint32_t v = (own.hint + k) % q->lanes;
    if (v == me) continue;
    wgq::Lane& o = q->lane[v];
    fh = o.f_head.load(std::memory_order_relaxed);
    if (fh == o.f_tail.load(std::memory_order_acquire)) continue;  // (a hint: checked again under the lock)
    if (o.lock.exchange(1, std::memory_order_acquire)) continue;
    fh = o.f_head.load(std::memory_order_relaxed);
    const uint64_t avail = o.f_tail.load(std::memory_order_acquire) - fh;
    // half of what the victim has free (its own producer keeps the rest), at most a stash
    const uint32_t take = (uint32_t)std::min<uint64_t>(wgq::Lane::kStash + 1u, (avail + 1u) / 2u);
    for (uint32_t t = 0; t < take; ++t) {
      const uint32_t x = o.freel[(fh + t) % q->per_lane];
      if (t == 0) *s = x;
      else own.stash[own.nstash++] = x;
    }
    o.f_head.store(fh + take, std::memory_order_relaxed);
    wgq::spin_unlock(o.lock);
    if (take) {
      own.hint = v;
      return true;
    }
  }
  return false;
}

// queue_take_slot with the lane lock taken.
// Returns 1 (the lock stays held: the caller publishes), 0 (no free slot in any lane) or 2 (this
// lane's ready ring is full: it holds at most per_lane slots, which slots taken from other lanes
// could otherwise overflow; the dispatcher empties it within its next gather).
int queue_try_slot(wg_queue* q, wgq::Lane& ln, uint32_t* s) {
  wgq::spin_lock(ln.lock);
  int r = 2;
  if (ln.r_tail.load(std::memory_order_relaxed) - ln.r_head.load(std::memory_order_acquire) < q->per_lane)
    r = queue_take_slot(q, ln, s) ? 1 : 0;
  if (r != 1) wgq::spin_unlock(ln.lock);
  return r;
}

// A free slot for lane `ln`, its lock held on return (WG_OK), waiting as the queue's submit policy says:
// WG_EAGAIN once none was free for the submit timeout (*deadline: 0 before the first wait).
int queue_acquire(wg_queue* q, wgq::Lane& ln, uint32_t* s, uint64_t* deadline) {
  for (uint32_t round = 0;; ++round) {
    const uint32_t w = q->wake_word.load(std::memory_order_acquire);
    const int r = queue_try_slot(q, ln, s);
    if (r == 1) return WG_OK;
    if (const uint64_t tmo = q->submit_timeout_ns.load(std::memory_order_relaxed)) {
      const uint64_t now = wgq::now_ns();
      if (!*deadline) *deadline = now + tmo;
      else if (now >= *deadline)
        return fail(WG_EAGAIN, "no free queue slot for %llu us (is the consumer calling wg_reap_done?)",
                    (unsigned long long)(tmo / 1000u));
    }
    // this lane's ready ring is full (the dispatcher is about to gather it), or every slot is in use:
    // wait for wg_reap_done without burning the CPU the consumers need to free them
    if (round < 2 || r == 2) {
      if (round < 64) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
      continue;
    }
    q->free_waiters.fetch_add(1, std::memory_order_seq_cst);
    if (queue_try_slot(q, ln, s) == 1) {  // freed before this thread counted as a waiter
      q->free_waiters.fetch_sub(1, std::memory_order_relaxed);
      return WG_OK;
    }
    const struct timespec ts = {0, 1000000};  // 1 ms: the last slots of a burst wake nobody
    futex(&q->wake_word, FUTEX_WAIT_PRIVATE, w, &ts);
    q->free_waiters.fetch_sub(1, std::memory_order_relaxed);
  }
}

// Fill slot s with one packet: its key as the key slot holds it now, its meta, its bytes. A key slot
// zeroed since queue_check_packet (a clean() racing the submit) marks the packet: it completes with
// WG_PKT_NOKEY and is never sealed or opened under the zero key.
void queue_fill(wg_queue* q, uint32_t s, uint32_t key_slot, uint64_t counter, const uint8_t* src, uint32_t len,
                uint64_t user) {
  wgq::SlotMeta& m = q->meta[s];
  m.nokey = key_snapshot(q->c, key_slot, q->h_key + 8ull * s) ? 0u : 1u;
  m.user = user;
  m.counter = counter;
  m.len = len;
  m.key_slot = key_slot;
  m.t_submit_ns = wgq::now_ns();
  const size_t n = (size_t)len + (q->mode == WG_MODE_OPEN ? 16u : 0u);
  if (n) memcpy(q->h_in + (size_t)s * q->stride, src, n);
}

// Publish the lane's ready entries up to rt (its lock held; released here) and wake the dispatcher
// if it sleeps.
void queue_publish(wg_queue* q, wgq::Lane& ln, uint64_t rt) {
  ln.r_tail.store(rt, std::memory_order_release);  // after the slots' bytes and meta
  wgq::spin_unlock(ln.lock);
  // (no shared per-packet counter: 16 producers incrementing one cache line per packet serialised on it)
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (q->disp_idle.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(q->mu);
    q->cv_disp.notify_one();
  }
}

int queue_check(wg_queue* q, int mode) {
  if (!q) return fail(WG_EINVAL, "NULL queue");
  if (q->mode != mode) return fail(WG_EINVAL, "a %s queue", q->mode == WG_MODE_SEAL ? "seal" : "open");
  if (const int e = q->err.load(std::memory_order_relaxed)) return fail(e, "queue failed earlier");
  return WG_OK;
}

int queue_check_packet(wg_queue* q, int mode, uint32_t key_slot, const uint8_t* src, uint32_t len) {
  if (!src && (len || mode == WG_MODE_OPEN)) return fail(WG_EINVAL, "NULL argument");
  if (len > q->max_len) return fail(WG_E2BIG, "packet of %u bytes > the queue's max_len %u", len, q->max_len);
  if (key_slot >= q->c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  if (!key_is_live(q->c, key_slot)) return fail(WG_ENOKEY, "key slot %u holds no key (zeroed or never set)", key_slot);
  return WG_OK;
}

int queue_submit(wg_queue* q, int mode, uint32_t key_slot, uint64_t counter, const uint8_t* src, uint32_t len,
                 uint64_t user) {
  int rc;
  if ((rc = queue_check(q, mode)) != WG_OK || (rc = queue_check_packet(q, mode, key_slot, src, len)) != WG_OK)
    return rc;
  wgq::Lane& ln = q->lane[wgq::thread_number() % q->lanes];
  uint32_t s = 0;
  uint64_t deadline = 0;  // wg_queue_set_submit_timeout: WG_EAGAIN once no slot was free for that long
  if ((rc = queue_acquire(q, ln, &s, &deadline)) != WG_OK) return rc;
  queue_fill(q, s, key_slot, counter, src, len, user);
  const uint64_t rt = ln.r_tail.load(std::memory_order_relaxed);
  ln.ready[rt % q->per_lane] = s;
  queue_publish(q, ln, rt + 1);
  return WG_OK;
}

// n packets in one call: one lane lock, one publication and one dispatcher check per run of free
// slots instead of per packet (the forwarder of tools/queue_bench spends its time in exactly that
// per-packet overhead on small packets). Returns how many were queued, in order: n, or fewer when
// the submit timeout ran out (none: WG_EAGAIN). A bad entry fails the call before anything is queued.
int queue_submit_n(wg_queue* q, int mode, const wg_submit* p, uint32_t n) {
  int rc;
  if ((rc = queue_check(q, mode)) != WG_OK) return rc;
  if (!p && n) return fail(WG_EINVAL, "NULL argument");
  if (n > (uint32_t)INT32_MAX) return fail(WG_EINVAL, "%u packets", n);
  for (uint32_t k = 0; k < n; ++k)
    if ((rc = queue_check_packet(q, mode, p[k].key_slot, p[k].data, p[k].len)) != WG_OK) return rc;
  wgq::Lane& ln = q->lane[wgq::thread_number() % q->lanes];
  uint64_t deadline = 0;
  uint32_t k = 0;
  while (k < n) {
    uint32_t s = 0;
    if ((rc = queue_acquire(q, ln, &s, &deadline)) != WG_OK) return k ? (int)k : rc;
    uint64_t rt = ln.r_tail.load(std::memory_order_relaxed);
    const uint64_t rh = ln.r_head.load(std::memory_order_acquire);
    for (;;) {
      // the bytes of a packet a few ahead: a forwarder's source is usually a completion in another queue's
      // ring, written by the GPU and so not in this core's caches; its first lines' misses overlap this copy
      if (k + q->prefetch < n && q->prefetch) {
        const uint8_t* a = p[k + q->prefetch].data;
        const uint32_t nb = p[k + q->prefetch].len + (mode == WG_MODE_OPEN ? 16u : 0u);
        for (uint32_t o = 0; o < nb; o += 64u) __builtin_prefetch(a + o, 0, 0);
      }
      queue_fill(q, s, p[k].key_slot, p[k].counter, p[k].data, p[k].len, p[k].user);
      ln.ready[rt % q->per_lane] = s;
      ++rt;
      ++k;
      // the lane's ready ring holds at most per_lane entries (queue_try_slot's bound)
      if (k == n || rt - rh >= q->per_lane || !queue_take_slot(q, ln, &s)) break;
    }
    queue_publish(q, ln, rt);
    deadline = 0;  // the timeout bounds each wait for a free slot, as for single submits
  }
  return (int)n;
}

uint32_t pow2_at_least(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace

extern "C" {

int wg_device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) return -1;
  for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

int wg_queue_create(wg_ctx* c, int mode, uint32_t capacity, uint32_t max_len, uint32_t max_batch, wg_queue** out) {
  if (!c || !out) return fail(WG_EINVAL, "NULL argument");
  *out = nullptr;
  if (mode != WG_MODE_SEAL && mode != WG_MODE_OPEN) return fail(WG_EINVAL, "mode must be WG_MODE_SEAL or WG_MODE_OPEN");
  if (max_len > WG_QUEUE_MAX_LEN) return fail(WG_E2BIG, "max_len %u > %u", max_len, WG_QUEUE_MAX_LEN);
  if (capacity == 0) capacity = 65536;
  if (capacity > (1u << 22)) return fail(WG_EINVAL, "capacity %u > 2^22", capacity);
  if (max_len == 0) max_len = 2032;  // the reference pipeline's incoming limit (4-KB buffers)
  DeviceGuard g(c->device);
  std::unique_ptr<wg_queue> q(new wg_queue());
  q->c = c;
  q->mode = mode;
  q->cap = pow2_at_least(capacity);
  q->stride = ((max_len + 16u) + 63u) & ~63u;  // 64-B aligned slots: every payload read / store is 16-B aligned
  q->max_len = max_len;
  q->max_batch = std::min<uint32_t>(max_batch ? max_batch : 8192u, q->cap);
  // up to `inflight` batches run at once; while one runs, the next is launched once min_batch
  // packets wait (WG_QUEUE_INFLIGHT / WG_QUEUE_MIN_BATCH override both for A/B runs)
  q->inflight = 4;
  q->min_batch = 512;
  q->window_ns = 20000;
  if (const char* e = getenv("WG_QUEUE_INFLIGHT")) q->inflight = std::max(1, std::min(16, atoi(e)));
  if (const char* e = getenv("WG_QUEUE_MIN_BATCH")) q->min_batch = (uint32_t)std::max(1, atoi(e));
  if (const char* e = getenv("WG_QUEUE_WINDOW_US")) q->window_ns = 1000ull * (uint64_t)std::max(0, atoi(e));
  if (const char* e = getenv("WG_QUEUE_STEAL")) q->steal = atoi(e) != 0;
  if (const char* e = getenv("WG_QUEUE_PREFETCH")) q->prefetch = (uint32_t)std::max(0, std::min(8, atoi(e)));
  q->min_batch = std::min(q->min_batch, q->max_batch);
  q->wake_batch = std::max(1u, std::min(256u, q->cap / 8u));
  q->meta.reset(new wgq::SlotMeta[q->cap]());
  q->done_q.init(q->cap);
  q->lanes = std::min<uint32_t>(64u, std::max<uint32_t>(1u, q->cap / 64u));
  q->per_lane = q->cap / q->lanes;
  q->lane.reset(new wgq::Lane[q->lanes]);
  for (uint32_t l = 0; l < q->lanes; ++l) {
    wgq::Lane& ln = q->lane[l];
    ln.ready.reset(new uint32_t[q->per_lane]);
    ln.freel.reset(new uint32_t[q->per_lane]);
    for (uint32_t k = 0; k < q->per_lane; ++k) ln.freel[k] = l * q->per_lane + k;
    ln.f_tail.store(q->per_lane);
  }
  const size_t ring = (size_t)q->cap * q->stride;
  bool ok = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking) == hipSuccess &&
            hipHostMalloc((void**)&q->h_in, ring, hipHostMallocMapped | hipHostMallocPortable) == hipSuccess &&
            hipHostMalloc((void**)&q->h_out, ring, hipHostMallocMapped | hipHostMallocPortable) == hipSuccess &&
            hipHostMalloc((void**)&q->h_key, (size_t)q->cap * 32, hipHostMallocMapped | hipHostMallocPortable) ==
                hipSuccess;
  if (ok) {
    q->z_in = mapped_alias(q->h_in);
    q->z_out = mapped_alias(q->h_out);
    q->z_key = (uint32_t*)mapped_alias(q->h_key);
    ok = q->z_in && q->z_out && q->z_key;
  }
  q->batches.resize(q->inflight);
  for (auto& b : q->batches) {
    if (!ok) break;
    b.slots.resize(q->max_batch);
    ok = hipHostMalloc((void**)&b.h_desc, sizeof(wg_pkt) * q->max_batch, hipHostMallocMapped | hipHostMallocPortable) ==
             hipSuccess &&
         hipHostMalloc((void**)&b.h_status, sizeof(uint32_t) * q->max_batch,
                       hipHostMallocMapped | hipHostMallocPortable) == hipSuccess &&
         hipEventCreateWithFlags(&b.done, hipEventDisableTiming) == hipSuccess;
    if (ok) {
      b.z_status = (uint32_t*)mapped_alias(b.h_status);
      b.z_desc = (wg_pkt*)mapped_alias(b.h_desc);
      ok = b.z_status != nullptr && b.z_desc != nullptr;
    }
  }
  if (!ok) {
    queue_free(q.get());
    return fail(WG_ENOMEM, "queue: pinned rings (2 x %zu B) or device buffers could not be allocated", ring);
  }
  wg_queue* qp = q.release();
  qp->disp = std::thread(queue_dispatch, qp);
  // the dispatcher on the device's NUMA node (WG_QUEUE_PIN=0: wherever the scheduler puts it): on
  // a two-socket host the far socket halved the harness's rate in some runs
  const char* pin = getenv("WG_QUEUE_PIN");
  cpu_set_t set;
  if ((!pin || atoi(pin) != 0) && wgq::node_cpus(wg_device_numa_node(c->device), &set))
    (void)pthread_setaffinity_np(qp->disp.native_handle(), sizeof set, &set);
  *out = qp;
  return WG_OK;
}

int wg_queue_destroy(wg_queue* q) {
  if (!q) return WG_OK;
  q->quit.store(true, std::memory_order_release);
  {
    std::lock_guard<std::mutex> lk(q->mu);
    q->cv_disp.notify_all();
  }
  if (q->disp.joinable()) q->disp.join();  // the dispatcher leaves once nothing is in flight
  DeviceGuard g(q->c->device);
  (void)hipStreamSynchronize(q->stream);
  queue_free(q);
  delete q;
  return WG_OK;
}

int wg_submit_seal(wg_queue* q, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint64_t user) {
  return queue_submit(q, WG_MODE_SEAL, key_slot, counter, pt, len, user);
}

int wg_submit_open(wg_queue* q, uint32_t key_slot, uint64_t counter, const uint8_t* ct_tag, uint32_t len,
                   uint64_t user) {
  return queue_submit(q, WG_MODE_OPEN, key_slot, counter, ct_tag, len, user);
}

int wg_submit_seal_n(wg_queue* q, const wg_submit* p, uint32_t n) { return queue_submit_n(q, WG_MODE_SEAL, p, n); }

int wg_submit_open_n(wg_queue* q, const wg_submit* p, uint32_t n) { return queue_submit_n(q, WG_MODE_OPEN, p, n); }

int wg_reap(wg_queue* q, wg_completion* out, uint32_t max, uint32_t timeout_us) {
  if (!q || (!out && max)) return fail(WG_EINVAL, "NULL argument");
  uint32_t n = 0, s;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
  while (true) {
    uint32_t ids[256];
    uint32_t got;
    while (n < max && (got = q->done_q.pop_n(ids, std::min<uint32_t>(256u, max - n))) > 0) {
     for (uint32_t k = 0; k < got; ++k) {
      s = ids[k];
      const wgq::SlotMeta& m = q->meta[s];
      wg_completion& o = out[n++];
      o.user = m.user;
      o.counter = m.counter;
      o.data = q->h_out + (size_t)s * q->stride;
      o.len = m.len;
      o.status = m.status;
      o.key_slot = m.key_slot;
      o.slot = s;
      o.submit_ns = m.t_submit_ns;
     }
    }
    if (n > 0 || timeout_us == 0 || max == 0) return (int)n;
    if (const int e = q->err.load(std::memory_order_relaxed)) return fail(e, "queue failed");
    if (std::chrono::steady_clock::now() >= deadline) return 0;
    std::unique_lock<std::mutex> lk(q->mu);
    q->reapers.fetch_add(1, std::memory_order_seq_cst);
    if (q->done_q.size_hint() == 0) q->cv_reap.wait_until(lk, std::min(deadline, std::chrono::steady_clock::now() +
                                                                                     std::chrono::microseconds(200)));
    q->reapers.fetch_sub(1, std::memory_order_relaxed);
  }
}

int wg_reap_done(wg_queue* q, const wg_completion* done, uint32_t n) {
  if (!q || (!done && n)) return fail(WG_EINVAL, "NULL argument");
  for (uint32_t i = 0; i < n; ++i)
    if (done[i].slot >= q->cap) return fail(WG_EINVAL, "completion %u: slot %u", i, done[i].slot);
  // grouped by home lane: one lock and one tail store per lane and chunk, not per slot (the free
  // ring's tail shares a cache line with the lane's producer, which reads it for every packet)
  constexpr uint32_t kChunk = 512;
  uint32_t cnt[64], at[64], tmp[kChunk];
  for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
    const uint32_t m = std::min(kChunk, n - c0);
    for (uint32_t l = 0; l < q->lanes; ++l) cnt[l] = 0;
    for (uint32_t i = 0; i < m; ++i) ++cnt[done[c0 + i].slot / q->per_lane];
    uint32_t acc = 0;
    for (uint32_t l = 0; l < q->lanes; ++l) {
      at[l] = acc;
      acc += cnt[l];
    }
    for (uint32_t i = 0; i < m; ++i) {
      const uint32_t sl = done[c0 + i].slot;
      tmp[at[sl / q->per_lane]++] = sl;
    }
    uint32_t k = 0;
    for (uint32_t l = 0; l < q->lanes; ++l) {
      if (!cnt[l]) continue;
      wgq::Lane& ln = q->lane[l];
      wgq::spin_lock(ln.flock);
      const uint64_t ft = ln.f_tail.load(std::memory_order_relaxed);
      for (uint32_t j = 0; j < cnt[l]; ++j) ln.freel[(ft + j) % q->per_lane] = tmp[k + j];
      ln.f_tail.store(ft + cnt[l], std::memory_order_release);
      wgq::spin_unlock(ln.flock);
      k += cnt[l];
    }
  }
  if (n && q->freed_acc.fetch_add(n, std::memory_order_seq_cst) + n >= q->wake_batch &&
      q->free_waiters.load(std::memory_order_seq_cst) > 0) {
    q->freed_acc.store(0, std::memory_order_relaxed);
    q->wake_word.fetch_add(1, std::memory_order_release);
    futex(&q->wake_word, FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr);
  }
  return WG_OK;
}

int wg_queue_set_submit_timeout(wg_queue* q, uint32_t timeout_us) {
  if (!q) return fail(WG_EINVAL, "NULL queue");
  q->submit_timeout_ns.store(1000ull * timeout_us, std::memory_order_relaxed);
  return WG_OK;
}

uint32_t wg_queue_key_residue(const wg_queue* q) {
  if (!q) return 0;
  uint32_t n = 0;
  for (uint32_t s = 0; s < q->cap; ++s) {
    uint32_t any = 0;
    for (uint32_t k = 0; k < 8u; ++k) any |= ((const volatile uint32_t*)q->h_key)[8ull * s + k];
    n += any ? 1u : 0u;
  }
  return n;
}

int wg_queue_stats(wg_queue* q, uint64_t* batches, uint64_t* packets) {
  if (!q) return fail(WG_EINVAL, "NULL queue");
  if (batches) *batches = q->n_batches.load();
  if (packets) *packets = q->n_packets.load();
  return WG_OK;
}

}  // extern "C"
