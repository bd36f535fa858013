// wg_batcher.hip — the per-packet entry points wg_seal1 / wg_open1 as batched device
// launches (included by wg_capi.hip).
//
// The reference fans every packet out to the ForkJoinPool and seals / opens it with one
// synchronous call per packet (TransportManager.java:41,79,152-158 ->
// SymmetricKeypair.java:63-83). Those calls stay per-packet and synchronous here, but
// they no longer each cost a device round trip: a caller copies its packet into the
// open batch (pinned, device-mapped host memory), a library-owned launcher thread
// launches k_transport over everything that has accumulated (seal and open entries as
// two launches on one stream; the kernel reads and writes the pinned batch directly,
// zero-copy), and the callers wake when their batch completes. While one batch runs on
// the device the next one fills, so the batch size follows the offered load: one packet
// when a single thread calls, hundreds when many threads do (no fixed window unless
// wg_batcher_config sets one). Callers never hold the context lock.
#pragma once

namespace {

constexpr int kBatchBufs = 3;
constexpr uint32_t kBatchPktsDefault = 8192;
constexpr uint64_t kBatchArena = 16ull << 20;  // bytes per direction per batch buffer

struct BatchBuf {
  enum State { FREE, OPEN, SUBMITTED, DONE };
  // pinned, device-mapped host memory; d_* are the device aliases
  wg_pkt* sdesc = nullptr;
  wg_pkt* odesc = nullptr;
  uint8_t* in = nullptr;
  uint8_t* out = nullptr;
  uint32_t* status = nullptr;
  wg_pkt* d_sdesc = nullptr;
  wg_pkt* d_odesc = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_out = nullptr;
  uint32_t* d_status = nullptr;
  // guarded by Batcher::mu
  State state = FREE;
  uint64_t gen = 0;
  uint32_t nseal = 0, nopen = 0, seal_max = 0, open_max = 0;
  uint64_t in_used = 0, out_used = 0;
  uint32_t writers = 0;  // reserved entries still being filled by their callers
  uint32_t users = 0;    // entries whose callers have not yet read their result
  std::chrono::steady_clock::time_point first;
  std::atomic<uint64_t> done_gen{0};  // gen of the last completed launch from this buffer
  std::condition_variable cv_done;    // this buffer's callers: their batch completed
};

struct Batcher {
  wg_ctx* c = nullptr;
  std::mutex mu;
  std::condition_variable cv_work;  // launcher: entries arrived / writers done / stop
  std::condition_variable cv_free;  // callers: room in a fresh open batch
  BatchBuf buf[kBatchBufs];
  int open_idx = 0;
  uint64_t next_gen = 1;
  uint32_t max_pkts = kBatchPktsDefault;
  uint32_t window_us = 0;
  bool stop = false;
  int launch_error = WG_OK;
  std::string launch_msg;
  uint64_t launches = 0, packets = 0;
  hipStream_t stream = nullptr;   // seal launches
  hipStream_t stream2 = nullptr;  // open launches
  std::thread th;
};

uint64_t align16(uint64_t x) { return (x + 15u) & ~15ull; }

void batcher_free_mem(Batcher* B) {
  for (BatchBuf& b : B->buf)
    for (void* p : {(void*)b.sdesc, (void*)b.odesc, (void*)b.in, (void*)b.out, (void*)b.status})
      if (p) (void)hipHostFree(p);
  if (B->stream) (void)hipStreamDestroy(B->stream);
  if (B->stream2) (void)hipStreamDestroy(B->stream2);
}

int batcher_launch(Batcher* B, BatchBuf& b) {
  wg_ctx* c = B->c;
  std::lock_guard<std::mutex> lk(c->mu);
  int rc = WG_OK;
  // seal and open entries are independent: two launches on two streams run side by side
  // (a small batch's launch is latency-bound, so this halves the batch round trip)
  if (b.nseal)
    rc = launch_transport<WG_MODE_SEAL>(c, b.d_sdesc, b.nseal, b.d_in, kBatchArena, b.d_out, kBatchArena, nullptr,
                                       b.seal_max, 0, B->stream);
  if (rc == WG_OK && b.nopen)
    rc = launch_transport<WG_MODE_OPEN>(c, b.d_odesc, b.nopen, b.d_in, kBatchArena, b.d_out, kBatchArena,
                                       b.d_status, b.open_max, 0, B->stream2);
  // wait by polling: a blocking synchronize sleeps on an interrupt and adds tens of µs to
  // every batch round trip; the launcher thread spins while its batch is on the device
  const bool used[2] = {b.nseal > 0, b.nopen > 0};
  const hipStream_t st[2] = {B->stream, B->stream2};
  for (int k = 0; k < 2; ++k) {
    if (!used[k]) continue;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    while ((e = hipStreamQuery(st[k])) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
        e = hipStreamSynchronize(st[k]);  // long batch: stop spinning
        break;
      }
    }
    if (e != hipSuccess && rc == WG_OK) rc = fail(WG_EDEVICE, "batch sync: %s", hipGetErrorString(e));
  }
  return rc;
}

void batcher_loop(Batcher* B) {
  (void)hipSetDevice(B->c->device);
  std::unique_lock<std::mutex> lk(B->mu);
  for (;;) {
    BatchBuf* b = &B->buf[B->open_idx];
    B->cv_work.wait(lk, [&] { return B->stop || b->nseal + b->nopen > 0; });
    if (B->stop && b->nseal + b->nopen == 0) break;
    if (B->window_us && b->nseal + b->nopen < B->max_pkts && !B->stop) {  // optional accumulation window
      const auto until = b->first + std::chrono::microseconds(B->window_us);
      B->cv_work.wait_until(lk, until, [&] { return B->stop || b->nseal + b->nopen >= B->max_pkts; });
    }
    // hand callers a fresh open batch, then launch this one once its writers are done
    int nxt = -1;
    B->cv_free.wait(lk, [&] {
      for (int k = 1; k < kBatchBufs; ++k) {
        const int i = (B->open_idx + k) % kBatchBufs;
        if (B->buf[i].state == BatchBuf::FREE) { nxt = i; return true; }
      }
      return false;
    });
    b->state = BatchBuf::SUBMITTED;
    BatchBuf& f = B->buf[nxt];
    f.state = BatchBuf::OPEN;
    f.gen = B->next_gen++;
    f.nseal = f.nopen = f.seal_max = f.open_max = 0;
    f.in_used = f.out_used = 0;
    f.writers = f.users = 0;
    B->open_idx = nxt;
    B->cv_free.notify_all();
    B->cv_work.wait(lk, [&] { return b->writers == 0; });
    lk.unlock();
    const int rc = batcher_launch(B, *b);
    lk.lock();
    if (rc != WG_OK) {
      B->launch_error = rc;
      B->launch_msg = g_err;
    }
    B->launches += 1;
    B->packets += b->nseal + b->nopen;
    b->state = b->users ? BatchBuf::DONE : BatchBuf::FREE;
    b->done_gen.store(b->gen, std::memory_order_release);
    b->cv_done.notify_all();
    B->cv_free.notify_all();
  }
}

int batcher_get(wg_ctx* c, Batcher** out) {
  std::lock_guard<std::mutex> lk(c->batcher_mu);
  if (c->batcher) {
    *out = c->batcher;
    return WG_OK;
  }
  DeviceGuard g(c->device);
  Batcher* B = new Batcher();
  B->c = c;
  bool ok = hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&B->stream2, hipStreamNonBlocking) == hipSuccess;
  const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
  for (BatchBuf& b : B->buf) {
    if (!ok) break;
    ok = hipHostMalloc((void**)&b.sdesc, sizeof(wg_pkt) * kBatchPktsDefault, fl) == hipSuccess &&
         hipHostMalloc((void**)&b.odesc, sizeof(wg_pkt) * kBatchPktsDefault, fl) == hipSuccess &&
         hipHostMalloc((void**)&b.in, kBatchArena, fl) == hipSuccess &&
         hipHostMalloc((void**)&b.out, kBatchArena, fl) == hipSuccess &&
         hipHostMalloc((void**)&b.status, sizeof(uint32_t) * kBatchPktsDefault, fl) == hipSuccess &&
         hipHostGetDevicePointer((void**)&b.d_sdesc, b.sdesc, 0) == hipSuccess &&
         hipHostGetDevicePointer((void**)&b.d_odesc, b.odesc, 0) == hipSuccess &&
         hipHostGetDevicePointer((void**)&b.d_in, b.in, 0) == hipSuccess &&
         hipHostGetDevicePointer((void**)&b.d_out, b.out, 0) == hipSuccess &&
         hipHostGetDevicePointer((void**)&b.d_status, b.status, 0) == hipSuccess;
  }
  if (!ok) {
    batcher_free_mem(B);
    delete B;
    return fail(WG_ENOMEM, "batcher: pinned batch buffers could not be allocated");
  }
  B->buf[0].state = BatchBuf::OPEN;
  B->buf[0].gen = B->next_gen++;
  B->th = std::thread(batcher_loop, B);
  c->batcher = B;
  *out = B;
  return WG_OK;
}

void batcher_stop(wg_ctx* c) {
  Batcher* B = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->batcher_mu);
    B = c->batcher;
    c->batcher = nullptr;
  }
  if (!B) return;
  {
    std::lock_guard<std::mutex> lk(B->mu);
    B->stop = true;
  }
  B->cv_work.notify_all();
  B->cv_free.notify_all();
  if (B->th.joinable()) B->th.join();
  batcher_free_mem(B);
  delete B;
}

// One packet through the batcher. open: src = ct || tag (len + 16 bytes), dst gets len
// bytes only if the tag verifies (returns 1 otherwise, dst untouched).
int batcher_submit(wg_ctx* c, bool open, uint32_t key_slot, uint64_t counter, const uint8_t* src, uint32_t len,
                   uint8_t* dst) {
  Batcher* B;
  int rc;
  if ((rc = batcher_get(c, &B)) != WG_OK) return rc;
  const uint64_t in_need = align16((uint64_t)len + (open ? 16u : 0u));
  const uint64_t out_need = align16((uint64_t)len + (open ? 0u : 16u));
  std::unique_lock<std::mutex> lk(B->mu);
  BatchBuf* b;
  for (;;) {
    if (B->stop) return fail(WG_EINVAL, "context is being destroyed");
    b = &B->buf[B->open_idx];
    if (b->state == BatchBuf::OPEN && b->nseal + b->nopen < B->max_pkts &&
        (open ? b->nopen : b->nseal) < kBatchPktsDefault && b->in_used + in_need <= kBatchArena &&
        b->out_used + out_need <= kBatchArena)
      break;
    B->cv_work.notify_one();  // full: the launcher takes it and opens a fresh one
    B->cv_free.wait(lk);
  }
  if (b->nseal + b->nopen == 0) b->first = std::chrono::steady_clock::now();
  const uint32_t idx = open ? b->nopen++ : b->nseal++;
  const uint64_t in_off = b->in_used, out_off = b->out_used;
  b->in_used += in_need;
  b->out_used += out_need;
  if (open) b->open_max = std::max(b->open_max, len);
  else b->seal_max = std::max(b->seal_max, len);
  b->writers += 1;
  b->users += 1;
  const uint64_t gen = b->gen;
  lk.unlock();
  if (len || open) memcpy(b->in + in_off, src, (size_t)len + (open ? 16u : 0u));
  wg_pkt d{in_off, out_off, counter, len, key_slot};
  (open ? b->odesc : b->sdesc)[idx] = d;
  lk.lock();
  b->writers -= 1;
  if (b->writers == 0 || b->nseal + b->nopen == 1) B->cv_work.notify_one();
  b->cv_done.wait(lk, [&] { return b->done_gen.load(std::memory_order_acquire) == gen; });
  rc = B->launch_error;
  const std::string msg = B->launch_msg;
  lk.unlock();
  int result = WG_OK;
  if (rc != WG_OK) {
    result = fail(rc, "batched launch failed: %s", msg.c_str());
  } else if (open) {
    if (b->status[idx] != WG_PKT_OK) result = 1;  // dst untouched, as ChaCha20Poly1305.java:51-53 throws first
    else if (len) memcpy(dst, b->out + out_off, len);
  } else {
    memcpy(dst, b->out + out_off, (size_t)len + 16u);
  }
  lk.lock();
  if (--b->users == 0 && b->state == BatchBuf::DONE) {
    b->state = BatchBuf::FREE;
    B->cv_free.notify_all();
  }
  return result;
}

}  // namespace

extern "C" {

int wg_seal1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint8_t* out) {
  if (!c || (!pt && len) || !out) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  return batcher_submit(c, false, key_slot, counter, pt, len, out);
}

int wg_open1(wg_ctx* c, uint32_t key_slot, uint64_t counter, const uint8_t* in, uint32_t len, uint8_t* pt) {
  if (!c || !in || (!pt && len)) return fail(WG_EINVAL, "NULL argument");
  if (len > WG_MAX_PACKET) return fail(WG_E2BIG, "packet of %u bytes", len);
  if (key_slot >= c->key_slots) return fail(WG_ERANGE, "key slot %u", key_slot);
  return batcher_submit(c, true, key_slot, counter, in, len, pt);
}

int wg_batcher_config(wg_ctx* c, uint32_t max_batch, uint32_t window_us) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  if (max_batch == 0 || max_batch > kBatchPktsDefault)
    return fail(WG_EINVAL, "max_batch must be 1..%u", kBatchPktsDefault);
  Batcher* B;
  int rc;
  if ((rc = batcher_get(c, &B)) != WG_OK) return rc;
  std::lock_guard<std::mutex> lk(B->mu);
  B->max_pkts = max_batch;
  B->window_us = window_us;
  return WG_OK;
}

int wg_batcher_stats(wg_ctx* c, uint64_t* launches, uint64_t* packets) {
  if (!c) return fail(WG_EINVAL, "NULL context");
  uint64_t l = 0, p = 0;
  {
    std::lock_guard<std::mutex> lk(c->batcher_mu);
    if (c->batcher) {
      std::lock_guard<std::mutex> lk2(c->batcher->mu);
      l = c->batcher->launches;
      p = c->batcher->packets;
    }
  }
  if (launches) *launches = l;
  if (packets) *packets = p;
  return WG_OK;
}

}  // extern "C"
