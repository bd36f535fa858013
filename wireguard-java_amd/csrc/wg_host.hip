// wg_host.hip — host-pointer entry points of libwgaead.so (included by wg_capi.hip):
// batches whose buffers live in host memory (tun ring in, UDP ring out), pinned rings,
// and the general AEAD / primitive call on host buffers.
#pragma once

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
  if (flags & ~WG_F_UNIFORM) return fail(WG_EINVAL, "host batches take only WG_F_UNIFORM (flags 0x%x)", flags);
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

extern "C" {

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

}  // extern "C"
