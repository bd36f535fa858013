/*
 * wgaead.h — C-ABI of libwgaead.so, the MI355X (gfx950) transport-data AEAD.
 *
 * This is the drop-in boundary for the reference's ChaCha20-Poly1305 path in
 * module ax.xz.wireguard.noise. Every entry point below names the reference
 * interface it replaces (file:line, paths relative to the reference root,
 * abbreviated: NOISE = ax.xz.wireguard.noise/src/main/java/ax/xz/wireguard/noise).
 * The Java host binds these through Panama exactly as the reference binds
 * libchacha / libpoly1305-donna today (NOISE/crypto/ChaCha20.java:14-42,
 * NOISE/crypto/Poly1305.java:24-77); see INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only; no exceptions cross the ABI.
 *  - Every function returns 0 (WG_OK) or a negative WG_E* code. A per-packet
 *    authentication failure is NOT an error return: it is reported in the
 *    status array (WG_PKT_BADTAG), mirroring the per-packet
 *    AEADBadTagException of NOISE/crypto/ChaCha20Poly1305.java:51-53.
 *  - "batch" calls take DEVICE pointers and are asynchronous on `stream`
 *    (a hipStream_t passed as void*, used as-is: NULL is HIP's default stream;
 *    wg_ctx_stream(ctx) returns the context's own non-blocking stream).
 *    The "host" calls take host pointers and return after completion.
 *  - Packets are independent (no cross-packet state): a batch shards freely
 *    across devices; no collective is involved (one wg_ctx per device).
 *  - Nonce layout of transport packets is the reference's, not the WireGuard
 *    spec's: nonce = LE64(counter) || 00 00 00 00 (NOISE/handshake/SymmetricKeypair.java:52-61).
 */
#ifndef WGAEAD_H
#define WGAEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WG_OK 0
#define WG_EINVAL (-22)    /* bad argument (NULL, n mismatch, unaligned key slot, ...) */
#define WG_ENOMEM (-12)    /* device or pinned allocation failed */
#define WG_ERANGE (-34)    /* key slot / buffer bound exceeded by a descriptor */
#define WG_E2BIG (-7)      /* packet longer than WG_MAX_PACKET */
#define WG_EDEVICE (-5)    /* HIP runtime error (message via wg_last_error) */
#define WG_ESELFTEST (-74) /* known-answer self test failed */
#define WG_EAGAIN (-11)    /* wg_submit_*: no free queue slot within the queue's submit timeout */
/* wg_seal1 / wg_open1 / wg_submit_*: the key slot holds no key (never set, or zeroed by wg_keys_zero).
 * SymmetricKeypair.clean() closes its key arena, so a later cipher() / decipher() throws instead of
 * encrypting (SymmetricKeypair.java:85-93); these paths refuse the packet the same way rather than
 * sealing it under the publicly known all-zero key. */
#define WG_ENOKEY (-126)

#define WG_PKT_OK 0u
#define WG_PKT_BADTAG 1u
/* (2 = WG_PKT_BADHDR, the parse status of wg_parse_open) */
/* written by wg_rx_check (receive-side checks after open; only WG_PKT_OK packets are examined) */
#define WG_PKT_KEEPALIVE 3u /* zero-length plaintext: a keepalive, not forwarded */
#define WG_PKT_BADIP 4u     /* IP version nibble not 4 or 6, or too short for the destination address */
#define WG_PKT_FILTERED 5u  /* destination outside the key slot's AllowedIPs filter */
#define WG_PKT_REPLAY 6u    /* counter replayed, too old for the window, or >= 2^64 - 2^13 - 1 */
/* a queued packet whose key slot was zeroed between its submit's check and its copy into the ring:
 * never sealed or opened (its output is untouched) */
#define WG_PKT_NOKEY 7u
/* a queued packet (wg_submit_*) whose batch could not run (launch or stream error) */
#define WG_PKT_FAILED 255u

#define WG_TAG_SIZE 16   /* Crypto.ChaChaPoly1305Overhead (NOISE/crypto/Crypto.java:14) */
#define WG_NONCE_SIZE 12 /* Crypto.ChaChaPoly1305NonceSize (NOISE/crypto/Crypto.java:13) */
#define WG_KEY_SIZE 32
#define WG_MAX_PACKET 65535u /* largest payload one workgroup tile accepts */

/* Transport packet descriptor (32 bytes). One per packet of a batch.
 *  seal: reads  in[in_off .. in_off+len)            plaintext
 *        writes out[out_off .. out_off+len+16)     ciphertext || tag
 *        (SymmetricKeypair.cipher: dst = ct || tag, SymmetricKeypair.java:63-74)
 *  open: reads  in[in_off .. in_off+len+16)         ciphertext || tag
 *        writes out[out_off .. out_off+len)         plaintext, only if the tag verifies;
 *        on a bad tag the plaintext range is zero-filled and status = WG_PKT_BADTAG;
 *        when the plaintext range overlaps in[in_off .. in_off+len+16) (in place, or moved back),
 *        the tag is verified before any byte is written and a forged packet's bytes stay as they
 *        were (ChaCha20Poly1305.java:40-56); an overlap that moves the plaintext forward is undefined
 *        (SymmetricKeypair.decipher: L = src.size - 16, SymmetricKeypair.java:76-83)
 *  counter: the 64-bit transport counter (TransportPacket.java:53-55); nonce built on device.
 *  key_slot: index into the context's device key table (wg_keys_set). */
typedef struct wg_pkt {
  uint64_t in_off;
  uint64_t out_off;
  uint64_t counter;
  uint32_t len;
  uint32_t key_slot;
} wg_pkt;

/* General AEAD / primitive descriptor (64 bytes) for the reference's static
 * crypto API (ChaCha20Poly1305, ChaCha20, Poly1305 classes): explicit 12-byte
 * nonce words, optional AAD, explicit initial block counter. */
typedef struct wg_aead_desc {
  uint64_t in_off;
  uint64_t out_off;
  uint64_t aad_off;   /* into the aad buffer (AEAD modes only) */
  uint32_t len;       /* payload bytes (excl. tag) */
  uint32_t aad_len;   /* 0 = no AAD (poly1305AeadEncrypt(key, nonce, ...) overloads) */
  uint32_t key_slot;  /* ChaCha key (AEAD, CIPHER) or 32-byte one-time key (MAC) */
  uint32_t ctr0;      /* CIPHER mode: initial 32-bit block counter (ChaCha20.chacha20(..., counter)) */
  uint32_t nonce[3];  /* state words 13..15, little-endian (ChaCha20.java:73) */
  uint32_t _reserved[3];
} wg_aead_desc;

typedef struct wg_ctx wg_ctx;

/* ---- library / context -------------------------------------------------- */

/* Known-answer self test on the device (RFC 8439 2.3.2/2.4.2/2.5.2/2.6.2/2.8.2
 * and the donna vectors). Returns 1 if all pass, like poly1305_power_on_self_test
 * which Poly1305.<clinit> checks (Poly1305.java:62-76). Creates and destroys a
 * temporary context on `device`. */
int wg_aead_selftest(int device);

/* Create a context bound to HIP device `device` with a key table of
 * `key_slots` 32-byte entries (zero-initialised).
 * Scheduling overrides read here from the environment, for A/B measurements only (none changes
 * a byte of output): WG_SLOT16=0|1, WG_MIXED_SPLIT=R, WG_UNIFORM16=k, WG_PRIO=0|1 (DESIGN.md §4.1,
 * §4.3); unset, the transport kernel plans every batch from its size and the WG_F_UNIFORM hint. */
int wg_ctx_create(int device, uint32_t key_slots, wg_ctx** out);
int wg_ctx_destroy(wg_ctx* ctx); /* zeroes the key table first */
int wg_ctx_device(const wg_ctx* ctx);
uint32_t wg_ctx_key_slots(const wg_ctx* ctx);
void* wg_ctx_stream(wg_ctx* ctx);       /* the context's hipStream_t */
int wg_sync(wg_ctx* ctx, void* stream); /* hipStreamSynchronize */
const char* wg_last_error(void);        /* thread-local text for the last error */
const char* wg_version(void);

/* NUMA node of HIP device `device`'s PCI function (sysfs), or -1 if unknown. A queue's dispatcher
 * thread runs on that node's CPUs (wg_queue_create); callers feeding the GPU from many threads
 * should place them there too (TransportManager's pools: numactl --cpunodebind, or a thread
 * factory that sets the affinity). */
int wg_device_numa_node(int device);

/* Transport kernel used by this context's wg_seal_batch / wg_open_batch / *_host calls
 * (a test and A/B hook beside the reference interface). name: "default"
 * or NULL or "transport" (k_transport, the product kernel), "wave1" (the round-1
 * k_wave kernel, kept as the performance baseline) or "tile" (k_tile, the general
 * AEAD kernel run on transport descriptors). lanes is ignored (kept for ABI stability).
 * variant (transport kernel only): 0 = a WG_F_AFTER_SEAL step is ONE k_step launch (each wave
 * seals its packets, then opens them); 1 = the same step as two launches, seal then open.
 * Every kernel and variant computes identical bytes; they differ only in speed. */
int wg_ctx_set_kernel(wg_ctx* ctx, const char* name, uint32_t lanes, uint32_t variant);

/* ---- keys: SymmetricKeypair(byte[] send, byte[] recv) and clean() ---------
 * (SymmetricKeypair.java:39-50 copies keys into a shared Arena; :85-93 zeroes them) */
int wg_keys_set(wg_ctx* ctx, uint32_t first_slot, uint32_t n, const uint8_t* keys_host /* n*32 */);
int wg_keys_zero(wg_ctx* ctx, uint32_t first_slot, uint32_t n);

/* ---- batched transport seal / open (device pointers) ----------------------
 * Replaces the per-packet ForkJoinPool fan-out of SymmetricKeypair.cipher /
 * decipher (TransportManager.java:41,70-93,137-158). `in_size` / `out_size`
 * are the byte sizes of the buffers; every descriptor is bounds-checked on
 * device against them (an out-of-range packet is skipped with status
 * WG_PKT_BADTAG on open / untouched output on seal, and the call returns 0).
 * `max_len`: every packet's len must be <= max_len (longer ones are treated
 * as out of range). Flags: WG_F_UNIFORM declares the lengths (nearly) equal: the
 * packets are taken in order; without it a mixed-length batch is first ordered
 * longest-first on the device, so every slot of the kernel gets a similar share of
 * rounds. Unknown flag bits are rejected (WG_EINVAL); wg_open_batch takes only
 * WG_F_UNIFORM and needs a status array when n > 0. Calls with mixed-length batches
 * on one context use a shared plan workspace: calls on different streams are ordered
 * by the library (the later one waits for the earlier one's plan). */
#define WG_F_UNIFORM 1u
/* WG_F_FRAME (wg_seal_batch only): also write the 16-B transport header at
 * out_off - 16 of every packet, exactly as wg_frame_seal does, from the receiver
 * table given to wg_ctx_set_receivers (k_frame_seal launched after the seal kernel
 * on the same stream). */
#define WG_F_FRAME 2u
/* WG_F_RX_FILTER (wg_open_batch only): the open kernel also runs wg_rx_check's WG_RX_FILTER
 * checks (keepalive, IP version, AllowedIPs of the key slot) on every packet whose tag verified
 * and writes the refined status itself, in the same launch; the replay window
 * stays a wg_rx_check call. */
#define WG_F_RX_FILTER 8u
/* Device array of receiver_index per key slot (n >= key_slots entries, device memory
 * of this context's device, 4-byte aligned, caller-owned, must outlive the seals that
 * use it); NULL clears it. */
int wg_ctx_set_receivers(wg_ctx* ctx, const uint32_t* receivers_dev, uint32_t n);
int wg_seal_batch(wg_ctx* ctx, const wg_pkt* desc_dev, uint32_t n, const uint8_t* in_dev, uint64_t in_size,
                  uint8_t* out_dev, uint64_t out_size, uint32_t max_len, uint32_t flags, void* stream);
int wg_open_batch(wg_ctx* ctx, const wg_pkt* desc_dev, uint32_t n, const uint8_t* in_dev, uint64_t in_size,
                  uint8_t* out_dev, uint64_t out_size, uint32_t* status_dev, uint32_t max_len, uint32_t flags,
                  void* stream);

/* ---- both directions in one launch (device pointers) ----------------------
 * A node seals its outgoing batch and opens its incoming batch at the same time: the
 * reference runs both on one ForkJoinPool (TransportManager.java:41 outgoing cipher,
 * :79 incoming decipher). wg_duplex_batch(seal, open) computes exactly what
 * wg_seal_batch(seal...) and wg_open_batch(open...) compute, in ONE kernel launch whose
 * workgroups alternate between the two batches, so neither batch's launch start and tail
 * leaves the device idle. The two batches run concurrently: the open batch must not read
 * bytes the seal batch writes in the same call (open the previous call's ciphertext).
 * seal->flags: WG_F_UNIFORM, WG_F_FRAME (as wg_seal_batch); seal->status is ignored.
 * open->flags: WG_F_UNIFORM, WG_F_AFTER_SEAL; open->status is required when open->n > 0.
 * Either n may be 0.
 * WG_F_AFTER_SEAL (open->flags): the open batch DOES read what the seal batch writes: open packet i
 *   is ordered after seal packet i, and after no other seal packet, so it may read what seal packet
 *   i writes but not what another seal packet of the call writes (same n in both batches; e.g. two
 *   peers in loopback, or a verify pass over what was just sealed). With the transport kernel and
 *   equal max_len / WG_F_UNIFORM on both sides (and no WG_F_FRAME) the step is ONE k_step launch in
 *   which every wave seals its packets and then opens the same batch positions; otherwise the seal
 *   launch and then the open launch run on `stream`. A mixed-length batch is ordered longest-first
 *   once, for both (its packets have the same lengths). Such a step on a mixed batch of max_len <= 2048
 *   plans in a workspace of its stream's own (up to 8 streams; WG_STREAM_WS=0: the shared one), so steps
 *   on different streams do not wait for each other. */
#define WG_F_AFTER_SEAL 4u
typedef struct wg_batch {
  const wg_pkt* desc; /* device, 16-byte aligned */
  const uint8_t* in;
  uint8_t* out;
  uint32_t* status;   /* open: WG_PKT_* per packet */
  uint64_t in_size;
  uint64_t out_size;
  uint32_t n;
  uint32_t max_len;
  uint32_t flags;
  uint32_t _reserved;
} wg_batch;
int wg_duplex_batch(wg_ctx* ctx, const wg_batch* seal, const wg_batch* open, void* stream);

/* ---- general AEAD + primitives (device pointers) --------------------------
 * WG_MODE_SEAL / WG_MODE_OPEN: ChaCha20Poly1305.poly1305AeadEncrypt / Decrypt
 *   with optional AAD and explicit nonce (ChaCha20Poly1305.java:31-60).
 * WG_MODE_CIPHER: ChaCha20.chacha20(key, nonce, in, out, counter) (ChaCha20.java:116-131)
 *   = libchacha chacha_cipher with state word 12 = ctr0 (chacha-generic.c:104-108).
 * WG_MODE_MAC: Poly1305 init/update/finish one-shot with a 32-byte one-time key
 *   (Poly1305.java:94-166 over poly1305-donna.c:26-69); tag at out[out_off]. */
#define WG_MODE_SEAL 0
#define WG_MODE_OPEN 1
#define WG_MODE_CIPHER 2
#define WG_MODE_MAC 3
int wg_aead_batch(wg_ctx* ctx, int mode, const wg_aead_desc* desc_dev, uint32_t n, const uint8_t* in_dev,
                  uint64_t in_size, const uint8_t* aad_dev, uint64_t aad_size, uint8_t* out_dev, uint64_t out_size,
                  uint32_t* status_dev, uint32_t max_len, void* stream);

/* ---- transport wire framing on device (device pointers) -------------------
 * Wire packet = 16-B header {u8 type=4, u8 zero[3], u32 receiver_index (LE),
 * u64 counter (LE)} followed by ct||tag (TransportPacket.java:18-35).
 * wg_frame_seal: for each desc[i] writes that header at out[desc[i].out_off - 16]
 *   with receiver_index = receivers_dev[desc[i].key_slot] and counter =
 *   desc[i].counter — UnencryptedOutgoingTransport.java:14-18 (type, receiver
 *   index) plus EncryptedOutgoingTransport.java:11-14 (counter). A header is
 *   written only for the packets the seal accepts (the same test: len <= max_len,
 *   key_slot < the context's key slots, in_off + len <= in_size, out_off + len + 16
 *   <= out_size) that also have out_off >= 16; every other packet is left untouched.
 *   Launch it on the same stream as wg_seal_batch, with the same in_size / max_len.
 * wg_parse_open: builds open descriptors from received wire packets without a
 *   host parse (UndecryptedIncomingTransport.java:20-33): wire packet i starts
 *   at wire_dev[pkt_off_dev[i]] and is pkt_len_dev[i] bytes long; desc_out[i] =
 *   {in_off = off + 16, out_off = off + pkt_len (plaintext right after the
 *   ciphertext in the same buffer, :30), counter = header counter, len =
 *   pkt_len - 32, key_slot = key_slot_dev[i]}. A packet whose type byte is not
 *   4, that is shorter than 32 bytes, or whose packet + plaintext overruns
 *   wire_size gets len = WG_LEN_INVALID (wg_open_batch then skips it with
 *   WG_PKT_BADTAG) and parse_status_dev[i] = WG_PKT_BADHDR (else WG_PKT_OK);
 *   parse_status_dev may be NULL. desc_out_dev must be 16-byte aligned. */
#define WG_PKT_BADHDR 2u
#define WG_LEN_INVALID 0xffffffffu
int wg_frame_seal(wg_ctx* ctx, const wg_pkt* desc_dev, uint32_t n, const uint32_t* receivers_dev, uint8_t* out_dev,
                  uint64_t out_size, uint64_t in_size, uint32_t max_len, void* stream);
int wg_parse_open(wg_ctx* ctx, const uint8_t* wire_dev, uint64_t wire_size, const uint64_t* pkt_off_dev,
                  const uint32_t* pkt_len_dev, const uint32_t* key_slot_dev, uint32_t n, wg_pkt* desc_out_dev,
                  uint32_t* parse_status_dev, void* stream);

/* ---- host-buffer entry points -----------------------------------------------
 * wg_seal1 / wg_open1 back the unchanged per-packet SymmetricKeypair API:
 *   cipher(src, dst): wg_seal1(ctx, send_slot, counter, src, L, dst) with dst of L+16 bytes
 *   decipher(counter, src, dst): wg_open1(ctx, recv_slot, counter, src, L, dst) with src of L+16 bytes
 *   returns WG_OK, or 1 for a bad tag (dst untouched, as NOISE/crypto/ChaCha20Poly1305.java:51-55).
 *   Thread-safe and synchronous per call (the per-packet ForkJoinPool fan-out of
 *   TransportManager.java:41,79,152-158), served without a kernel launch per packet: the
 *   packet (with its key, from a host mirror of the key table) goes into any free entry of a
 *   pinned 512-entry ring and is published by toggling the entry's doorbell bit; a persistent
 *   device kernel (k_pp, W waves, wave w owning entries [w 512/W, (w+1) 512/W)) polls the
 *   doorbells over PCIe, serves every published entry of its range in any order, and writes the
 *   result and a completion word back into pinned memory, on which the caller spins. A caller
 *   held up between claiming and publishing delays no other call. The kernel leaves the device
 *   as a whole after idle_us without work anywhere in it (and after at most 250 ms) and the next
 *   call relaunches it. A call that fails after publishing (a refused launch) leaves its entry to
 *   the next server, which completes it; the entry is then reused. Packets longer than 4080 bytes
 *   (past the reference pipeline's 4-KB buffers) take the host batch path.
 * wg_pp_config(ctx, waves, idle_us): waves of that kernel (a power of two, 1..64, default 16) and
 *   its idle timeout (µs, default 20000; 0 = default). Changing it stops a running server first.
 * wg_batcher_config(ctx, max_batch, window_us): the round-2 batcher's knobs; accepted and ignored
 *   (the persistent server has no batch size or window).
 * wg_batcher_stats: server launches and packets served by the per-packet path.
 * wg_seal_host / wg_open_host: a batch in host memory (tun ring in, UDP ring out).
 *   If `in` and `out` are pinned, device-mapped host memory (wg_host_alloc /
 *   wg_host_register) the kernel reads and writes them directly over PCIe
 *   (zero-copy); otherwise the batch moves through device mirrors in chunks with
 *   H2D, kernel and D2H overlapped on three streams. Only packet bytes are written
 *   to `out_host` (bytes between packets — wire headers, ring slack — are kept).
 *   On a bad tag the plaintext range is zero-filled and status[i] = WG_PKT_BADTAG.
 *   flags: WG_F_UNIFORM only. */
/* ---- receive side after open: keepalives, AllowedIPs, replay window -------
 * TransportManager.processDecryptedTransport (TransportManager.java:98-119) for a whole
 * opened batch, on the device: a packet whose status is WG_PKT_OK becomes
 *   WG_PKT_KEEPALIVE  if len == 0 (:103-105, not forwarded to the tun device);
 *   WG_PKT_BADIP      if its first nibble is not 4 or 6, or it is shorter than the
 *                     destination address's end (destinationIPOf, :124-130, throws);
 *   WG_PKT_FILTERED   if its key slot has an AllowedIPs filter (wg_slot_filters_set) and
 *                     the destination (bytes 16..19 of IPv4, 24..39 of IPv6) is not in it
 *                     (destinationFilter.search, :106-108; util/IPFilter.java:49-61);
 * and stays WG_PKT_OK otherwise (forwarded). Flags: WG_RX_FILTER runs those checks;
 * WG_RX_REPLAY first applies the key slot's replay window (wg_replay_enable), which the
 * reference does not have: a packet is WG_PKT_REPLAY if its counter is >= 2^64 - 2^13 - 1,
 * repeats an earlier WG_PKT_OK packet of the same key slot in this batch, is more than
 * window_bits behind the highest counter accepted before this batch, or was already
 * accepted; the window then advances past this batch's accepted counters (the window slides
 * between batches). Asynchronous on `stream`; run it after wg_open_batch on
 * the same stream. pt / pt_size: the open's output buffer (plaintexts at out_off). With
 * WG_RX_REPLAY a batch holds at most 2^30 packets; checks on different streams of one context
 * are ordered by the library (they share the window's scratch).
 *
 * wg_filter_set: AllowedIPs filter `filter_id` (< WG_MAX_FILTERS) from n prefixes, exactly as
 *   IPFilter.insert builds its trie (util/IPFilter.java:30-42), including its search rule:
 *   a prefix matches an address if the trie walk passes the prefix's node at a depth below
 *   the address width, so /32 (IPv4) and /128 (IPv6) entries never match - as in the
 *   reference, whose IPFilter.allowingAll() (0.0.0.0/32, ::/128) lets nothing through.
 *   Replaces any earlier filter with that id. A key slot without a filter passes every
 *   destination; a slot mapped to an id never set drops every destination (an empty
 *   IPFilter, :9-16).
 * wg_slot_filters_set: filter id per key slot for slots [first_slot, first_slot + n)
 *   (WG_NO_FILTER: none); the reference keeps one filter per peer (TransportManager.java:44,53).
 * wg_replay_enable: window of window_bits (a multiple of 64, <= 65536; 0 disables) per key
 *   slot, all windows empty. wg_keys_set / wg_keys_zero and wg_replay_reset empty the
 *   windows of the slots they touch (a new key is a new session).
 * wg_replay_state: a slot's window (top = highest accepted counter + 1, 0 if none; bits =
 *   window_bits / 64 words, bit (c mod window_bits) set for accepted counter c in the window). */
#define WG_MAX_FILTERS 65536u
#define WG_NO_FILTER 0xFFFFFFFFu
#define WG_RX_FILTER 1u
#define WG_RX_REPLAY 2u
typedef struct wg_prefix {
  uint8_t family;     /* 4 or 6 */
  uint8_t prefix_len; /* 0..32 or 0..128 */
  uint8_t addr[16];   /* network byte order; IPv4 in addr[0..3] */
} wg_prefix;
int wg_filter_set(wg_ctx* ctx, uint32_t filter_id, const wg_prefix* prefixes, uint32_t n);
int wg_slot_filters_set(wg_ctx* ctx, uint32_t first_slot, uint32_t n, const uint32_t* filter_ids_host);
int wg_replay_enable(wg_ctx* ctx, uint32_t window_bits);
int wg_replay_reset(wg_ctx* ctx, uint32_t first_slot, uint32_t n);
int wg_replay_state(wg_ctx* ctx, uint32_t slot, uint64_t* top, uint64_t* bits, uint32_t words);
int wg_rx_check(wg_ctx* ctx, const wg_pkt* desc_dev, uint32_t n, const uint8_t* pt_dev, uint64_t pt_size,
                uint32_t* status_dev, uint32_t flags, void* stream);

int wg_seal1(wg_ctx* ctx, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint8_t* out);
int wg_open1(wg_ctx* ctx, uint32_t key_slot, uint64_t counter, const uint8_t* in, uint32_t len, uint8_t* pt);
int wg_pp_config(wg_ctx* ctx, uint32_t waves, uint32_t idle_us);
/* Diagnostic: the stages of the calling thread's last wg_seal1 / wg_open1, in ns (out[0..7]: total,
 * claim, publish, wait for the completion, device service time, copy-out, slept on the futex 0/1,
 * relaunched the server 0/1); recorded only when WG_PP_CALL_STAMPS=1 is set before the context's
 * first per-packet call (zeros otherwise); tools/batcher_bench stamps=1 reports the slowest call's. */
int wg_pp_last_call(uint64_t* out, uint32_t n);
int wg_batcher_config(wg_ctx* ctx, uint32_t max_batch, uint32_t window_us);
int wg_batcher_stats(wg_ctx* ctx, uint64_t* launches, uint64_t* packets);
int wg_seal_host(wg_ctx* ctx, const wg_pkt* desc_host, uint32_t n, const uint8_t* in_host, uint64_t in_size,
                 uint8_t* out_host, uint64_t out_size, uint32_t max_len, uint32_t flags);
int wg_open_host(wg_ctx* ctx, const wg_pkt* desc_host, uint32_t n, const uint8_t* in_host, uint64_t in_size,
                 uint8_t* out_host, uint64_t out_size, uint32_t* status_host, uint32_t max_len, uint32_t flags);
/* ---- asynchronous batch submission -----------------------
 * The reference's TransportManager hands every packet to a ForkJoinPool worker that calls
 * cipher / decipher synchronously and then queues the result for the UDP / tun worker
 * (TransportManager.java:41,70-93,137-158; EstablishedSession.java:88-90). A queue replaces
 * that synchronous call: producers enqueue packets and return at once, one host thread per
 * queue batches whatever is waiting into k_transport launches over a pinned, device-mapped
 * ring (zero-copy), and the consumer reaps the results from a completion queue.
 *   wg_queue_create(ctx, mode, capacity, max_len, max_batch, &q): a seal (WG_MODE_SEAL) or open
 *     (WG_MODE_OPEN) queue of `capacity` slots (rounded up to a power of two; 0 = 65536) for
 *     payloads of at most max_len bytes (0 = 2032, the reference pipeline's incoming limit;
 *     at most WG_QUEUE_MAX_LEN), batches of at most max_batch packets (0 = 8192).
 *   wg_submit_seal(q, key_slot, counter, pt, len, user): copies the plaintext into a free slot
 *     and queues it; the nonce is LE64(counter) || 0^4 (SymmetricKeypair.java:52-61), the key
 *     the one key_slot holds at the time of the submit (copied into the slot with the packet, as the
 *     reference's synchronous cipher() uses the key it holds when called: a later wg_keys_set /
 *     wg_keys_zero of the slot does not change a queued packet; the copy is wiped when the packet's
 *     batch completes). A slot without a key (never set, or zeroed) is refused: WG_ENOKEY. Blocks only while every slot is in
 *     use (until the consumer calls wg_reap_done), and then at most the queue's submit timeout:
 *     returns WG_EAGAIN after it. Thread-safe: any number of producers.
 *   wg_submit_open(q, key_slot, counter, ct_tag, len, user): the same for ct || tag (len + 16 B).
 *   wg_submit_seal_n / wg_submit_open_n(q, p, n): n packets in one call, as n wg_submit_* calls in
 *     order from one thread, but with one lane lock and one publication per run of free slots.
 *     Returns how many were queued: n, or fewer (at least 1) when the submit timeout ran out
 *     partway; WG_EAGAIN when it ran out before the first. Every entry is checked first: a bad one
 *     fails the call (WG_EINVAL / WG_E2BIG / WG_ERANGE) with nothing queued. While it copies packet
 *     k it prefetches the bytes of packet k + 2 (WG_QUEUE_PREFETCH=0..8 sets the distance), so
 *     handing over completions of another queue (GPU-written, not in this core's caches) is fast.
 *   wg_reap(q, out, max, timeout_us): up to max completions (waits up to timeout_us for the
 *     first); returns how many, or a negative error. completion.data points into the queue's
 *     pinned ring: ct || tag (len + 16 B) for a seal, the plaintext (len B, valid when status is
 *     WG_PKT_OK; WG_PKT_BADTAG: rejected, ChaCha20Poly1305.java:51-55) for an open. Completions
 *     come back in batch order, not in submission order.
 *   wg_reap_done(q, c, n): the consumer is done with these completions (their slots are reused);
 *     each completion exactly once (a slot handed back twice would be given to two producers).
 *   wg_queue_set_submit_timeout(q, timeout_us): how long wg_submit_* waits for a free slot before it
 *     returns WG_EAGAIN (0, the default: without bound). A consumer that stalls then cannot wedge the
 *     producers (ForkJoinPool workers) for good.
 *   wg_queue_destroy: waits for the batches in flight; unreaped completions are dropped. Call it
 *     only once no thread is inside (or can still enter) wg_submit_* / wg_reap* on this queue.
 * A producer thread keeps up to 32 slots taken from other lanes in its lane's stash; slots stashed
 * by a thread that exits are used by the next thread that maps to the same lane. */
#define WG_QUEUE_MAX_LEN 16384u
typedef struct wg_queue wg_queue;
typedef struct wg_completion {
  uint64_t user;      /* the submitter's tag */
  uint64_t counter;
  uint8_t* data;      /* result in the pinned ring (see above) */
  uint32_t len;       /* payload bytes */
  uint32_t status;    /* WG_PKT_OK, WG_PKT_BADTAG (open), WG_PKT_NOKEY or WG_PKT_FAILED */
  uint32_t key_slot;
  uint32_t slot;      /* ring slot (handed back by wg_reap_done) */
  uint64_t submit_ns; /* steady-clock time of the submit (latency accounting) */
} wg_completion;
int wg_queue_create(wg_ctx* ctx, int mode, uint32_t capacity, uint32_t max_len, uint32_t max_batch, wg_queue** q);
int wg_queue_destroy(wg_queue* q);
int wg_submit_seal(wg_queue* q, uint32_t key_slot, uint64_t counter, const uint8_t* pt, uint32_t len, uint64_t user);
int wg_submit_open(wg_queue* q, uint32_t key_slot, uint64_t counter, const uint8_t* ct_tag, uint32_t len,
                   uint64_t user);
typedef struct wg_submit {
  uint64_t user;        /* the submitter's tag (echoed in the completion) */
  uint64_t counter;     /* nonce = LE64(counter) || 0^4 */
  const uint8_t* data;  /* seal: the plaintext (len B); open: ct || tag (len + 16 B) */
  uint32_t len;         /* payload bytes */
  uint32_t key_slot;
} wg_submit;
int wg_submit_seal_n(wg_queue* q, const wg_submit* p, uint32_t n);
int wg_submit_open_n(wg_queue* q, const wg_submit* p, uint32_t n);
int wg_reap(wg_queue* q, wg_completion* out, uint32_t max, uint32_t timeout_us);
int wg_reap_done(wg_queue* q, const wg_completion* done, uint32_t n);
int wg_queue_stats(wg_queue* q, uint64_t* batches, uint64_t* packets);
int wg_queue_set_submit_timeout(wg_queue* q, uint32_t timeout_us);
/* Diagnostic: ring slots whose copy of a session key is not all zero. A slot's key copy is wiped as
 * soon as its batch has completed, so with nothing in flight this is 0 (no key outlives the packets
 * that used it in pinned memory, as clean() leaves none, SymmetricKeypair.java:85-89). */
uint32_t wg_queue_key_residue(const wg_queue* q);

/* Pinned host rings for the host path (the reference's packet buffers come from
 * a native pool, Pool.java:96; pinning them makes wg_seal_host/wg_open_host zero-copy).
 * wg_host_alloc: page-locked, device-mapped, portable across devices.
 * wg_host_register: pin existing memory (e.g. a Java Arena segment) in place. */
int wg_host_alloc(wg_ctx* ctx, uint64_t bytes, void** out);
int wg_host_free(wg_ctx* ctx, void* p);
int wg_host_register(wg_ctx* ctx, void* p, uint64_t bytes);
int wg_host_unregister(wg_ctx* ctx, void* p);
/* General AEAD / primitives on host buffers with a per-call key list
 * (desc[i].key_slot indexes keys_host[nkeys][32]); the device copy of the keys
 * is zeroed before returning. */
int wg_aead_host(wg_ctx* ctx, int mode, const wg_aead_desc* desc_host, uint32_t n, const uint8_t* keys_host,
                 uint32_t nkeys, const uint8_t* in_host, uint64_t in_size, const uint8_t* aad_host, uint64_t aad_size,
                 uint8_t* out_host, uint64_t out_size, uint32_t* status_host);

/* ---- instrumentation -------------------------------------------------------
 * Average duration (ms) of the last `wg_timing_launches` kernel launches made
 * by batch calls on this context, measured with HIP events on the launch
 * stream (used by bench.py for the roofline `achieved` figure). */
int wg_timing_enable(wg_ctx* ctx, int on);
int wg_timing_read(wg_ctx* ctx, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* WGAEAD_H */
