/*
 * wg_oracle.c — CPU restatement of the reference's transport-data AEAD.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the checker for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product library (libwgaead.so) never links or calls it.
 *
 * Restated from the algorithm, not copied. Each function cites the reference
 * file:line it follows (paths relative to the reference repository root):
 *   ChaCha20 block        ax.xz.wireguard.noise/src/main/c/chacha-generic.c:10-78
 *   ChaCha20 XOR stream   chacha-generic.c:81-97 (32-bit counter in state word 12)
 *   state layout          ax.xz.wireguard.noise/src/main/java/ax/xz/wireguard/noise/crypto/ChaCha20.java:55-74
 *   Poly1305              poly1305-donna.c:26-61, poly1305-donna-64.h:75-223 (restated in radix 2^64)
 *   AEAD composition      .../noise/crypto/ChaCha20Poly1305.java:31-97
 *   transport nonce       .../noise/handshake/SymmetricKeypair.java:52-61 (LE64(counter) || 0^4)
 *   cipher / decipher     SymmetricKeypair.java:63-83
 *
 * Parity pinning: tests/test_oracle.py checks this file against the RFC 8439
 * vectors held in the reference's own tests (ChaCha20Test.java, Poly1305Test.java),
 * the donna self-test vectors (poly1305-donna.c:83-201) and OpenSSL's
 * EVP_chacha20_poly1305 with the reference nonce layout (tests/golden/, scripts beside
 * the fixtures). There is no oracle/_ref build of the reference C.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#include "../include/wgaead.h"

typedef unsigned __int128 u128;

static inline uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t ld64(const uint8_t* p) { return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32); }
static inline void st32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void st64(uint8_t* p, uint64_t v) { st32(p, (uint32_t)v); st32(p + 4, (uint32_t)(v >> 32)); }
static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* One ChaCha20 block: 20 rounds (RFC 8439 2.3) + feed-forward, little-endian
 * serialisation. chacha-generic.c:65-78 (the reference increments state[12]
 * after the block; callers here pass the counter explicitly instead). */
void oracle_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u; /* ChaCha20.java:61-64 */
  for (int i = 0; i < 8; ++i) s[4 + i] = ld32(key + 4 * i);                         /* ChaCha20.java:67 */
  s[12] = counter;                                                                 /* ChaCha20.java:70 */
  for (int i = 0; i < 3; ++i) s[13 + i] = ld32(nonce + 4 * i);                      /* ChaCha20.java:73 */
  memcpy(x, s, sizeof x);
#define QR(a, b, c, d)                                   \
  x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);            \
  x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);            \
  x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);             \
  x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
  for (int r = 0; r < 10; ++r) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
#undef QR
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + s[i]);
}

/* ChaCha20 stream XOR starting at block counter ctr0; counter wraps at 2^32
 * exactly as state[12]++ does (chacha-generic.c:77, :81-97). */
void oracle_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t ctr0, const uint8_t* in,
                         uint8_t* out, size_t len) {
  uint8_t ks[64];
  uint32_t ctr = ctr0;
  for (size_t off = 0; off < len; off += 64, ++ctr) {
    oracle_chacha20_block(key, ctr, nonce, ks);
    size_t n = len - off < 64 ? len - off : 64;
    for (size_t i = 0; i < n; ++i) out[off + i] = in[off + i] ^ ks[i];
  }
}

/* ---- Poly1305 (RFC 8439 2.5), radix 2^64 with 128-bit products ---- */
typedef struct {
  uint64_t r0, r1, s1; /* s1 = r1 + r1/4 (= 5*r1/4, valid because clamping clears r1's low 2 bits) */
  uint64_t h0, h1, h2;
  uint64_t pad0, pad1;
  uint8_t buf[16];
  size_t used;
} poly_state;

/* clamp r &= 0x0ffffffc0ffffffc0ffffffc0fffffff (poly1305-donna-64.h:80-86) */
static void poly_init(poly_state* st, const uint8_t key[32]) {
  st->r0 = ld64(key) & 0x0ffffffc0fffffffULL;
  st->r1 = ld64(key + 8) & 0x0ffffffc0ffffffcULL;
  st->s1 = st->r1 + (st->r1 >> 2);
  st->h0 = st->h1 = st->h2 = 0;
  st->pad0 = ld64(key + 16);
  st->pad1 = ld64(key + 24);
  st->used = 0;
}

/* h = (h + m + hibit*2^128) * r mod 2^130-5, partially reduced (donna-64.h:101-151) */
static void poly_block(poly_state* st, const uint8_t m[16], uint64_t hibit) {
  uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2;
  u128 t = (u128)h0 + ld64(m);
  h0 = (uint64_t)t;
  t = (u128)h1 + ld64(m + 8) + (uint64_t)(t >> 64);
  h1 = (uint64_t)t;
  h2 += (uint64_t)(t >> 64) + hibit;
  /* (h0 + h1 2^64 + h2 2^128)(r0 + r1 2^64), folding 2^128*r1 = 2^130*(r1/4) == 5*(r1/4) */
  u128 d0 = (u128)h0 * st->r0 + (u128)h1 * st->s1;
  u128 d1 = (u128)h0 * st->r1 + (u128)h1 * st->r0 + (u128)h2 * st->s1;
  uint64_t d2 = h2 * st->r0; /* h2 <= 7, r0 < 2^60 */
  h0 = (uint64_t)d0;
  d1 += (uint64_t)(d0 >> 64);
  h1 = (uint64_t)d1;
  d2 += (uint64_t)(d1 >> 64);
  /* d2 holds bits >= 2^128: keep 2 bits in h2, fold the rest (x 2^130 == x*5) */
  h2 = d2 & 3;
  uint64_t c = (d2 >> 2) * 5;
  t = (u128)h0 + c;
  h0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64);
  h1 = (uint64_t)t;
  h2 += (uint64_t)(t >> 64);
  st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

/* streaming update with a 16-byte carry buffer (poly1305-donna.c:26-61) */
static void poly_update(poly_state* st, const uint8_t* m, size_t n) {
  while (n) {
    if (st->used == 0 && n >= 16) {
      poly_block(st, m, 1);
      m += 16; n -= 16;
      continue;
    }
    size_t k = 16 - st->used < n ? 16 - st->used : n;
    memcpy(st->buf + st->used, m, k);
    st->used += k; m += k; n -= k;
    if (st->used == 16) { poly_block(st, st->buf, 1); st->used = 0; }
  }
}

/* final partial block (0x01 pad, no hibit), canonical reduction, + s (donna-64.h:154-223) */
static void poly_finish(poly_state* st, uint8_t mac[16]) {
  if (st->used) {
    uint8_t b[16] = {0};
    memcpy(b, st->buf, st->used);
    b[st->used] = 1;
    poly_block(st, b, 0);
  }
  uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2;
  /* h < 2^130 + small; reduce once more so h < 2^130 */
  uint64_t c = (h2 >> 2) * 5;
  h2 &= 3;
  u128 t = (u128)h0 + c; h0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64); h1 = (uint64_t)t; h2 += (uint64_t)(t >> 64);
  /* g = h + 5 - 2^130; select g if h >= p */
  t = (u128)h0 + 5; uint64_t g0 = (uint64_t)t;
  t = (u128)h1 + (uint64_t)(t >> 64); uint64_t g1 = (uint64_t)t;
  uint64_t g2 = h2 + (uint64_t)(t >> 64);
  if (g2 >> 2) { h0 = g0; h1 = g1; }
  t = (u128)h0 + st->pad0; h0 = (uint64_t)t;
  h1 = h1 + st->pad1 + (uint64_t)(t >> 64);
  st64(mac, h0);
  st64(mac + 8, h1);
  memset(st, 0, sizeof *st);
}

void oracle_poly1305(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t tag[16]) {
  poly_state st;
  poly_init(&st, key);
  poly_update(&st, msg, len);
  poly_finish(&st, tag);
}

/* RFC 8439 2.6: one-time key = first 32 bytes of block 0 (ChaCha20Poly1305.java:11-14) */
void oracle_poly1305_keygen(const uint8_t key[32], const uint8_t nonce[12], uint8_t otk[32]) {
  uint8_t b[64];
  oracle_chacha20_block(key, 0, nonce, b);
  memcpy(otk, b, 32);
}

/* MAC over aad || pad16 || ct || pad16 || le64(aadLen or 0) || le64(ctLen)
 * (ChaCha20Poly1305.java:63-93; a NULL aad still contributes the 0 length word, :88) */
static void aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad, size_t aad_len,
                     const uint8_t* ct, size_t len, uint8_t tag[16]) {
  static const uint8_t zeros[16] = {0};
  uint8_t otk[32], lens[16];
  poly_state st;
  oracle_poly1305_keygen(key, nonce, otk);
  poly_init(&st, otk);
  if (aad_len) {
    poly_update(&st, aad, aad_len);
    if (aad_len % 16) poly_update(&st, zeros, 16 - aad_len % 16);
  }
  poly_update(&st, ct, len);
  if (len % 16) poly_update(&st, zeros, 16 - len % 16);
  st64(lens, (uint64_t)aad_len);
  st64(lens + 8, (uint64_t)len);
  poly_update(&st, lens, 16);
  poly_finish(&st, tag);
}

/* poly1305AeadEncrypt: ct = ChaCha20(ctr=1) ^ pt, tag over ct (ChaCha20Poly1305.java:35-38) */
void oracle_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad, size_t aad_len,
                      const uint8_t* pt, size_t len, uint8_t* ct, uint8_t tag[16]) {
  oracle_chacha20_xor(key, nonce, 1, pt, ct, len);
  aead_tag(key, nonce, aad, aad_len, ct, len, tag);
}

/* poly1305AeadDecrypt: verify first, decrypt only on success; pt untouched on failure
 * (ChaCha20Poly1305.java:40-56). Returns 0 on success, -1 on a bad tag. */
int oracle_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad, size_t aad_len,
                     const uint8_t* ct, size_t len, const uint8_t tag[16], uint8_t* pt) {
  uint8_t expect[16];
  aead_tag(key, nonce, aad, aad_len, ct, len, expect);
  if (memcmp(expect, tag, 16) != 0) return -1;
  oracle_chacha20_xor(key, nonce, 1, ct, pt, len);
  return 0;
}

/* SymmetricKeypair.getNonceBytes: JAVA_LONG (native = little-endian) at offset 0
 * of a 12-byte buffer whose last 4 bytes stay zero (SymmetricKeypair.java:52-61). */
void oracle_transport_nonce(uint64_t counter, uint8_t nonce[12]) {
  st64(nonce, counter);
  nonce[8] = nonce[9] = nonce[10] = nonce[11] = 0;
}

/* ---- batch drivers over the same descriptors as the C-ABI (include/wgaead.h) ---- */
typedef struct {
  const wg_pkt* d;
  size_t lo, hi;
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* keys;
  uint32_t* status;
  int open;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  uint8_t nonce[12];
  for (size_t i = j->lo; i < j->hi; ++i) {
    const wg_pkt* p = &j->d[i];
    const uint8_t* key = j->keys + 32 * (size_t)p->key_slot;
    oracle_transport_nonce(p->counter, nonce);
    if (!j->open) {
      uint8_t* o = j->out + p->out_off;
      oracle_aead_seal(key, nonce, NULL, 0, j->in + p->in_off, p->len, o, o + p->len);
    } else {
      const uint8_t* c = j->in + p->in_off;
      int rc = oracle_aead_open(key, nonce, NULL, 0, c, p->len, c + p->len, j->out + p->out_off);
      if (j->status) j->status[i] = rc == 0 ? WG_PKT_OK : WG_PKT_BADTAG;
    }
  }
  return NULL;
}

static int run_batch(const wg_pkt* d, size_t n, const uint8_t* in, uint8_t* out, const uint8_t* keys,
                     uint32_t* status, int open, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  batch_job jobs[256];
  size_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    size_t lo = t * per, hi = lo + per < n ? lo + per : n;
    if (lo >= hi) break;
    jobs[t] = (batch_job){d, lo, hi, in, out, keys, status, open};
    if (threads == 1) { batch_worker(&jobs[t]); continue; }
    if (pthread_create(&tid[t], NULL, batch_worker, &jobs[t]) != 0) return -1;
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  return 0;
}

int oracle_seal_batch(const wg_pkt* d, size_t n, const uint8_t* in, uint8_t* out, const uint8_t* keys, int threads) {
  return run_batch(d, n, in, out, keys, NULL, 0, threads);
}

int oracle_open_batch(const wg_pkt* d, size_t n, const uint8_t* in, uint8_t* out, const uint8_t* keys,
                      uint32_t* status, int threads) {
  return run_batch(d, n, in, out, keys, status, 1, threads);
}
