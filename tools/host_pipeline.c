/* Host-to-host transport pipeline (BASELINE configs[4]): tun ring -> seal -> UDP send ->
 * UDP receive -> open -> tun ring, with every packet byte checked at the end.
 *
 * The reference reads tun packets (TunnelDeviceBond.java:30-41, POSIXTun.java:86-100), seals
 * each one and sends it as one UDP datagram with its 16-B transport header
 * (EstablishedSession.java:59-71, channel.send at :63); the receiver opens each datagram and
 * writes the plaintext to tun (TunnelDeviceBond.java:43-51). Here the same shape runs in
 * batches: the tun side is a ring of n IP packets in pinned host memory, the seal writes
 * header room + ct||tag into a UDP ring, sendmmsg() sends one datagram per packet to a
 * loopback UDP socket, a receiver thread recvmmsg()s them into a second ring, and the open
 * decrypts the received datagrams back into a tun-side ring.
 *
 * Backends: "gpu" = libwgaead (wg_seal_host / wg_open_host on pinned, device-mapped rings:
 * the kernels read and write host memory over PCIe); "cpu" = the C restatement of the
 * reference's AEAD (oracle/liboracle.so, dlopen'ed from --oracle PATH; bench.py runs this
 * only as its cpu_baseline leg) over T threads, the config[0]-shaped CPU pipeline.
 *
 * tun: when /dev/net/tun can be opened and configured (root / CAP_NET_ADMIN) the tun ring is
 * filled by reading a real tun device, fed by a local UDP sender; otherwise the ring holds
 * synthetic IPv4 packets and the JSON says why ("tun": "unavailable: ...").
 *
 * Build: gcc -O2 -pthread -Iinclude -o tools/host_pipeline tools/host_pipeline.c \
 *          -Lwireguard-java_amd -l:libwgaead.so -ldl -Wl,-rpath,'$ORIGIN/../wireguard-java_amd'
 * Run:   tools/host_pipeline [--backend gpu|cpu] [--oracle PATH] [--threads T] [--packets N]
 *                            [--len L] [--reps R] [--udp-streams K] [--chunks C] [--tun]
 *        (--tun: try a real tun device; K socket pairs with a sender and a receiver thread each;
 *         --chunks C > 1: seal, UDP and open overlap chunk by chunk, see "pipelined mode" below)
 * Output: one JSON line. */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/if.h>
#include <linux/if_tun.h>
#include <netinet/in.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "wgaead.h"

#define TUN_STRIDE 1440u
#define UDP_STRIDE 1472u /* 16-B header + up to 1420 + 16 tag, 16-B aligned slots */
#define HDR 16u

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* ---- backends ------------------------------------------------------------------------- */
typedef struct {
  int gpu;
  wg_ctx* ctx;
  int threads;
  uint8_t keys[32];
  int (*o_seal)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, int);
  int (*o_open)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, uint32_t*, int);
} backend;

static void* ring_alloc(backend* b, size_t bytes) {
  void* p = NULL;
  if (b->gpu) {
    if (wg_host_alloc(b->ctx, bytes, &p) != WG_OK) return NULL;
  } else if (posix_memalign(&p, 4096, bytes)) {
    return NULL;
  }
  memset(p, 0, bytes);
  return p;
}

static int do_seal(backend* b, const wg_pkt* d, uint32_t n, const uint8_t* in, uint64_t isz, uint8_t* out,
                   uint64_t osz, uint32_t max_len) {
  if (b->gpu) return wg_seal_host(b->ctx, d, n, in, isz, out, osz, max_len, WG_F_UNIFORM);
  return b->o_seal(d, n, in, out, b->keys, b->threads);
}

static int do_open(backend* b, const wg_pkt* d, uint32_t n, const uint8_t* in, uint64_t isz, uint8_t* out,
                   uint64_t osz, uint32_t* status, uint32_t max_len) {
  if (b->gpu) return wg_open_host(b->ctx, d, n, in, isz, out, osz, status, max_len, 0);
  return b->o_open(d, n, in, out, b->keys, status, b->threads);
}

/* ---- tun (optional) ------------------------------------------------------------------- */
static char g_tun_note[160] = "unavailable";

/* fill the tun ring by reading a real tun device fed with n local UDP datagrams of the
 * right size; returns 0 and stores the read rate on success */
static int tun_fill(uint8_t* ring, uint32_t n, uint32_t L, double* rate_gib) {
  int fd = open("/dev/net/tun", O_RDWR);
  if (fd < 0) {
    snprintf(g_tun_note, sizeof g_tun_note, "unavailable: open /dev/net/tun: %s", strerror(errno));
    return -1;
  }
  struct ifreq ifr;
  memset(&ifr, 0, sizeof ifr);
  ifr.ifr_flags = IFF_TUN | IFF_NO_PI;
  strncpy(ifr.ifr_name, "wgbench%d", IFNAMSIZ - 1);
  if (ioctl(fd, TUNSETIFF, &ifr) < 0) {
    snprintf(g_tun_note, sizeof g_tun_note, "unavailable: TUNSETIFF: %s", strerror(errno));
    close(fd);
    return -1;
  }
  int s = socket(AF_INET, SOCK_DGRAM, 0);
  struct ifreq a;
  memset(&a, 0, sizeof a);
  strncpy(a.ifr_name, ifr.ifr_name, IFNAMSIZ - 1);
  struct sockaddr_in* sin = (struct sockaddr_in*)&a.ifr_addr;
  sin->sin_family = AF_INET;
  inet_pton(AF_INET, "10.213.0.1", &sin->sin_addr);
  int ok = ioctl(s, SIOCSIFADDR, &a) == 0;
  inet_pton(AF_INET, "255.255.255.0", &sin->sin_addr);
  ok = ok && ioctl(s, SIOCSIFNETMASK, &a) == 0;
  a.ifr_mtu = 1500;
  ok = ok && ioctl(s, SIOCSIFMTU, &a) == 0;
  ok = ok && ioctl(s, SIOCGIFFLAGS, &a) == 0;
  a.ifr_flags |= IFF_UP | IFF_RUNNING;
  ok = ok && ioctl(s, SIOCSIFFLAGS, &a) == 0;
  if (!ok) {
    snprintf(g_tun_note, sizeof g_tun_note, "unavailable: configuring %s: %s", ifr.ifr_name, strerror(errno));
    close(s);
    close(fd);
    return -1;
  }
  /* L-byte IPv4 packets: 20 B IP + 8 B UDP + L - 28 B payload to 10.213.0.2 */
  struct sockaddr_in dst = {0};
  dst.sin_family = AF_INET;
  dst.sin_port = htons(9);
  inet_pton(AF_INET, "10.213.0.2", &dst.sin_addr);
  static uint8_t payload[1500];
  uint32_t got = 0;
  double t0 = now_s();
  while (got < n) {
    uint32_t burst = n - got < 64 ? n - got : 64;
    for (uint32_t k = 0; k < burst; ++k) sendto(s, payload, L - 28, 0, (struct sockaddr*)&dst, sizeof dst);
    for (uint32_t k = 0; k < burst && got < n; ++k) {
      ssize_t r = read(fd, ring + (size_t)got * TUN_STRIDE, TUN_STRIDE);
      if (r == (ssize_t)L) ++got;
      else if (r < 0) break;
    }
  }
  double dt = now_s() - t0;
  *rate_gib = (double)n * L / dt / (double)(1u << 30);
  snprintf(g_tun_note, sizeof g_tun_note, "read from %s (fed by local UDP sends)", ifr.ifr_name);
  close(s);
  close(fd);
  return 0;
}

/* ---- UDP receiver thread ---------------------------------------------------------------- */
typedef struct {
  int sock;
  uint8_t* ring;
  uint32_t n;
  uint32_t* lens;
  _Atomic uint32_t received;
  _Atomic int stop;
} rx_t;

static void* rx_loop(void* arg) {
  rx_t* r = (rx_t*)arg;
  struct mmsghdr msgs[256];
  struct iovec iov[256];
  while (!atomic_load(&r->stop)) {
    uint32_t base = atomic_load(&r->received);
    if (base >= r->n) break;
    uint32_t want = r->n - base < 256 ? r->n - base : 256;
    for (uint32_t k = 0; k < want; ++k) {
      iov[k].iov_base = r->ring + (size_t)(base + k) * UDP_STRIDE;
      iov[k].iov_len = UDP_STRIDE;
      memset(&msgs[k].msg_hdr, 0, sizeof msgs[k].msg_hdr);
      msgs[k].msg_hdr.msg_iov = &iov[k];
      msgs[k].msg_hdr.msg_iovlen = 1;
    }
    struct timespec to = {0, 20 * 1000 * 1000};
    int got = recvmmsg(r->sock, msgs, want, MSG_WAITFORONE, &to);
    if (got <= 0) continue;
    for (int k = 0; k < got; ++k) r->lens[base + k] = msgs[k].msg_len;
    atomic_store(&r->received, base + (uint32_t)got);
  }
  return NULL;
}

/* ---- one UDP stripe: a sender thread and a receiver thread on their own socket pair ---- */
typedef struct {
  int tx_sock;
  struct sockaddr_in addr;
  uint8_t* tx;
  uint32_t lo, hi, window, L, sent;
  rx_t R;
} stripe_t;

static void* tx_loop(void* arg) {
  stripe_t* S = (stripe_t*)arg;
  struct mmsghdr msgs[256];
  struct iovec iov[256];
  const uint32_t n = S->hi - S->lo;
  uint32_t sent = 0;
  double last_progress = now_s();
  while (sent < n) {
    const uint32_t inflight = sent - atomic_load(&S->R.received);
    if (inflight + 256 > S->window) {
      if (now_s() - last_progress > 0.2) break; /* receiver stalled: datagrams were dropped */
      continue;
    }
    last_progress = now_s();
    const uint32_t k = n - sent < 256 ? n - sent : 256;
    for (uint32_t j = 0; j < k; ++j) {
      iov[j].iov_base = S->tx + (size_t)(S->lo + sent + j) * UDP_STRIDE;
      iov[j].iov_len = HDR + S->L + 16;
      memset(&msgs[j].msg_hdr, 0, sizeof msgs[j].msg_hdr);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
      msgs[j].msg_hdr.msg_name = &S->addr;
      msgs[j].msg_hdr.msg_namelen = sizeof S->addr;
    }
    const int m = sendmmsg(S->tx_sock, msgs, k, 0);
    if (m > 0) sent += (uint32_t)m;
  }
  S->sent = sent;
  return NULL;
}

/* ---- pipelined mode (--chunks C > 1): seal, UDP and open overlap chunk by chunk --------------
 * The batch is cut into C chunks; the main thread seals chunk c+1 while the senders send chunk c and
 * an opener thread opens every chunk the receivers have completely received, as a tun reader, the
 * UDP workers and the peer's receive side would run at once. Stripe k of K sends, from every chunk,
 * the packets [c cs + k cs/K, c cs + (k+1) cs/K); its receiver places the i-th datagram it gets at
 * the position of the stripe's i-th packet (loopback UDP keeps a socket's order). */
typedef struct {
  stripe_t* S;
  int k, K;
  uint32_t n, cs, C;
  _Atomic uint32_t* sealed; /* chunks sealed so far */
} ptx_t;

static uint32_t ppos(uint32_t i, int k, int K, uint32_t cs) { /* the stripe's i-th packet */
  const uint32_t m = cs / (uint32_t)K;
  return (i / m) * cs + (uint32_t)k * m + i % m;
}

typedef struct {
  rx_t* R;
  int k, K;
  uint32_t cs;
  uint8_t* base; /* the whole received ring */
  uint32_t* lens;
} prx_t;

static void* prx_loop(void* arg) {
  prx_t* P = (prx_t*)arg;
  rx_t* r = P->R;
  struct mmsghdr msgs[256];
  struct iovec iov[256];
  while (!atomic_load(&r->stop)) {
    uint32_t have = atomic_load(&r->received);
    if (have >= r->n) break;
    uint32_t want = r->n - have < 256 ? r->n - have : 256;
    for (uint32_t j = 0; j < want; ++j) {
      iov[j].iov_base = P->base + (size_t)ppos(have + j, P->k, P->K, P->cs) * UDP_STRIDE;
      iov[j].iov_len = UDP_STRIDE;
      memset(&msgs[j].msg_hdr, 0, sizeof msgs[j].msg_hdr);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
    }
    struct timespec to = {0, 20 * 1000 * 1000};
    int got = recvmmsg(r->sock, msgs, want, MSG_WAITFORONE, &to);
    if (got <= 0) continue;
    for (int j = 0; j < got; ++j) P->lens[ppos(have + (uint32_t)j, P->k, P->K, P->cs)] = msgs[j].msg_len;
    atomic_store(&r->received, have + (uint32_t)got);
  }
  return NULL;
}

static void* ptx_loop(void* arg) {
  ptx_t* T = (ptx_t*)arg;
  stripe_t* S = T->S;
  struct mmsghdr msgs[256];
  struct iovec iov[256];
  const uint32_t total = T->n / (uint32_t)T->K, m = T->cs / (uint32_t)T->K;
  uint32_t sent = 0;
  double last_progress = now_s();
  while (sent < total) {
    const uint32_t ready = atomic_load(T->sealed) * m;  /* the stripe's packets sealed so far */
    const uint32_t inflight = sent - atomic_load(&S->R.received);
    if (sent >= ready || inflight + 256 > S->window) {
      if (now_s() - last_progress > 1.0) break; /* sealer or receiver stalled */
      sched_yield();                             /* the CPUs belong to the crypto and the sockets */
      continue;
    }
    last_progress = now_s();
    uint32_t k = ready - sent < 256 ? ready - sent : 256;
    for (uint32_t j = 0; j < k; ++j) {
      iov[j].iov_base = S->tx + (size_t)ppos(sent + j, T->k, T->K, T->cs) * UDP_STRIDE;
      iov[j].iov_len = HDR + S->L + 16;
      memset(&msgs[j].msg_hdr, 0, sizeof msgs[j].msg_hdr);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
      msgs[j].msg_hdr.msg_name = &S->addr;
      msgs[j].msg_hdr.msg_namelen = sizeof S->addr;
    }
    const int got = sendmmsg(S->tx_sock, msgs, k, 0);
    if (got > 0) sent += (uint32_t)got;
  }
  S->sent = sent;
  return NULL;
}

typedef struct {
  backend* B;
  stripe_t* SS;
  int K;
  uint32_t n, cs, C, L;
  uint64_t ctr;
  uint8_t *rxr, *back;
  uint32_t* lens;
  wg_pkt* od;
  uint32_t* st;
  double t_open;    /* time inside do_open */
  uint32_t opened;  /* packets opened */
  int failed;
} popen_t;

static void* popen_loop(void* arg) {
  popen_t* O = (popen_t*)arg;
  const uint32_t m = O->cs / (uint32_t)O->K;
  for (uint32_t c = 0; c < O->C; ++c) {
    const double w0 = now_s();
    for (int k = 0; k < O->K; ++k)  /* every stripe's share of chunk c has arrived */
      while (atomic_load(&O->SS[k].R.received) < (c + 1) * m) {
        if (now_s() - w0 > 2.0) return NULL; /* dropped datagrams: the chunk never completes */
        sched_yield();
      }
    uint32_t got = 0;
    for (uint32_t i = 0; i < O->cs; ++i) {
      const uint32_t pos = c * O->cs + i;
      const uint8_t* h = O->rxr + (size_t)pos * UDP_STRIDE;
      uint64_t cc;
      memcpy(&cc, h + 8, 8);
      const uint32_t idx = (uint32_t)(cc - O->ctr);
      O->od[pos] = (wg_pkt){(uint64_t)pos * UDP_STRIDE + HDR, (uint64_t)(idx < O->n ? idx : 0) * TUN_STRIDE, cc,
                            O->lens[pos] >= HDR + 16 ? O->lens[pos] - HDR - 16 : 0, 0};
      ++got;
    }
    const double a = now_s();
    if (do_open(O->B, O->od + (size_t)c * O->cs, got, O->rxr, (uint64_t)O->n * UDP_STRIDE, O->back,
                (uint64_t)O->n * TUN_STRIDE, O->st + (size_t)c * O->cs, O->L) != 0) {
      O->failed = 1;
      return NULL;
    }
    O->t_open += now_s() - a;
    O->opened += got;
  }
  return NULL;
}

int main(int argc, char** argv) {
  const char* bk = "gpu";
  const char* oracle_path = NULL;
  uint32_t n = 65536, L = 1420, reps = 5;
  int threads = 16, try_tun = 0, streams = 1;
  uint32_t chunks = 1;
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--tun")) try_tun = 1;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--tun")) { --i; continue; }
    if (!strcmp(argv[i], "--backend")) bk = argv[i + 1];
    else if (!strcmp(argv[i], "--oracle")) oracle_path = argv[i + 1];
    else if (!strcmp(argv[i], "--threads")) threads = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--packets")) n = (uint32_t)atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--len")) L = (uint32_t)atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--reps")) reps = (uint32_t)atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--udp-streams")) streams = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--chunks")) chunks = (uint32_t)atoi(argv[i + 1]);
  }
  if (chunks < 1 || n % chunks || (n / chunks) % (uint32_t)(streams > 0 ? streams : 1)) {
    fprintf(stderr, "--chunks must divide --packets into chunks that --udp-streams divides\n");
    return 2;
  }
  if (L < 28 || L > 1420 || n == 0 || reps == 0 || streams < 1 || streams > 64) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  backend B = {0};
  B.threads = threads;
  uint64_t ks = 0xC0FFEE;
  for (int i = 0; i < 32; ++i) B.keys[i] = (uint8_t)splitmix(&ks);
  if (!strcmp(bk, "gpu")) {
    B.gpu = 1;
    if (wg_ctx_create(0, 1, &B.ctx) != WG_OK || wg_keys_set(B.ctx, 0, 1, B.keys) != WG_OK) {
      fprintf(stderr, "libwgaead: %s\n", wg_last_error());
      return 1;
    }
  } else {
    void* h = oracle_path ? dlopen(oracle_path, RTLD_NOW) : NULL;
    if (!h) {
      fprintf(stderr, "cpu backend needs --oracle PATH to liboracle.so (%s)\n", dlerror());
      return 1;
    }
    B.o_seal = dlsym(h, "oracle_seal_batch");
    B.o_open = dlsym(h, "oracle_open_batch");
    if (!B.o_seal || !B.o_open) return 1;
  }
  uint8_t* tun = ring_alloc(&B, (size_t)n * TUN_STRIDE);
  uint8_t* tx = ring_alloc(&B, (size_t)n * UDP_STRIDE);
  uint8_t* rxr = ring_alloc(&B, (size_t)n * UDP_STRIDE);
  uint8_t* back = ring_alloc(&B, (size_t)n * TUN_STRIDE);
  wg_pkt* sd = calloc(n, sizeof(wg_pkt));
  wg_pkt* od = calloc(n, sizeof(wg_pkt));
  uint32_t* st = calloc(n, sizeof(uint32_t));
  uint32_t* lens = calloc(n, sizeof(uint32_t));
  if (!tun || !tx || !rxr || !back || !sd || !od || !st || !lens) {
    fprintf(stderr, "allocation failed\n");
    return 1;
  }
  double tun_rate = 0;
  if (!try_tun) snprintf(g_tun_note, sizeof g_tun_note, "not attempted (no --tun)");
  if (!try_tun || tun_fill(tun, n, L, &tun_rate) != 0) {  /* synthetic IPv4 packets */
    uint64_t s = 0x5EED2026;
    for (size_t i = 0; i < (size_t)n * TUN_STRIDE; ++i) tun[i] = (uint8_t)splitmix(&s);
    for (uint32_t i = 0; i < n; ++i) tun[(size_t)i * TUN_STRIDE] = 0x45;
  }
  /* loopback UDP: `streams` socket pairs, each with a sender and a receiver thread over its
   * share of the batch (one flow per socket, as several peers' sessions would be) */
  stripe_t* SS = calloc((size_t)streams, sizeof(stripe_t));
  int rcvbuf = 0;
  for (int k = 0; k < streams; ++k) {
    stripe_t* S = &SS[k];
    S->tx_sock = socket(AF_INET, SOCK_DGRAM, 0);
    S->R.sock = socket(AF_INET, SOCK_DGRAM, 0);
    int big = 64 << 20;
    setsockopt(S->R.sock, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(S->tx_sock, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    socklen_t rl = sizeof rcvbuf;
    getsockopt(S->R.sock, SOL_SOCKET, SO_RCVBUF, &rcvbuf, &rl);
    S->addr.sin_family = AF_INET;
    inet_pton(AF_INET, "127.0.0.1", &S->addr.sin_addr);
    if (bind(S->R.sock, (struct sockaddr*)&S->addr, sizeof S->addr) != 0) return 1;
    socklen_t al = sizeof S->addr;
    getsockname(S->R.sock, (struct sockaddr*)&S->addr, &al);
    S->lo = (uint32_t)((uint64_t)n * k / streams);
    S->hi = (uint32_t)((uint64_t)n * (k + 1) / streams);
    S->L = L;
    S->tx = tx;
    /* datagrams in flight at most ~half the receive buffer (loopback UDP drops, not blocks) */
    S->window = (uint32_t)(rcvbuf / 2 / (int)(UDP_STRIDE + 512));
    if (S->window < 16) S->window = 16;
  }
  const uint32_t window = SS[0].window;

  double t_seal = 0, t_xfer = 0, t_open = 0, t_total = 0;
  uint64_t delivered = 0, dropped = 0, bad = 0, mismatched = 0;
  uint64_t ctr = 0;
  const uint32_t cs = n / chunks;
  for (uint32_t rep = 0; chunks > 1 && rep <= reps; ++rep) { /* pipelined; rep 0: warm-up */
    _Atomic uint32_t sealed = 0;
    pthread_t rth[64], tth[64], oth;
    prx_t PR[64];
    ptx_t PT[64];
    popen_t O = {&B, SS, streams, n, cs, chunks, L, ctr, rxr, back, lens, od, st, 0.0, 0u, 0};
    memset(lens, 0, sizeof(uint32_t) * n);
    const double a = now_s();
    for (int k = 0; k < streams; ++k) {
      stripe_t* S = &SS[k];
      S->R.n = n / (uint32_t)streams;
      atomic_store(&S->R.received, 0);
      atomic_store(&S->R.stop, 0);
      PR[k] = (prx_t){&S->R, k, streams, cs, rxr, lens};
      PT[k] = (ptx_t){S, k, streams, n, cs, chunks, &sealed};
      pthread_create(&rth[k], NULL, prx_loop, &PR[k]);
      pthread_create(&tth[k], NULL, ptx_loop, &PT[k]);
    }
    pthread_create(&oth, NULL, popen_loop, &O);
    double ts = 0;
    for (uint32_t c = 0; c < chunks; ++c) {
      for (uint32_t i = c * cs; i < (c + 1) * cs; ++i) {
        uint8_t* h = tx + (size_t)i * UDP_STRIDE;
        const uint32_t type = 4, rcv = 0x01020304u;
        const uint64_t cc = ctr + i;
        memcpy(h, &type, 4); memcpy(h + 4, &rcv, 4); memcpy(h + 8, &cc, 8);
        sd[i] = (wg_pkt){(uint64_t)i * TUN_STRIDE, (uint64_t)i * UDP_STRIDE + HDR, cc, L, 0};
      }
      const double s0 = now_s();
      if (do_seal(&B, sd + (size_t)c * cs, cs, tun, (uint64_t)n * TUN_STRIDE, tx, (uint64_t)n * UDP_STRIDE, L) != 0) {
        fprintf(stderr, "seal failed: %s\n", B.gpu ? wg_last_error() : "");
        return 1;
      }
      ts += now_s() - s0;
      atomic_store(&sealed, c + 1);
    }
    for (int k = 0; k < streams; ++k) pthread_join(tth[k], NULL);
    pthread_join(oth, NULL);
    for (int k = 0; k < streams; ++k) {
      atomic_store(&SS[k].R.stop, 1);
      pthread_join(rth[k], NULL);
    }
    const double d = now_s();
    if (O.failed) {
      fprintf(stderr, "open failed: %s\n", B.gpu ? wg_last_error() : "");
      return 1;
    }
    if (rep > 0) {
      t_seal += ts;
      t_open += O.t_open;
      t_total += d - a;
      t_xfer += d - a;  /* the sockets run the whole time */
      delivered += O.opened;
      dropped += n - O.opened;
      for (uint32_t i = 0; i < O.opened; ++i) {
        if (st[i]) { ++bad; continue; }
        const uint32_t idx = (uint32_t)(od[i].counter - ctr);
        if (memcmp(back + (size_t)idx * TUN_STRIDE, tun + (size_t)idx * TUN_STRIDE, L)) ++mismatched;
      }
    }
    ctr += n;
  }
  for (uint32_t rep = 0; chunks == 1 && rep <= reps; ++rep) { /* rep 0: warm-up */
    const double a = now_s();
    for (uint32_t i = 0; i < n; ++i) {
      uint8_t* h = tx + (size_t)i * UDP_STRIDE;
      const uint32_t type = 4, rcv = 0x01020304u;
      const uint64_t c = ctr + i;
      memcpy(h, &type, 4); memcpy(h + 4, &rcv, 4); memcpy(h + 8, &c, 8);
      sd[i] = (wg_pkt){(uint64_t)i * TUN_STRIDE, (uint64_t)i * UDP_STRIDE + HDR, c, L, 0};
    }
    if (do_seal(&B, sd, n, tun, (uint64_t)n * TUN_STRIDE, tx, (uint64_t)n * UDP_STRIDE, L) != 0) {
      fprintf(stderr, "seal failed: %s\n", B.gpu ? wg_last_error() : "");
      return 1;
    }
    const double b = now_s();
    pthread_t rth[64], tth[64];
    for (int k = 0; k < streams; ++k) {
      stripe_t* S = &SS[k];
      S->R.ring = rxr + (size_t)S->lo * UDP_STRIDE;
      S->R.lens = lens + S->lo;
      S->R.n = S->hi - S->lo;
      atomic_store(&S->R.received, 0);
      atomic_store(&S->R.stop, 0);
      pthread_create(&rth[k], NULL, rx_loop, &S->R);
      pthread_create(&tth[k], NULL, tx_loop, S);
    }
    for (int k = 0; k < streams; ++k) pthread_join(tth[k], NULL);
    const double t_wait = now_s();
    for (int k = 0; k < streams; ++k) {
      while (atomic_load(&SS[k].R.received) < SS[k].sent && now_s() - t_wait < 0.5) {
      }
      atomic_store(&SS[k].R.stop, 1);
      pthread_join(rth[k], NULL);
    }
    /* open what arrived: header -> counter, descriptor into the received ring */
    uint32_t got = 0;
    for (int k = 0; k < streams; ++k) {
      const uint32_t gk = atomic_load(&SS[k].R.received);
      for (uint32_t i = 0; i < gk; ++i) {
        const uint32_t pos = SS[k].lo + i;
        const uint8_t* h = rxr + (size_t)pos * UDP_STRIDE;
        uint64_t cc;
        memcpy(&cc, h + 8, 8);
        const uint32_t idx = (uint32_t)(cc - ctr);
        od[got++] = (wg_pkt){(uint64_t)pos * UDP_STRIDE + HDR, (uint64_t)(idx < n ? idx : 0) * TUN_STRIDE, cc,
                             lens[pos] >= HDR + 16 ? lens[pos] - HDR - 16 : 0, 0};
      }
    }
    const double c2 = now_s();
    if (got && do_open(&B, od, got, rxr, (uint64_t)n * UDP_STRIDE, back, (uint64_t)n * TUN_STRIDE, st, L) != 0) {
      fprintf(stderr, "open failed: %s\n", B.gpu ? wg_last_error() : "");
      return 1;
    }
    const double d = now_s();
    if (rep > 0) {
      t_seal += b - a;
      t_xfer += c2 - b;
      t_open += d - c2;
      t_total += d - a;
      delivered += got;
      dropped += n - got;
      for (uint32_t i = 0; i < got; ++i) {
        if (st[i]) { ++bad; continue; }
        const uint32_t idx = (uint32_t)(od[i].counter - ctr);
        if (memcmp(back + (size_t)idx * TUN_STRIDE, tun + (size_t)idx * TUN_STRIDE, L)) ++mismatched;
      }
    }
    ctr += n;
  }
  const double GiB = (double)(1u << 30), per = (double)n * L;
  printf("{\"tool\": \"host_pipeline\", \"mode\": \"%s\", \"chunks\": %u, \"backend\": \"%s\", \"threads\": %d, \"packets\": %u, \"len\": %u, "
         "\"reps\": %u, \"udp_streams\": %d, \"tun\": \"%s\", \"tun_read_gib_s\": %.3f, \"udp_rcvbuf\": %d, \"inflight_window\": %u, "
         "\"seal_gib_s\": %.3f, \"udp_loopback_gib_s\": %.3f, \"open_gib_s\": %.3f, "
         "\"end_to_end_gib_s\": %.3f, \"delivered\": %llu, \"dropped\": %llu, \"bad_tag\": %llu, "
         "\"mismatched\": %llu}\n",
         chunks > 1 ? "pipelined" : "stages in turn", chunks, bk, B.gpu ? 0 : threads, n, L, reps, streams, g_tun_note, tun_rate, rcvbuf, window, per * reps / t_seal / GiB,
         (double)delivered * L / t_xfer / GiB, (double)delivered * L / t_open / GiB,
         (double)delivered * L / t_total / GiB, (unsigned long long)delivered, (unsigned long long)dropped,
         (unsigned long long)bad, (unsigned long long)mismatched);
  if (B.gpu) {
    void* rings[4] = {tun, tx, rxr, back};
    for (int k = 0; k < 4; ++k) wg_host_free(B.ctx, rings[k]);
    wg_ctx_destroy(B.ctx);
  }
  return (bad || mismatched) ? 3 : 0;
}
