/* Asynchronous batch submission under the reference's caller shape (TransportManager.java:41,70-93,
 * 137-158; EstablishedSession.java:88-90): P producer threads (the ForkJoinPool workers) submit
 * 1420-B packets to a seal queue without waiting (wg_submit_seal); a forwarder thread (the UDP
 * worker, and the peer's receiving side) reaps the sealed packets and submits each ct||tag to an
 * open queue (wg_submit_open); a verifier thread (the tun writer) reaps the plaintexts, checks every
 * status and every byte against what the producer sealed, and gives the slots back.
 *
 * Build: make -C tools queue_bench
 * Run:   tools/queue_bench [producers=16] [packets_per_producer=200000] [len=1420|0 mixed 64..1500]
 *                          [max_batch=8192] [forwarders=1] [verifiers=1] [cpu_port=PATH] [fwd_batch=1]
 * cpu_port=oracle/liboracle.so: after the queue run, the CPU restatement of the reference's AEAD seals
 * and opens the SAME packets (lengths, keys, counters) on `producers` threads, in the same process and
 * run, so the line compares the queue with the CPU port on exactly this packet mix ("cpu_port_gib_s").
 * Output: one JSON line: seal+open payload GiB/s over the whole run (both directions' payload bytes,
 * as bench.py's cpu_baseline counts them), seal-side rate, latency percentiles per queue (submit ->
 * reap), batches per queue. Exit status 1 on any failed status or byte mismatch. */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>
#include <dlfcn.h>

#include "wgaead.h"

#define KEYS 64
#define RB 65536
static wg_ctx* g_ctx;
static wg_queue *g_qs, *g_qo;
static int g_P, g_N, g_len;
static uint8_t** g_rb;           /* per producer: random bytes the payloads are cut from */
static _Atomic uint64_t g_fwd, g_ver, g_bad;
static uint64_t g_total;
static double *g_lat_s, *g_lat_o; /* sampled latencies, us */
static _Atomic uint64_t g_ns, g_no;
#define LAT_SAMPLES (1u << 20)

static uint64_t now_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static uint32_t pkt_len(uint64_t user) {
  if (g_len) return (uint32_t)g_len;
  uint64_t s = user * 0x2545F4914F6CDD1Dull;
  return 64u + (uint32_t)(splitmix(&s) % 1437u);
}

/* payload of packet `user` = (producer t, index i): its 8-byte tag, then bytes of t's buffer */
static void fill(uint8_t* p, uint64_t user, uint32_t L) {
  const int t = (int)(user >> 40);
  const uint32_t i = (uint32_t)user;
  const uint32_t off = (i * 61u) % (RB - 1600u);
  memcpy(p, g_rb[t] + off, L);
  if (L >= 8) memcpy(p, &user, 8);
}

static void* producer(void* arg) {
  const int t = (int)(intptr_t)arg;
  uint8_t pt[1600];
  for (int i = 0; i < g_N; ++i) {
    const uint64_t user = ((uint64_t)t << 40) | (uint64_t)i;
    const uint32_t L = pkt_len(user);
    fill(pt, user, L);
    /* the counter: SymmetricKeypair's getAndAdd per session; one session per producer here */
    if (wg_submit_seal(g_qs, (uint32_t)t % KEYS, (uint64_t)i, pt, L, user) != WG_OK) {
      fprintf(stderr, "submit_seal: %s\n", wg_last_error());
      exit(1);
    }
  }
  return NULL;
}

static int g_fwd_batch; /* fwd_batch=1: the forwarder hands each reap's completions over in one wg_submit_open_n */

static void* forwarder(void* arg) {
  (void)arg;
  wg_completion c[1024];
  wg_submit sub[1024];
  while (atomic_load(&g_fwd) < g_total) {
    const int n = wg_reap(g_qs, c, 1024, 1000);
    if (n < 0) {
      fprintf(stderr, "reap seal: %s\n", wg_last_error());
      exit(1);
    }
    const uint64_t now = now_ns();
    const uint64_t j0 = atomic_fetch_add(&g_ns, (uint64_t)(n > 0 ? n : 0));
    for (int k = 0; k < n; ++k) {
      if (c[k].status != WG_PKT_OK) atomic_fetch_add(&g_bad, 1);
      if (j0 + k < LAT_SAMPLES) g_lat_s[j0 + k] = (now - c[k].submit_ns) * 1e-3;
      /* ct || tag as it would arrive at the peer */
      if (g_fwd_batch) {
        sub[k] = (wg_submit){c[k].user, c[k].counter, c[k].data, c[k].len, c[k].key_slot};
      } else if (wg_submit_open(g_qo, c[k].key_slot, c[k].counter, c[k].data, c[k].len, c[k].user) != WG_OK) {
        fprintf(stderr, "submit_open: %s\n", wg_last_error());
        exit(1);
      }
    }
    if (g_fwd_batch && n > 0 && wg_submit_open_n(g_qo, sub, (uint32_t)n) != n) {  /* one call per reap */
      fprintf(stderr, "submit_open_n: %s\n", wg_last_error());
      exit(1);
    }
    wg_reap_done(g_qs, c, (uint32_t)n);
    atomic_fetch_add(&g_fwd, (uint64_t)n);
  }
  return NULL;
}

static void* verifier(void* arg) {
  (void)arg;
  wg_completion c[1024];
  uint8_t want[1600];
  while (atomic_load(&g_ver) < g_total) {
    const int n = wg_reap(g_qo, c, 1024, 1000);
    if (n < 0) {
      fprintf(stderr, "reap open: %s\n", wg_last_error());
      exit(1);
    }
    const uint64_t now = now_ns();
    const uint64_t j0 = atomic_fetch_add(&g_no, (uint64_t)(n > 0 ? n : 0));
    for (int k = 0; k < n; ++k) {
      /* a consumer of GPU-written completions prefetches a few ahead (as wg_submit_*_n does) */
      if (k + 2 < n)
        for (uint32_t o = 0; o < c[k + 2].len; o += 64) __builtin_prefetch(c[k + 2].data + o, 0, 0);
      if (j0 + k < LAT_SAMPLES) g_lat_o[j0 + k] = (now - c[k].submit_ns) * 1e-3;
      fill(want, c[k].user, c[k].len);
      if (c[k].status != WG_PKT_OK || c[k].len != pkt_len(c[k].user) || memcmp(c[k].data, want, c[k].len) != 0)
        atomic_fetch_add(&g_bad, 1);
    }
    wg_reap_done(g_qo, c, (uint32_t)n);
    atomic_fetch_add(&g_ver, (uint64_t)n);
  }
  return NULL;
}

/* the cgroup's CPU throttling counters (cgroup v2 cpu.stat), 0 where absent: the GPU box allows 16
 * CPUs to a process that may run on all of them, and a run that exceeds the quota stalls every thread */
static void throttled(unsigned long long* periods, unsigned long long* usec) {
  *periods = *usec = 0;
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return;
  char k[64];
  unsigned long long v;
  while (fscanf(f, "%63s %llu", k, &v) == 2) {
    if (!strcmp(k, "nr_throttled")) *periods = v;
    if (!strcmp(k, "throttled_usec")) *usec = v;
  }
  fclose(f);
}

static double cpu_seconds(void) {
  struct rusage r;
  getrusage(RUSAGE_SELF, &r);
  return r.ru_utime.tv_sec + r.ru_stime.tv_sec + 1e-6 * (r.ru_utime.tv_usec + r.ru_stime.tv_usec);
}

/* the CPUs of NUMA node `node` from sysfs ("0-63,128-191"); 0 if unreadable */
static int node_cpus(int node, cpu_set_t* set) {
  char path[96], buf[4096];
  if (node < 0) return 0;
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  const int ok = fgets(buf, sizeof buf, f) != NULL;
  fclose(f);
  if (!ok) return 0;
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
  return n;
}

static int cmpd(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

static void pct(double* v, uint64_t n, double out[4]) {
  if (n == 0) {
    out[0] = out[1] = out[2] = out[3] = 0;
    return;
  }
  qsort(v, n, sizeof(double), cmpd);
  out[0] = v[n / 2];
  out[1] = v[n * 99 / 100];
  out[2] = v[n * 999 / 1000];
  out[3] = v[n - 1];
}

int main(int argc, char** argv) {
  g_P = argc > 1 ? atoi(argv[1]) : 16;
  g_N = argc > 2 ? atoi(argv[2]) : 200000;
  g_len = argc > 3 ? atoi(argv[3]) : 1420;
  const int max_batch = argc > 4 ? atoi(argv[4]) : 8192;
  const int nf = argc > 5 ? atoi(argv[5]) : 1, nv = argc > 6 ? atoi(argv[6]) : 1;
  const char* cpu_port = NULL;
  for (int a = 1; a < argc; ++a) {
    if (!strncmp(argv[a], "cpu_port=", 9)) cpu_port = argv[a] + 9;
    if (!strncmp(argv[a], "fwd_batch=", 10)) g_fwd_batch = atoi(argv[a] + 10);
  }
  if (g_P < 1 || g_P > 256 || g_N < 1 || g_len < 0 || g_len > 1500) {
    fprintf(stderr, "usage: queue_bench [producers] [packets_per_producer] [len 0..1500] [max_batch]\n");
    return 2;
  }
  /* every thread on the GPU's NUMA node (as numactl --cpunodebind would place a TransportManager's
   * pools; QB_PIN=0: wherever the scheduler puts them), before the pinned rings are allocated */
  const char* pin = getenv("QB_PIN");
  const int node = wg_device_numa_node(0);
  cpu_set_t set;
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  int pinned = -1;
  if ((!pin || atoi(pin) != 0) && node_cpus(node, &set)) {
    pthread_attr_setaffinity_np(&attr, sizeof set, &set);
    pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    pinned = node;
  }
  if (wg_ctx_create(0, KEYS, &g_ctx) != WG_OK) {
    fprintf(stderr, "wg_ctx_create: %s\n", wg_last_error());
    return 1;
  }
  uint8_t keys[KEYS * 32];
  uint64_t ks = 11;
  for (int i = 0; i < KEYS * 32; ++i) keys[i] = (uint8_t)splitmix(&ks);
  if (wg_keys_set(g_ctx, 0, KEYS, keys) != WG_OK ||
      wg_queue_create(g_ctx, WG_MODE_SEAL, 65536, 1500, (uint32_t)max_batch, &g_qs) != WG_OK ||
      wg_queue_create(g_ctx, WG_MODE_OPEN, 65536, 1500, (uint32_t)max_batch, &g_qo) != WG_OK) {
    fprintf(stderr, "setup: %s\n", wg_last_error());
    return 1;
  }
  g_rb = calloc((size_t)g_P, sizeof(uint8_t*));
  for (int t = 0; t < g_P; ++t) {
    g_rb[t] = malloc(RB);
    uint64_t s = 1000 + (uint64_t)t;
    for (int i = 0; i < RB; ++i) g_rb[t][i] = (uint8_t)splitmix(&s);
  }
  g_lat_s = calloc(LAT_SAMPLES, sizeof(double));
  g_lat_o = calloc(LAT_SAMPLES, sizeof(double));
  g_total = (uint64_t)g_P * (uint64_t)g_N;
  uint64_t bytes = 0;
  for (int t = 0; t < g_P; ++t)
    for (int i = 0; i < g_N; ++i) bytes += pkt_len(((uint64_t)t << 40) | (uint64_t)i);

  if (nf < 1 || nf > 8 || nv < 1 || nv > 8) {
    fprintf(stderr, "forwarders / verifiers: 1..8\n");
    return 2;
  }
  pthread_t th[256 + 16];
  unsigned long long thp0, thu0, thp1, thu1;
  throttled(&thp0, &thu0);
  const double cpu0 = cpu_seconds();
  const uint64_t t0 = now_ns();
  for (int k = 0; k < nf; ++k) pthread_create(&th[g_P + k], &attr, forwarder, NULL);
  for (int k = 0; k < nv; ++k) pthread_create(&th[g_P + nf + k], &attr, verifier, NULL);
  for (int t = 0; t < g_P; ++t) pthread_create(&th[t], &attr, producer, (void*)(intptr_t)t);
  for (int t = 0; t < g_P; ++t) pthread_join(th[t], NULL);
  const double t_submit = (now_ns() - t0) * 1e-9;
  for (int k = 0; k < nf; ++k) pthread_join(th[g_P + k], NULL);
  const double t_sealed = (now_ns() - t0) * 1e-9;
  for (int k = 0; k < nv; ++k) pthread_join(th[g_P + nf + k], NULL);
  const double wall = (now_ns() - t0) * 1e-9;
  const double cpu = cpu_seconds() - cpu0;
  throttled(&thp1, &thu1);
  uint64_t bs = 0, ps = 0, bo = 0, po = 0;
  wg_queue_stats(g_qs, &bs, &ps);
  wg_queue_stats(g_qo, &bo, &po);
  const uint64_t ns = g_ns < LAT_SAMPLES ? g_ns : LAT_SAMPLES, no = g_no < LAT_SAMPLES ? g_no : LAT_SAMPLES;
  double ls[4], lo[4];
  pct(g_lat_s, ns, ls);
  pct(g_lat_o, no, lo);
  const double gib = (double)(1u << 30);
  /* the CPU port on the same packets: seal every packet, then open every ct || tag, producers threads */
  double cpu_port_gib_s = 0, cpu_port_s = 0;
  int cpu_port_ok = 1;
  if (cpu_port) {
    void* h = dlopen(cpu_port, RTLD_NOW);
    int (*o_seal)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, int) =
        h ? (int (*)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, int))dlsym(h, "oracle_seal_batch") : NULL;
    int (*o_open)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, uint32_t*, int) =
        h ? (int (*)(const wg_pkt*, size_t, const uint8_t*, uint8_t*, const uint8_t*, uint32_t*, int))dlsym(h, "oracle_open_batch") : NULL;
    if (!o_seal || !o_open) {
      fprintf(stderr, "cpu_port=%s: %s\n", cpu_port, dlerror());
      return 1;
    }
    /* a bounded sample of the same packets (at most 1M): user ids t << 40 | i, round robin over producers */
    const uint64_t n = g_total < (1u << 20) ? g_total : (1u << 20);
    wg_pkt* sd = calloc(n, sizeof(wg_pkt));
    wg_pkt* od = calloc(n, sizeof(wg_pkt));
    uint32_t* st = calloc(n, sizeof(uint32_t));
    uint64_t off = 0, cbytes = 0;
    for (uint64_t k = 0; k < n; ++k) {
      const uint64_t user = ((k % (uint64_t)g_P) << 40) | (k / (uint64_t)g_P);
      const uint32_t L = pkt_len(user);
      sd[k] = (wg_pkt){off, off, k / (uint64_t)g_P, L, (uint32_t)(k % (uint64_t)g_P) % KEYS};
      off += ((uint64_t)L + 16u + 15u) & ~15ull;
      cbytes += L;
    }
    uint8_t* pt = malloc(off), *ct = malloc(off), *back = malloc(off);
    for (uint64_t k = 0; k < n; ++k) fill(pt + sd[k].in_off, ((k % (uint64_t)g_P) << 40) | (k / (uint64_t)g_P), sd[k].len);
    memcpy(od, sd, n * sizeof(wg_pkt));
    const uint64_t c0 = now_ns();
    o_seal(sd, n, pt, ct, keys, g_P);
    o_open(od, n, ct, back, keys, st, g_P);
    cpu_port_s = (now_ns() - c0) * 1e-9;
    for (uint64_t k = 0; k < n; ++k)
      if (st[k] != WG_PKT_OK || memcmp(back + sd[k].in_off, pt + sd[k].in_off, sd[k].len) != 0) cpu_port_ok = 0;
    cpu_port_gib_s = 2.0 * cbytes / cpu_port_s / gib;
    free(sd); free(od); free(st); free(pt); free(ct); free(back);
  }
  char cpu_json[256] = "";
  if (cpu_port)
    snprintf(cpu_json, sizeof cpu_json, ", \"cpu_port_gib_s\": %.3f, \"cpu_port_threads\": %d, \"cpu_port_ok\": %d",
             cpu_port_gib_s, g_P, cpu_port_ok);
  printf("{\"tool\": \"queue_bench\", \"producers\": %d, \"forwarders\": %d, \"verifiers\": %d, \"packets\": %llu, \"len\": \"%s\", \"max_batch\": %d, "
         "\"bad\": %llu, \"wall_s\": %.4f, \"seal_open_gib_s\": %.3f, \"seal_gib_s\": %.3f, "
         "\"submit_gib_s\": %.3f, \"packets_per_s\": %.0f, "
         "\"seal_lat_us\": {\"p50\": %.1f, \"p99\": %.1f, \"p999\": %.1f, \"max\": %.1f}, "
         "\"open_lat_us\": {\"p50\": %.1f, \"p99\": %.1f, \"p999\": %.1f, \"max\": %.1f}, "
         "\"seal_batches\": %llu, \"seal_mean_batch\": %.1f, \"open_batches\": %llu, \"open_mean_batch\": %.1f, "
         "\"cpu_s\": %.3f, \"cpus_busy\": %.2f, \"throttled_periods\": %llu, \"throttled_ms\": %.1f, \"pinned_node\": %d, \"fwd_batch\": %d%s}\n",
         g_P, nf, nv, (unsigned long long)g_total, g_len ? argv[3] : "mixed 64..1500", max_batch,
         (unsigned long long)g_bad, wall, 2.0 * bytes / wall / gib, bytes / t_sealed / gib, bytes / t_submit / gib,
         g_total / wall, ls[0], ls[1], ls[2], ls[3], lo[0], lo[1], lo[2], lo[3], (unsigned long long)bs,
         bs ? (double)ps / bs : 0.0, (unsigned long long)bo, bo ? (double)po / bo : 0.0, cpu, cpu / wall,
         thp1 - thp0, (thu1 - thu0) * 1e-3, pinned, g_fwd_batch, cpu_json);
  wg_queue_destroy(g_qs);
  wg_queue_destroy(g_qo);
  wg_ctx_destroy(g_ctx);
  return (g_bad || !cpu_port_ok) ? 1 : 0;
}
