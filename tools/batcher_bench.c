/* Per-packet API under load: T caller threads each issue N wg_seal1 / wg_open1 calls
 * (alternating; each open takes the packet the thread just sealed, so every tag verifies),
 * the way the reference's ForkJoinPool workers call SymmetricKeypair.cipher / decipher one
 * packet at a time (TransportManager.java:41,79,152-158). Reports per-call latency
 * percentiles, the aggregate payload rate and the batcher's mean launch size.
 *
 * Build: gcc -O2 -pthread -Iinclude -o tools/batcher_bench tools/batcher_bench.c \
 *          -Lwireguard-java_amd -l:libwgaead.so -Wl,-rpath,'$ORIGIN/../wireguard-java_amd'
 * Run:   tools/batcher_bench [threads=16] [calls=10000] [len=1420|0 for mixed 64..1500] [key=value ...]
 *   gap_us=G        each caller sleeps G us between calls (a quiet tunnel: low call rate)
 *   hold_us=H       one extra caller, started 20 ms into the run, is held H us between claiming its
 *                   ring entry and publishing it (test hook WG_PP_TEST_HOLD_*: a caller descheduled
 *                   mid-call); its latency is reported apart ("held_us") from everyone else's
 *   fail_launches=F the first F server launches are refused (WG_PP_TEST_FAIL_LAUNCHES); the warm-up
 *                   call must fail, every timed call must then succeed
 *   waves=W idle_us=I  wg_pp_config before the first call
 *   stamps=1        after every call read its stages (wg_pp_last_call) and the thread's context
 *                   switches (getrusage RUSAGE_THREAD): the slowest call's breakdown goes into the
 *                   line ("slowest"), with the count of calls over 1 ms and how many of those were
 *                   preempted (an involuntary context switch during the call)
 * Output: one JSON line. */
#define _GNU_SOURCE
#include <pthread.h>
#include <sys/resource.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "wgaead.h"

static wg_ctx* g_ctx;
static int g_calls, g_len;
static double* g_lat;          /* [threads][calls] microseconds */
static uint64_t* g_bytes;      /* payload bytes per thread */
static int* g_fail;
static int g_gap_us;
#define HOLD_COUNTER 0x0D0D0D0D0D0Dull
static double g_held_us = -1.0;
static int g_held_rc = 0;
static int g_stamps;
static int g_pinned = -1; /* the NUMA node every thread runs on, -1: not pinned */
typedef struct {
  double lat_us;
  uint64_t st[8];   /* wg_pp_last_call */
  long nivcsw, nvcsw; /* context switches of the thread during the call */
  int op, thread;
} slow_t;
static slow_t* g_slowest;        /* per thread */
static double (*g_stage_sum)[5]; /* per thread: sums of claim, publish, wait, device service, copy-out (ns) */
static int* g_over1ms, *g_over1ms_preempted;

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void* worker(void* arg) {
  const int t = (int)(intptr_t)arg;
  uint64_t rs = 1000 + t;
  uint8_t pt[1500], ct[1516], back[1500];
  for (int i = 0; i < 1500; ++i) pt[i] = (uint8_t)splitmix(&rs);
  const uint32_t slot = (uint32_t)t % 64u;
  uint64_t ctr = (uint64_t)t << 40;
  uint32_t L = 0;
  for (int i = 0; i < g_calls; ++i) {
    struct rusage ru0, ru1;
    if (g_stamps) getrusage(RUSAGE_THREAD, &ru0);
    double t0 = now_us();
    int rc;
    if ((i & 1) == 0) {
      L = g_len ? (uint32_t)g_len : 64u + (uint32_t)(splitmix(&rs) % 1437u);
      rc = wg_seal1(g_ctx, slot, ctr, pt, L, ct);
    } else {
      rc = wg_open1(g_ctx, slot, ctr, ct, L, back);
      if (rc == 0 && memcmp(back, pt, L) != 0) rc = -100;
      ++ctr;
    }
    const double lat = now_us() - t0;
    g_lat[(size_t)t * g_calls + i] = lat;
    if (g_stamps) {
      uint64_t st[8];
      wg_pp_last_call(st, 8);
      getrusage(RUSAGE_THREAD, &ru1);
      const long niv = ru1.ru_nivcsw - ru0.ru_nivcsw, nv = ru1.ru_nvcsw - ru0.ru_nvcsw;
      if (lat > 1000.0) {
        ++g_over1ms[t];
        if (niv > 0) ++g_over1ms_preempted[t];
      }
      for (int k = 0; k < 5; ++k) g_stage_sum[t][k] += (double)st[k + 1];
      if (lat > g_slowest[t].lat_us) {
        g_slowest[t].lat_us = lat;
        memcpy(g_slowest[t].st, st, sizeof st);
        g_slowest[t].nivcsw = niv;
        g_slowest[t].nvcsw = nv;
        g_slowest[t].op = i & 1;
        g_slowest[t].thread = t;
      }
    }
    if (rc != 0) ++g_fail[t];
    g_bytes[t] += L;
    if (g_gap_us) {
      struct timespec ts = {g_gap_us / 1000000, (long)(g_gap_us % 1000000) * 1000};
      nanosleep(&ts, NULL);
    }
  }
  return NULL;
}

static void* held(void* arg) {
  (void)arg;
  struct timespec ts = {0, 20 * 1000 * 1000};
  nanosleep(&ts, NULL);
  uint8_t pt[1420], ct[1436];
  memset(pt, 0x5a, sizeof pt);
  double t0 = now_us();
  g_held_rc = wg_seal1(g_ctx, 1, HOLD_COUNTER, pt, sizeof pt, ct);
  g_held_us = now_us() - t0;
  return NULL;
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

/* the cgroup's throttled periods (cgroup v2 cpu.stat), 0 where absent: the GPU box allows the
 * process 16 CPUs of time while it may run on all of them */
static unsigned long long throttled_periods(void) {
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return 0;
  char k[64];
  unsigned long long v, r = 0;
  while (fscanf(f, "%63s %llu", k, &v) == 2)
    if (!strcmp(k, "nr_throttled")) r = v;
  fclose(f);
  return r;
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  g_calls = argc > 2 ? atoi(argv[2]) : 10000;
  g_len = argc > 3 ? atoi(argv[3]) : 1420;
  int hold_us = 0, fail_launches = 0, waves = 16, idle_us = 0;
  for (int a = 4; a < argc; ++a) {
    const char* v = strchr(argv[a], '=');
    if (!v) continue;
    const int x = atoi(v + 1);
    if (!strncmp(argv[a], "gap_us=", 7)) g_gap_us = x;
    else if (!strncmp(argv[a], "hold_us=", 8)) hold_us = x;
    else if (!strncmp(argv[a], "fail_launches=", 14)) fail_launches = x;
    else if (!strncmp(argv[a], "waves=", 6)) waves = x;
    else if (!strncmp(argv[a], "idle_us=", 8)) idle_us = x;
    else if (!strncmp(argv[a], "stamps=", 7)) g_stamps = x;
  }
  if (T < 1 || T > 1024 || g_calls < 2 || g_len < 0 || g_len > 1500) {
    fprintf(stderr, "usage: batcher_bench [threads] [calls] [len 0..1500] [gap_us= hold_us= fail_launches= waves= idle_us=]\n");
    return 2;
  }
  char buf[64];
  if (hold_us) {
    snprintf(buf, sizeof buf, "%llu", (unsigned long long)HOLD_COUNTER);
    setenv("WG_PP_TEST_HOLD_COUNTER", buf, 1);
    snprintf(buf, sizeof buf, "%d", hold_us);
    setenv("WG_PP_TEST_HOLD_US", buf, 1);
  }
  if (g_stamps) setenv("WG_PP_CALL_STAMPS", "1", 1);
  if (fail_launches) {
    snprintf(buf, sizeof buf, "%d", fail_launches);
    setenv("WG_PP_TEST_FAIL_LAUNCHES", buf, 1);
  }
  /* every thread on the GPU's NUMA node (BB_PIN=0: wherever the scheduler puts them), before the
   * context and its rings exist: a caller on the other socket adds a cross-socket snoop to every
   * device read of the payload it just wrote (about 0.7 us) and to its own completion polls */
  const char* pin = getenv("BB_PIN");
  cpu_set_t set;
  if ((!pin || atoi(pin) != 0) && node_cpus(wg_device_numa_node(0), &set)) {
    pthread_setaffinity_np(pthread_self(), sizeof set, &set);  /* threads created later inherit it */
    g_pinned = wg_device_numa_node(0);
  }
  if (wg_ctx_create(0, 64, &g_ctx) != WG_OK) {
    fprintf(stderr, "wg_ctx_create: %s\n", wg_last_error());
    return 1;
  }
  if (getenv("WG_BENCH_KERNEL") && wg_ctx_set_kernel(g_ctx, getenv("WG_BENCH_KERNEL"), 0, 0) != WG_OK) {
    fprintf(stderr, "wg_ctx_set_kernel: %s\n", wg_last_error());
    return 1;
  }
  uint8_t keys[64 * 32];
  uint64_t ks = 7;
  for (int i = 0; i < 64 * 32; ++i) keys[i] = (uint8_t)splitmix(&ks);
  wg_keys_set(g_ctx, 0, 64, keys);
  g_lat = calloc((size_t)T * g_calls, sizeof(double));
  g_bytes = calloc(T, sizeof(uint64_t));
  g_fail = calloc(T, sizeof(int));
  g_slowest = calloc(T, sizeof(slow_t));
  g_stage_sum = calloc(T, sizeof *g_stage_sum);
  g_over1ms = calloc(T, sizeof(int));
  g_over1ms_preempted = calloc(T, sizeof(int));
  pthread_t th[1024];
  if (wg_pp_config(g_ctx, (uint32_t)waves, (uint32_t)idle_us) != WG_OK) {
    fprintf(stderr, "wg_pp_config: %s\n", wg_last_error());
    return 1;
  }
  /* warm-up: one call, untimed (with fail_launches it must be refused) */
  int warm_rc;
  { uint8_t a[64], b[80]; memset(a, 1, 64); warm_rc = wg_seal1(g_ctx, 0, 1ull << 60, a, 64, b); }
  if (fail_launches ? warm_rc == 0 : warm_rc != 0) {
    fprintf(stderr, "warm-up call: rc %d (%s)\n", warm_rc, wg_last_error());
    return 1;
  }
  uint64_t l0 = 0, p0 = 0;
  wg_batcher_stats(g_ctx, &l0, &p0);
  const unsigned long long thr0 = throttled_periods();
  double t0 = now_us();
  pthread_t hth;
  if (hold_us) pthread_create(&hth, NULL, held, NULL);
  for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  if (hold_us) pthread_join(hth, NULL);
  double wall = now_us() - t0;
  const unsigned long long thr1 = throttled_periods();
  uint64_t l1 = 0, p1 = 0;
  wg_batcher_stats(g_ctx, &l1, &p1);
  size_t n = (size_t)T * g_calls;
  qsort(g_lat, n, sizeof(double), cmpd);
  uint64_t bytes = 0;
  int fails = 0;
  for (int t = 0; t < T; ++t) {
    bytes += g_bytes[t];
    fails += g_fail[t];
  }
  char slow[1024] = "";
  if (g_stamps) {
    int w = 0, o1 = 0, o1p = 0;
    for (int t = 0; t < T; ++t) {
      if (g_slowest[t].lat_us > g_slowest[w].lat_us) w = t;
      o1 += g_over1ms[t];
      o1p += g_over1ms_preempted[t];
    }
    const slow_t* x = &g_slowest[w];
    snprintf(slow, sizeof slow,
             ", \"slowest\": {\"lat_us\": %.1f, \"op\": \"%s\", \"thread\": %d, \"claim_us\": %.1f, "
             "\"publish_us\": %.1f, \"wait_us\": %.1f, \"device_service_us\": %.1f, \"copy_out_us\": %.1f, "
             "\"slept\": %llu, \"relaunched\": %llu, \"involuntary_csw\": %ld, \"voluntary_csw\": %ld}, "
             "\"calls_over_1ms\": %d, \"calls_over_1ms_preempted\": %d",
             x->lat_us, x->op ? "open" : "seal", x->thread, x->st[1] * 1e-3, x->st[2] * 1e-3, x->st[3] * 1e-3,
             x->st[4] * 1e-3, x->st[5] * 1e-3, (unsigned long long)x->st[6], (unsigned long long)x->st[7],
             x->nivcsw, x->nvcsw, o1, o1p);
    double m[5] = {0, 0, 0, 0, 0};
    for (int t = 0; t < T; ++t)
      for (int k = 0; k < 5; ++k) m[k] += g_stage_sum[t][k] / ((double)T * g_calls) * 1e-3;
    const size_t used = strlen(slow);
    snprintf(slow + used, sizeof slow - used,
             ", \"stage_mean_us\": {\"claim\": %.2f, \"publish\": %.2f, \"wait\": %.2f, \"device_service\": %.2f, "
             "\"copy_out\": %.2f}", m[0], m[1], m[2], m[3], m[4]);
  }
  printf("{\"tool\": \"batcher_bench\", \"threads\": %d, \"calls_per_thread\": %d, \"len\": \"%s\", "
         "\"calls\": %zu, \"failures\": %d, \"wall_s\": %.4f, \"calls_per_s\": %.0f, "
         "\"payload_gib_s\": %.4f, \"lat_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"p999\": %.1f, "
         "\"max\": %.1f}, \"launches\": %llu, \"mean_batch\": %.1f, \"gap_us\": %d, \"waves\": %d, "
         "\"fail_launches\": %d, \"hold_us\": %d, \"held_us\": %.1f, \"held_rc\": %d, \"throttled_periods\": %llu, "
         "\"pinned_node\": %d%s}\n",
         T, g_calls, g_len ? argv[3] : "mixed 64..1500", n, fails, wall * 1e-6, n / (wall * 1e-6),
         bytes / (wall * 1e-6) / (double)(1u << 30), g_lat[n / 2], g_lat[n * 9 / 10], g_lat[n * 99 / 100],
         g_lat[n * 999 / 1000], g_lat[n - 1], (unsigned long long)(l1 - l0),
         (l1 > l0) ? (double)(p1 - p0) / (double)(l1 - l0) : 0.0, g_gap_us, waves, fail_launches, hold_us,
         g_held_us, g_held_rc, thr1 - thr0, g_pinned, slow);
  wg_ctx_destroy(g_ctx);
  return (fails || g_held_rc) ? 1 : 0;
}
