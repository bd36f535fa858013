// Per-phase timing of the per-packet server (k_pp): the library compiled into this tool with
// WG_PP_STAMPS, one caller issuing wg_seal1 / wg_open1, and the device's s_memrealtime stamps
// per ticket (100 MHz) next to the host-measured call latency. Diagnostic only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DWG_PP_STAMPS -I../include -o pp_stamps pp_stamps.hip
#include "../wireguard-java_amd/csrc/wg_capi.hip"

#include <time.h>

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

// Medians over the calls of one kind (op = 0: seal, 1: open, -1: all) past the first 100; call i is
// ticket i + 1.
static void report(const std::vector<uint64_t>& st, const std::vector<double>& lat, int N, uint32_t L, int op,
                   int alt) {
  auto pick = [&](int i) { return i >= 100 && (op < 0 || (i & 1) == op); };
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  auto row = [&](int i) { return &st[(size_t)((i + 1) % 4096) * 10]; };
  std::vector<double> h;
  for (int i = 0; i < N; ++i)
    if (pick(i)) h.push_back(lat[i]);
  printf("{\"len\": %u, \"calls\": %d, \"op\": \"%s\", \"host_p50_us\": %.2f", L, N,
         op < 0 ? "seal" : op == 0 ? "seal (alternating)" : "open (alternating)", med(h));
  const char* names[] = {"seen->prefix loaded", "->payload loaded", "->chacha+xor", "->poly tag", "->stores issued",
                         "->stores acked"};
  for (int k = 0; k < 6; ++k) {
    std::vector<double> d;
    for (int i = 0; i < N; ++i)
      if (pick(i)) d.push_back((double)(row(i)[k + 1] - row(i)[k]) * 0.01);
    printf(", \"%s_us\": %.2f", names[k], med(d));
  }
  std::vector<double> d;  // from the previous ticket's completion to this ticket's doorbell seen (host turnaround + poll)
  for (int i = 1; i < N; ++i)
    if (pick(i)) d.push_back((double)(row(i)[0] - row(i - 1)[6]) * 0.01);
  printf(", \"prev ack->seen_us\": %.2f", med(d));
  std::vector<double> g;  // shader clock over the compute phases: s_memtime cycles / s_memrealtime time
  for (int i = 0; i < N; ++i) {
    const double us = (double)(row(i)[4] - row(i)[2]) * 0.01;
    if (pick(i) && us > 0) g.push_back((double)row(i)[7] / us * 1e-3);
  }
  printf(", \"compute_clock_ghz\": %.3f}\n", med(g));
  (void)alt;
}

// Per XCC of the serving unit (PP_BY_XCC=1; run with WG_PP_CLAIM_PER_CALL=1 so calls visit every
// unit): call count, host latency and the payload read's round trip, medians.
static void by_xcc(const std::vector<uint64_t>& st, const std::vector<double>& lat, int N) {
  for (uint32_t x = 0; x < 16; ++x) {
    std::vector<double> h, rd, ss;
    for (int i = 100; i < N; ++i) {
      const uint64_t* r = &st[(size_t)((i + 1) % 4096) * 10];
      if (r[8] != x) continue;
      h.push_back(lat[i]);
      rd.push_back((double)(r[1] - r[0]) * 0.01);
      ss.push_back((double)(r[6] - r[0]) * 0.01);
    }
    if (h.empty()) continue;
    std::sort(h.begin(), h.end());
    std::sort(rd.begin(), rd.end());
    std::sort(ss.begin(), ss.end());
    printf("{\"xcc\": %u, \"calls\": %zu, \"host_p50_us\": %.2f, \"prefix_read_us\": %.2f, \"device_service_us\": %.2f}\n", x,
           h.size(), h[h.size() / 2], rd[rd.size() / 2], ss[ss.size() / 2]);
  }
}

int main(int argc, char** argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 1420;
  const int alt = argc > 2 && !strcmp(argv[2], "alt");  // alternate seal and open (tools/batcher_bench's shape)
  const int N = 2000;
  {  // on the GPU's NUMA node, as tools/batcher_bench (PP_PIN=0: not)
    const char* pin = getenv("PP_PIN");
    const int node = wg_device_numa_node(0);
    char path[96], buf[4096];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE* f = (!pin || atoi(pin) != 0) && node >= 0 ? fopen(path, "r") : nullptr;
    if (f && fgets(buf, sizeof buf, f)) {
      cpu_set_t set;
      CPU_ZERO(&set);
      for (char* p = buf; *p && *p != '\n';) {
        char* e;
        const long a = strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        if (*e == '-') b = strtol(e + 1, &e, 10);
        for (long x = a; x <= b && x < CPU_SETSIZE; ++x) CPU_SET((int)x, &set);
        p = *e == ',' ? e + 1 : e;
      }
      sched_setaffinity(0, sizeof set, &set);
    }
    if (f) fclose(f);
  }
  wg_ctx* c;
  if (wg_ctx_create(0, 1, &c) != WG_OK) return 1;
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 13 + 1);
  wg_keys_set(c, 0, 1, key);
  std::vector<uint8_t> pt(L + 16, 7), ct(L + 16), back(L + 16);
  std::vector<double> lat(N);
  for (int i = 0; i < N; ++i) {
    const double t0 = now_us();
    if (alt && (i & 1)) {
      if (wg_open1(c, 0, (uint64_t)(i / 2), ct.data(), L, back.data()) != WG_OK) return 3;
    } else if (wg_seal1(c, 0, (uint64_t)(alt ? i / 2 : i), pt.data(), L, ct.data()) != WG_OK) {
      return 2;
    }
    lat[i] = now_us() - t0;
  }
  std::vector<uint64_t> st(4096 * 10);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(wgpp::g_pp_stamps), st.size() * 8);
  if (getenv("PP_BY_XCC")) by_xcc(st, lat, N);
  if (alt) {
    report(st, lat, N, L, 0, alt);
    report(st, lat, N, L, 1, alt);
  } else {
    report(st, lat, N, L, -1, alt);
  }
  wg_ctx_destroy(c);
  return 0;
}
