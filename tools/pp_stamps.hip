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

int main(int argc, char** argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 1420;
  const int N = 2000;
  wg_ctx* c;
  if (wg_ctx_create(0, 1, &c) != WG_OK) return 1;
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 13 + 1);
  wg_keys_set(c, 0, 1, key);
  std::vector<uint8_t> pt(L + 16, 7), ct(L + 16), back(L + 16);
  std::vector<double> lat(N);
  for (int i = 0; i < N; ++i) {
    const double t0 = now_us();
    if (wg_seal1(c, 0, (uint64_t)i, pt.data(), L, ct.data()) != WG_OK) return 2;
    lat[i] = now_us() - t0;
  }
  std::vector<uint64_t> st(4096 * 8);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(wgpp::g_pp_stamps), st.size() * 8);
  const char* names[] = {"seen->prefix loaded", "->payload loaded", "->chacha+xor", "->poly tag", "->stores issued",
                         "->stores acked"};
  printf("{\"len\": %u, \"calls\": %d, \"host_p50_us\": %.2f", L, N, [&] {
    std::vector<double> v(lat.begin() + 100, lat.end());
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  }());
  for (int k = 0; k < 6; ++k) {
    std::vector<double> d;
    for (int i = 100; i < N; ++i) d.push_back((double)(st[(size_t)i * 8 + k + 1] - st[(size_t)i * 8 + k]) * 0.01);
    std::sort(d.begin(), d.end());
    printf(", \"%s_us\": %.2f", names[k], d[d.size() / 2]);
  }
  {
    std::vector<double> d;  // gap between one ticket's ack and the next ticket's seq seen (host turnaround + poll)
    for (int i = 100; i < N - 1; ++i) d.push_back((double)(st[(size_t)(i + 1) * 8 + 0] - st[(size_t)i * 8 + 6]) * 0.01);
    std::sort(d.begin(), d.end());
    printf(", \"ack->next seen_us\": %.2f", d[d.size() / 2]);
  }
  printf("}\n");
  wg_ctx_destroy(c);
  return 0;
}
