// Round-7 probe: does ChaCha20 issue faster with more independent quarter-round
// chains per wave? One lane computes NB interleaved 64-byte blocks (4*NB independent
// QR chains per half-round) at 2/4/8 waves per SIMD; no memory traffic.
// Build: hipcc --offload-arch=gfx950 -O3 -I wireguard-java_amd/csrc -o tools/microbench7 tools/microbench7.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "wg_device.h"

#define QR(a, b, c, d)                       \
  a += b; d ^= a; d = wgd::rotl16(d);        \
  c += d; b ^= c; b = wgd::rotl(b, 12);      \
  a += b; d ^= a; d = wgd::rotl8(d);         \
  c += d; b ^= c; b = wgd::rotl(b, 7);

template <int NB>
__device__ __forceinline__ uint32_t blocks(const uint32_t k[8], uint32_t ctr, uint32_t n0) {
  uint32_t x[NB][16];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    x[q][0] = 0x61707865u; x[q][1] = 0x3320646eu; x[q][2] = 0x79622d32u; x[q][3] = 0x6b206574u;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[q][4 + i] = k[i];
    x[q][12] = ctr + q; x[q][13] = n0; x[q][14] = 0; x[q][15] = 0;
  }
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      QR(x[q][0], x[q][4], x[q][8], x[q][12]) QR(x[q][1], x[q][5], x[q][9], x[q][13])
      QR(x[q][2], x[q][6], x[q][10], x[q][14]) QR(x[q][3], x[q][7], x[q][11], x[q][15])
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      QR(x[q][0], x[q][5], x[q][10], x[q][15]) QR(x[q][1], x[q][6], x[q][11], x[q][12])
      QR(x[q][2], x[q][7], x[q][8], x[q][13]) QR(x[q][3], x[q][4], x[q][9], x[q][14])
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int q = 0; q < NB; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[q][i] + (i >= 4 && i < 12 ? k[i - 4] : (uint32_t)i);
  return acc;
}

template <int NB, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
k_chacha(uint32_t* out, uint32_t seed, int iters) {
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = seed * (i + 3) + threadIdx.x;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) acc ^= blocks<NB>(k, blockIdx.x * 65536u + threadIdx.x * 64u + it * NB, seed);
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static float time_kernel(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

template <int NB, int WPE>
void run(int cus, uint32_t* d, int wps) {
  const int blocks_ = cus * wps, iters = 256 / NB;
  float ms = time_kernel([&] { hipLaunchKernelGGL((k_chacha<NB, WPE>), dim3(blocks_), dim3(256), 0, 0, d, 7u, iters); }, 5);
  double nblk = (double)blocks_ * 256 * iters * NB;
  printf("NB=%d %d waves/SIMD: %.3f ms  %.3f G blocks/s = %.0f GiB/s keystream  %.0f cyc/wave-block@2.4GHz\n", NB, wps,
         ms, nblk / (ms * 1e-3) / 1e9, nblk * 64 / (ms * 1e-3) / (1u << 30),
         ms * 1e-3 * 2.4e9 / (nblk / 64 / (cus * 4)));
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  uint32_t* d; (void)hipMalloc(&d, 64);
  const int cus = prop.multiProcessorCount;
  run<1, 8>(cus, d, 8); run<1, 4>(cus, d, 4); run<1, 2>(cus, d, 2);
  run<2, 8>(cus, d, 8); run<2, 4>(cus, d, 4); run<2, 2>(cus, d, 2);
  run<4, 4>(cus, d, 4); run<4, 2>(cus, d, 2);
  return 0;
}
