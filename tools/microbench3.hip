// Round-3 probe: ChaCha20 keystream XOR over a flat HBM buffer, one 64-byte block
// per lane, to separate compute from memory effects in the seal kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench3 tools/microbench3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "../wireguard-java_amd/csrc/wg_device.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

// MODE 0: keystream only (sink); 1: load before rounds, xor, store; 2: load after rounds
template <int MODE, int LB>
__global__ void __launch_bounds__(256, LB) k_xor(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t nblk,
                                                 uint32_t seed, uint32_t* sink) {
  uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  uint32_t key[8];
  for (int i = 0; i < 8; ++i) key[i] = seed * (i + 1);
  uint4 a0, a1, a2, a3;
  if (MODE == 1) { a0 = in[4 * b]; a1 = in[4 * b + 1]; a2 = in[4 * b + 2]; a3 = in[4 * b + 3]; }
  uint32_t ks[16];
  wgd::chacha20_block(key, b % 23 + 1, b / 23, 0, 0, ks);
  if (MODE == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= ks[i];
    if (acc == 0x12345678u) sink[0] = acc;
    return;
  }
  if (MODE == 2) { a0 = in[4 * b]; a1 = in[4 * b + 1]; a2 = in[4 * b + 2]; a3 = in[4 * b + 3]; }
  out[4 * b] = make_uint4(a0.x ^ ks[0], a0.y ^ ks[1], a0.z ^ ks[2], a0.w ^ ks[3]);
  out[4 * b + 1] = make_uint4(a1.x ^ ks[4], a1.y ^ ks[5], a1.z ^ ks[6], a1.w ^ ks[7]);
  out[4 * b + 2] = make_uint4(a2.x ^ ks[8], a2.y ^ ks[9], a2.z ^ ks[10], a2.w ^ ks[11]);
  out[4 * b + 3] = make_uint4(a3.x ^ ks[12], a3.y ^ ks[13], a3.z ^ ks[14], a3.w ^ ks[15]);
}

template <typename F>
static float time_kernel(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  launch(); launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const uint32_t nblk = 65536u * 23u;
  uint4 *in, *out; uint32_t* sink;
  CHECK(hipMalloc(&in, (size_t)nblk * 64)); CHECK(hipMalloc(&out, (size_t)nblk * 64)); CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(in, 3, (size_t)nblk * 64));
  dim3 g((nblk + 255) / 256), t(256);
#define RUN(M, LB, name) { float ms = time_kernel([&] { hipLaunchKernelGGL((k_xor<M, LB>), g, t, 0, 0, in, out, nblk, 7u, sink); }, 20); \
    printf("%-34s %8.2f us  %6.1f blocks/ns  %7.1f GB/s (r+w)\n", name, ms * 1e3, nblk / (ms * 1e6), 2.0 * nblk * 64 / (ms * 1e-3) / 1e9); }
  RUN(0, 1, "keystream only (lb1)");
  RUN(0, 2, "keystream only (lb2 waves/SIMD)");
  RUN(1, 1, "load-before + xor + store (lb1)");
  RUN(1, 2, "load-before + xor + store (lb2)");
  RUN(2, 1, "load-after + xor + store (lb1)");
  RUN(2, 2, "load-after + xor + store (lb2)");
  return 0;
}
