// Instruction-rate and bandwidth probes for gfx950 (MI355X), used to size the
// seal/open kernels (DESIGN.md "Roofline"). Not part of the product library.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
// Run (GPU box): ./tools/microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// 8 independent chains of one op kind per lane; `asm volatile("" : "+v")` keeps
// every intermediate opaque so the compiler cannot fold the chain.
#define OPAQUE(x) asm volatile("" : "+v"(x))

__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b = seed ^ threadIdx.x;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = a[i] + b; OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_xor(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b = seed ^ threadIdx.x;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = a[i] ^ (b + it); OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_rot(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = __builtin_amdgcn_alignbit(a[i], a[i], 7); OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_perm(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = __builtin_amdgcn_perm(a[i], a[i], 0x01000302u); OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t a[8];
  uint32_t x = seed ^ threadIdx.x, y = seed * 3 + 1;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = (uint64_t)(uint32_t)a[i] * y + a[i]; OPAQUE(a[i]); }
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = (uint32_t)r;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b = seed | 1u;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = a[i] * b; OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_mul24(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b = (seed | 1u) & 0xffffff;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = __umul24(a[i], b) ; OPAQUE(a[i]); }
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}

__global__ void k_fma64(double* out, double seed) {
  double a[8], b = seed * 0.5;
  for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = __builtin_fma(a[i], b, seed); OPAQUE(a[i]); }
  }
  double r = 0; for (int i = 0; i < 8; ++i) r += a[i];
  if (r == 1.2345) out[0] = r;
}

// ChaCha20 block function, register-only: measures the pure-VALU keystream ceiling.
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define QR(a, b, c, d) \
  a += b; d ^= a; d = rotl(d, 16); \
  c += d; b ^= c; b = rotl(b, 12); \
  a += b; d ^= a; d = rotl(d, 8);  \
  c += d; b ^= c; b = rotl(b, 7);

__global__ void k_chacha(uint32_t* out, uint32_t seed, int nblocks) {
  uint32_t acc = 0;
  uint32_t k0 = seed, k1 = seed * 3, k2 = seed * 5, k3 = seed * 7;
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
    uint32_t x4 = k0, x5 = k1, x6 = k2, x7 = k3, x8 = k0 ^ 1, x9 = k1 ^ 2, x10 = k2 ^ 3, x11 = k3 ^ 4;
    uint32_t x12 = blk + threadIdx.x, x13 = blockIdx.x, x14 = 0, x15 = 0;
    OPAQUE(x4);
    for (int r = 0; r < 10; ++r) {
      QR(x0, x4, x8, x12); QR(x1, x5, x9, x13); QR(x2, x6, x10, x14); QR(x3, x7, x11, x15);
      QR(x0, x5, x10, x15); QR(x1, x6, x11, x12); QR(x2, x7, x8, x13); QR(x3, x4, x9, x14);
    }
    acc ^= x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

// Lane-per-64B-block access pattern (4 x dwordx4 at 64-B lane stride) vs coalesced.
__global__ void k_copy_strided64(const uint4* __restrict__ in, uint4* __restrict__ out, size_t nblk) {
  size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; b < nblk; b += stride) {
    uint4 v0 = in[4 * b + 0], v1 = in[4 * b + 1], v2 = in[4 * b + 2], v3 = in[4 * b + 3];
    out[4 * b + 0] = v0; out[4 * b + 1] = v1; out[4 * b + 2] = v2; out[4 * b + 3] = v3;
  }
}

template <typename F>
static float time_kernel(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a); hipEventDestroy(b);
  return ms / reps;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  uint32_t* d; CHECK(hipMalloc(&d, 64));
  double* dd; CHECK(hipMalloc(&dd, 64));
  const int blocks = prop.multiProcessorCount * 8, tpb = 256;
  const double lane_ops = (double)blocks * tpb * ITERS * 8;
  struct { const char* name; void (*k)(uint32_t*, uint32_t); } ks[] = {
    {"v_add_u32", k_add}, {"v_xor_b32(+add)", k_xor}, {"v_alignbit_b32", k_rot}, {"v_perm_b32", k_perm},
    {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_u32_u24(+and)", k_mul24}};
  for (auto& k : ks) {
    float ms = time_kernel([&] { hipLaunchKernelGGL(k.k, dim3(blocks), dim3(tpb), 0, 0, d, 12345u); }, 5);
    printf("%-22s %8.3f ms  %7.2f T lane-ops/s\n", k.name, ms, lane_ops / (ms * 1e-3) / 1e12);
  }
  {
    float ms = time_kernel([&] { hipLaunchKernelGGL(k_fma64, dim3(blocks), dim3(tpb), 0, 0, dd, 1.5); }, 5);
    printf("%-22s %8.3f ms  %7.2f T lane-ops/s\n", "v_fma_f64", ms, lane_ops / (ms * 1e-3) / 1e12);
  }
  for (int wpc : {4, 8, 16}) {
    const int nb = 64;
    int cb = prop.multiProcessorCount * wpc / 4;
    float ms = time_kernel([&] { hipLaunchKernelGGL(k_chacha, dim3(cb), dim3(256), 0, 0, d, 777u, nb); }, 5);
    double bytes = (double)cb * 256 * nb * 64;
    printf("chacha20 keystream (%2d waves/CU): %8.3f ms  %8.1f GB/s  (%.1f blocks/ns)\n", wpc, ms, bytes / (ms * 1e-3) / 1e9,
           bytes / 64 / (ms * 1e6));
  }
  {
    size_t bytes = (size_t)1 << 30;
    uint4 *a, *b;
    CHECK(hipMalloc(&a, bytes)); CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 1, bytes)); CHECK(hipMemset(b, 0, bytes));
    size_t n = bytes / 16;
    for (int g : {1024, 2048, 4096, 8192}) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, a, b, n); }, 10);
      printf("copy coalesced grid=%5d: %8.3f ms  %8.1f GB/s (r+w)\n", g, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    }
    for (int g : {1024, 2048, 4096, 8192}) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(k_copy_strided64, dim3(g), dim3(256), 0, 0, a, b, n / 4); }, 10);
      printf("copy 64B-per-lane grid=%5d: %8.3f ms  %8.1f GB/s (r+w)\n", g, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    }
    hipFree(a); hipFree(b);
  }
  return 0;
}
