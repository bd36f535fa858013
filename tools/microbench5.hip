// Round-5 probe: do different VALU instruction classes from DIFFERENT waves on one
// SIMD overlap (separate pipes), or share one issue port? Each kernel runs W waves
// per SIMD; a wave's role (instruction class) is chosen by its wave index, so a
// "mixed" launch puts both roles on every SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench5 tools/microbench5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 2048;

__device__ __forceinline__ void add_body(uint32_t* a, uint32_t b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
}
__device__ __forceinline__ void perm_body(uint32_t* a, uint32_t sel) {
#pragma unroll
  for (int i = 0; i < 8; ++i) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[i]) : "s"(sel));
}
__device__ __forceinline__ void mad_body(uint64_t* d, uint32_t x, uint32_t y) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(d[i]), "=s"(c) : "v"(x), "v"(y));
  }
}

// role bits: 1 = add, 2 = perm, 4 = mad ; mixA/mixB pick the role by wave parity
template <int ROLE_EVEN, int ROLE_ODD>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  const int wave = threadIdx.x >> 6;
  const int role = (wave & 1) ? ROLE_ODD : ROLE_EVEN;
  uint32_t a[8];
  uint64_t d[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed + i + threadIdx.x; d[i] = a[i]; }
  const uint32_t b = seed ^ threadIdx.x, sel = 0x01000302u;
  for (int it = 0; it < ITERS; ++it) {
    if (role == 1) add_body(a, b);
    else if (role == 2) perm_body(a, sel);
    else if (role == 4) mad_body(d, a[it & 7], b);
    else if (role == 5) { add_body(a, b); mad_body(d, a[3], b); }   // same wave, interleaved classes
    else if (role == 3) { add_body(a, b); perm_body(a, sel); }
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)d[i] ^ (uint32_t)(d[i] >> 32);
  if (r == 0x12345678u) out[0] = r;
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

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  uint32_t* dptr; (void)hipMalloc(&dptr, 64);
  const int cus = prop.multiProcessorCount;
  struct { const char* name; void (*fn)(uint32_t*, uint32_t); double instrs_per_iter_even, instrs_per_iter_odd; } ks[] = {
    {"add | add", k<1, 1>, 8, 8},
    {"perm | perm", k<2, 2>, 8, 8},
    {"mad64 | mad64", k<4, 4>, 8, 8},
    {"add | mad64 (separate waves)", k<1, 4>, 8, 8},
    {"add | perm (separate waves)", k<1, 2>, 8, 8},
    {"add+mad64 (same wave) x2", k<5, 5>, 16, 16},
    {"add+perm (same wave) x2", k<3, 3>, 16, 16},
  };
  for (int wps : {2, 4, 8}) {  // waves per SIMD
    const int blocks = cus * wps;  // 256-thread blocks = 4 waves, one per SIMD
    for (auto& kk : ks) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(kk.fn, dim3(blocks), dim3(256), 0, 0, dptr, 7u); }, 5);
      // per SIMD: wps waves, half even half odd (wave parity alternates across a block's 4 waves)
      double instr = (double)ITERS * wps * 0.5 * (kk.instrs_per_iter_even + kk.instrs_per_iter_odd);
      double cyc = ms * 1e-3 * 2.4e9;
      printf("%d waves/SIMD  %-30s %8.3f ms  %5.2f cyc/instr per SIMD\n", wps, kk.name, ms, cyc / instr);
    }
  }
  return 0;
}
