// Round-4 probe: VALU issue cost of instruction MIXES on gfx950 (fast add/xor vs
// "slow" perm/alignbit/shift), to model the ChaCha20 quarter-round stream.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench4 tools/microbench4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 1024;

// 8 independent chains; each iteration issues the pattern once per chain.
#define K(NAME, BODY)                                                                       \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                      \
    uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 5 + 1, sel = 0x01000302u;            \
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;                         \
    for (int it = 0; it < ITERS; ++it) {                                                    \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) { BODY; }                               \
    }                                                                                       \
    uint32_t r = 0;                                                                         \
    for (int i = 0; i < 8; ++i) r ^= a[i];                                                  \
    if (r == 0x12345678u) out[0] = r;                                                       \
  }

#define ADD asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define XOR asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
#define PERM asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[i]) : "s"(sel));
#define ALIGN asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a[i]));
#define SHL asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a[i]));
#define ADDV asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));

K(k_add, ADD ADD ADD)
K(k_perm, PERM PERM PERM)
K(k_align, ALIGN ALIGN ALIGN)
K(k_add_add_perm, ADD XOR PERM)
K(k_add_add_align, ADD XOR ALIGN)
K(k_add_perm, ADD PERM ADD)
K(k_addxor6_perm2, ADD XOR ADD XOR PERM ALIGN)
K(k_addv, ADDV ADDV ADDV)
K(k_shl, SHL SHL SHL)
K(k_add_shl, ADD SHL XOR)

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
  uint32_t* d; (void)hipMalloc(&d, 64);
  struct { const char* name; void (*k)(uint32_t*, uint32_t); int per; } ks[] = {
    {"add add add", k_add, 3}, {"perm x3", k_perm, 3}, {"alignbit x3", k_align, 3}, {"lshl x3", k_shl, 3},
    {"add xor perm", k_add_add_perm, 3}, {"add xor alignbit", k_add_add_align, 3}, {"add perm add", k_add_perm, 3},
    {"add xor add xor perm align", k_addxor6_perm2, 6}, {"add (cross-chain src) x3", k_addv, 3},
    {"add lshl xor", k_add_shl, 3}};
  for (int wpc : {8, 16, 32}) {
    const int blocks = prop.multiProcessorCount * wpc / 4;
    for (auto& k : ks) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, 12345u); }, 5);
      double winst = (double)blocks * 4 * ITERS * 8 * k.per;  // wave-instructions
      double per_simd = winst / (prop.multiProcessorCount * 4);
      // cycles at the nominal 2.4 GHz (a lower sustained clock makes these read high)
      double cyc = ms * 1e-3 * 2.4e9 / per_simd;
      printf("%2d waves/CU %-28s %7.3f ms  %5.2f cyc/instr@2.4GHz  %6.2f T lane-op/s\n", wpc, k.name, ms, cyc,
             winst * 64 / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
