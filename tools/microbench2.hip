// Round-2 probes: which ChaCha20 quarter-round encoding issues fastest on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench2 tools/microbench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)
#define OPAQUE(x) asm volatile("" : "+v"(x))

constexpr int ITERS = 2048;

// ---- single-op chains through inline asm (exact instruction) ----
#define OPCHAIN(NAME, ASM)                                                          \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                              \
    uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 5;                            \
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;                  \
    for (int it = 0; it < ITERS; ++it) {                                            \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c)); \
    }                                                                               \
    uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= a[i];                          \
    if (r == 0x12345678u) out[0] = r;                                               \
  }

OPCHAIN(o_add, "v_add_u32 %0, %0, %1")
OPCHAIN(o_xor, "v_xor_b32 %0, %0, %1")
OPCHAIN(o_lshl, "v_lshlrev_b32 %0, 7, %0")
OPCHAIN(o_alignbit, "v_alignbit_b32 %0, %0, %0, 25")
OPCHAIN(o_perm, "v_perm_b32 %0, %0, %0, %2")
OPCHAIN(o_lshlor, "v_lshl_or_b32 %0, %0, 7, %1")
OPCHAIN(o_xor3, "v_or3_b32 %0, %0, %1, %2")
OPCHAIN(o_add3, "v_add3_u32 %0, %0, %1, %2")
OPCHAIN(o_xad, "v_xad_u32 %0, %0, %1, %2")
OPCHAIN(o_sdwa, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
OPCHAIN(o_add_e64, "v_add_u32_e64 %0, %0, %1")
OPCHAIN(o_bfi, "v_bfi_b32 %0, %0, %1, %2")

// ---- ChaCha20 variants ----
__device__ __forceinline__ uint32_t rot_align(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t rot_perm16(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
__device__ __forceinline__ uint32_t rot_perm8(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }
__device__ __forceinline__ uint32_t xor_rot16_sdwa(uint32_t d, uint32_t a) {
  uint32_t t;
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(t) : "v"(d), "v"(a));
  return t;
}
__device__ __forceinline__ uint32_t rot_shift(uint32_t x, int n) {
  uint32_t hi, lo;
  asm("v_lshlrev_b32 %0, %2, %1" : "=v"(hi) : "v"(x), "i"(n));
  asm("v_lshrrev_b32 %0, %2, %1" : "=v"(lo) : "v"(x), "i"(32 - n));
  uint32_t r;
  asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(hi), "v"(lo));
  return r;
}

template <int V>
__device__ __forceinline__ void qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  if constexpr (V == 0) {  // alignbit everywhere
    a += b; d ^= a; d = rot_align(d, 16); c += d; b ^= c; b = rot_align(b, 12);
    a += b; d ^= a; d = rot_align(d, 8);  c += d; b ^= c; b = rot_align(b, 7);
  } else if constexpr (V == 1) {  // SDWA xor-rot16, alignbit others
    a += b; d = xor_rot16_sdwa(d, a); c += d; b ^= c; b = rot_align(b, 12);
    a += b; d ^= a; d = rot_align(d, 8); c += d; b ^= c; b = rot_align(b, 7);
  } else if constexpr (V == 2) {  // perm for 16/8
    a += b; d ^= a; d = rot_perm16(d); c += d; b ^= c; b = rot_align(b, 12);
    a += b; d ^= a; d = rot_perm8(d);  c += d; b ^= c; b = rot_align(b, 7);
  } else {  // pure VOP2 shifts
    a += b; d = xor_rot16_sdwa(d, a); c += d; b ^= c; b = rot_shift(b, 12);
    a += b; d ^= a; d = rot_shift(d, 8); c += d; b ^= c; b = rot_shift(b, 7);
  }
}

template <int V, int NB>  // NB independent blocks interleaved per lane
__global__ void k_chacha(uint32_t* out, uint32_t seed, int nblocks) {
  uint32_t acc = 0;
  uint32_t k0 = seed, k1 = seed * 3, k2 = seed * 5, k3 = seed * 7;
  OPAQUE(k0);
  for (int blk = 0; blk < nblocks; blk += NB) {
    uint32_t x[NB][16];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      x[j][0] = 0x61707865; x[j][1] = 0x3320646e; x[j][2] = 0x79622d32; x[j][3] = 0x6b206574;
      x[j][4] = k0; x[j][5] = k1; x[j][6] = k2; x[j][7] = k3;
      x[j][8] = k0 ^ 1; x[j][9] = k1 ^ 2; x[j][10] = k2 ^ 3; x[j][11] = k3 ^ 4;
      x[j][12] = blk + j + threadIdx.x; x[j][13] = blockIdx.x; x[j][14] = 0; x[j][15] = 0;
    }
    for (int r = 0; r < 10; ++r) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        qr<V>(x[j][0], x[j][4], x[j][8], x[j][12]); qr<V>(x[j][1], x[j][5], x[j][9], x[j][13]);
        qr<V>(x[j][2], x[j][6], x[j][10], x[j][14]); qr<V>(x[j][3], x[j][7], x[j][11], x[j][15]);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        qr<V>(x[j][0], x[j][5], x[j][10], x[j][15]); qr<V>(x[j][1], x[j][6], x[j][11], x[j][12]);
        qr<V>(x[j][2], x[j][7], x[j][8], x[j][13]); qr<V>(x[j][3], x[j][4], x[j][9], x[j][14]);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= x[j][i];
  }
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
  (void)hipEventDestroy(a); (void)hipEventDestroy(b);
  return ms / reps;
}

template <int V, int NB>
static void run_chacha(const char* name, uint32_t* d, int cus) {
  for (int wpc : {8, 16, 32}) {
    const int nb = 64;
    int cb = cus * wpc / 4;
    float ms = time_kernel([&] { hipLaunchKernelGGL((k_chacha<V, NB>), dim3(cb), dim3(256), 0, 0, d, 777u, nb); }, 5);
    double blocks = (double)cb * 256 * nb;
    printf("chacha %-14s NB=%d %2d waves/CU: %7.3f ms %6.1f blocks/ns %7.1f GB/s\n", name, NB, wpc, ms,
           blocks / (ms * 1e6), blocks * 64 / (ms * 1e-3) / 1e9);
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d\n", prop.gcnArchName, prop.multiProcessorCount);
  uint32_t* d; CHECK(hipMalloc(&d, 64));
  const int cus = prop.multiProcessorCount;
  struct { const char* name; void (*k)(uint32_t*, uint32_t); } ks[] = {
    {"v_add_u32", o_add}, {"v_add_u32_e64", o_add_e64}, {"v_xor_b32", o_xor}, {"v_lshlrev_b32", o_lshl},
    {"v_alignbit_b32", o_alignbit}, {"v_perm_b32", o_perm}, {"v_lshl_or_b32", o_lshlor}, {"v_or3_b32", o_xor3},
    {"v_add3_u32", o_add3}, {"v_xad_u32", o_xad}, {"v_xor_b32_sdwa", o_sdwa}, {"v_bfi_b32", o_bfi}};
  for (int wpc : {8, 32}) {
    const int blocks = cus * wpc / 4;
    const double lane_ops = (double)blocks * 256 * ITERS * 8;
    for (auto& k : ks) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, 12345u); }, 5);
      printf("%2d waves/CU %-16s %7.3f ms %6.2f T lane-ops/s\n", wpc, k.name, ms, lane_ops / (ms * 1e-3) / 1e12);
    }
  }
  run_chacha<0, 1>("alignbit", d, cus);
  run_chacha<0, 2>("alignbit", d, cus);
  run_chacha<1, 1>("sdwa16", d, cus);
  run_chacha<1, 2>("sdwa16", d, cus);
  run_chacha<2, 1>("perm16/8", d, cus);
  run_chacha<3, 1>("sdwa+shifts", d, cus);
  return 0;
}
