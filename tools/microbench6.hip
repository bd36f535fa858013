// Round-6 probe: issue cost of the instruction forms a ChaCha20 quarter round can
// be written with on gfx950, and the chip-wide ChaCha20 block rate with no memory
// traffic (the VALU ceiling of the transport kernels).
//  part 1: one instruction form, 8 independent chains per wave
//  part 2: chacha20_block_lds (wg_device.h) per lane in a loop, perm/alignbit
//          rotates vs SDWA word-swap xor for rotl16; 4/8 waves per SIMD
// Build: hipcc --offload-arch=gfx950 -O3 -I wireguard-java_amd/csrc -o tools/microbench6 tools/microbench6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "wg_device.h"

constexpr int ITERS = 1024;

#define K(NAME, BODY)                                                                       \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {              \
    uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 5 + 1, sel = 0x01000302u;            \
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 7 + threadIdx.x;                         \
    for (int it = 0; it < ITERS; ++it) {                                                    \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) { BODY; }                               \
    }                                                                                       \
    uint32_t r = 0;                                                                         \
    for (int i = 0; i < 8; ++i) r ^= a[i];                                                  \
    if (r == 0x12345678u) out[0] = r + b + c + sel;                                         \
  }

#define ADD asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define XOR asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
#define PERM asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[i]) : "s"(sel));
#define ALIGN asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a[i]));
#define ALIGNBYTE asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(a[i]));
#define XOR3 asm volatile("v_xor3_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define ADD3 asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define XAD asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define LSHLOR asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[i]) : "v"(c));
#define SHL asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a[i]));
#define SWAPXOR                                                                                         \
  {                                                                                                     \
    uint32_t t;                                                                                         \
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0" \
                 : "=&v"(t) : "v"(a[i]), "v"(c));                                                      \
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" \
                 : "+v"(t) : "v"(a[i]), "v"(c));                                                       \
    a[i] = t;                                                                                           \
  }
#define XORSDWA asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(a[i]) : "v"(c));
#define ADDSDWA asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(a[i]) : "v"(c));
#define MUL24 asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define MAD24 asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define PKADD16 asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define BFI asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define ADDDPP asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(b));

K(k_add, ADD ADD ADD)
K(k_xor, XOR XOR XOR)
K(k_perm, PERM PERM PERM)
K(k_align, ALIGN ALIGN ALIGN)
K(k_alignbyte, ALIGNBYTE ALIGNBYTE ALIGNBYTE)
K(k_add3, ADD3 ADD3 ADD3)
K(k_lshlor, LSHLOR LSHLOR LSHLOR)
K(k_shl, SHL SHL SHL)
K(k_swapxor, SWAPXOR SWAPXOR SWAPXOR)  // 2 instructions each
K(k_xorsdwa, XORSDWA XORSDWA XORSDWA)
K(k_addsdwa, ADDSDWA ADDSDWA ADDSDWA)
K(k_mul24, MUL24 MUL24 MUL24)
K(k_mad24, MAD24 MAD24 MAD24)
K(k_pkadd16, PKADD16 PKADD16 PKADD16)
K(k_bfi, BFI BFI BFI)
K(k_adddpp, ADDDPP ADDDPP ADDDPP)

// ---- part 2: ChaCha20 block rate (no memory traffic) -----------------------------------
template <bool SDWA>
__global__ void __launch_bounds__(256) k_chacha(uint32_t* out, uint32_t seed, int blocks_per_lane) {
  __shared__ uint4 key[2];
  if (threadIdx.x < 2) key[threadIdx.x] = make_uint4(seed, seed * 3, seed * 5, seed * 7 + threadIdx.x);
  __syncthreads();
  uint32_t acc = 0;
  for (int it = 0; it < blocks_per_lane; ++it) {
    const uint32_t ctr = blockIdx.x * 4096u + threadIdx.x * 16u + it;
    uint32_t ks[16];
    wgd::chacha20_block_lds<SDWA>(key, ctr, seed, 0u, 0u, ks);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= ks[i];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the SDWA block against the reference form, every lane a different counter
__global__ void k_check(uint32_t* out) {
  __shared__ uint4 key[2];
  if (threadIdx.x < 2) key[threadIdx.x] = make_uint4(0x03020100u, 0x07060504u, 0x0b0a0908u, 0x0f0e0d0cu + threadIdx.x);
  __syncthreads();
  uint32_t a[16], b[16];
  wgd::chacha20_block_lds<false>(key, threadIdx.x * 977u, 0x09000000u, 0x4a000000u, 0u, a);
  wgd::chacha20_block_lds<true>(key, threadIdx.x * 977u, 0x09000000u, 0x4a000000u, 0u, b);
  for (int i = 0; i < 16; ++i)
    if (a[i] != b[i]) atomicAdd(out, 1u);
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
  uint32_t* d; (void)hipMalloc(&d, 64);
  (void)hipMemset(d, 0, 64);
  hipLaunchKernelGGL(k_check, dim3(4), dim3(256), 0, 0, d);
  uint32_t bad = 0;
  (void)hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost);
  printf("sdwa chacha20 block check: %s (%u mismatching words)\n", bad ? "MISMATCH" : "ok", bad);
  const int cus = prop.multiProcessorCount;
  struct { const char* name; void (*k)(uint32_t*, uint32_t); int per; } ks[] = {
    {"v_add_u32", k_add, 3}, {"v_xor_b32", k_xor, 3}, {"v_perm_b32", k_perm, 3}, {"v_alignbit_b32", k_align, 3},
    {"v_alignbyte_b32", k_alignbyte, 3}, {"v_add3_u32", k_add3, 3},
    {"v_lshl_or_b32", k_lshlor, 3}, {"v_lshlrev_b32", k_shl, 3},
    {"2x v_xor_b32_sdwa (rotl16 xor)", k_swapxor, 6}, {"v_xor_b32_sdwa preserve", k_xorsdwa, 3},
    {"v_add_u32_sdwa", k_addsdwa, 3}, {"v_mul_u32_u24", k_mul24, 3}, {"v_mad_u32_u24", k_mad24, 3},
    {"v_pk_add_u16", k_pkadd16, 3}, {"v_bfi_b32", k_bfi, 3}, {"v_add_u32_dpp", k_adddpp, 3}};
  for (int wps : {4, 8}) {
    const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
    for (auto& k : ks) {
      float ms = time_kernel([&] { hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, 12345u); }, 5);
      double per_simd = (double)wps * ITERS * 8 * k.per;
      printf("%d waves/SIMD  %-32s %7.3f ms  %5.2f cyc/instr@2.4GHz\n", wps, k.name, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  for (int form = 0; form < 2; ++form) {
    for (int wps : {4, 8}) {
      const int blocks = cus * wps, bpl = 256;
      auto launch = [&] {
        if (form == 0) hipLaunchKernelGGL(k_chacha<false>, dim3(blocks), dim3(256), 0, 0, d, 7u, bpl);
        else hipLaunchKernelGGL(k_chacha<true>, dim3(blocks), dim3(256), 0, 0, d, 7u, bpl);
      };
      float ms = time_kernel(launch, 5);
      double nblk = (double)blocks * 256 * bpl;
      double wave_blocks_per_simd = nblk / 64 / (cus * 4);
      printf("chacha20 %s %d waves/SIMD: %.3f ms  %.3f G blocks/s = %.0f GiB/s keystream  %.0f cyc/wave-block@2.4GHz\n",
             form ? "sdwa-rotl16" : "perm/align ", wps, ms, nblk / (ms * 1e-3) / 1e9,
             nblk * 64 / (ms * 1e-3) / (1u << 30), ms * 1e-3 * 2.4e9 / wave_blocks_per_simd);
    }
  }
  return 0;
}
