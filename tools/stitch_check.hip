// tools/stitch_check.hip — the stitched asm of wg_stitch.h on the device against a plain C++ restatement
// (ChaCha20 half rounds + four poly_mul steps), lane by lane, for G = 4, 8, 16. Diagnostic only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/stitch_check tools/stitch_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../wireguard-java_amd/csrc/wg_device.h"
#include "../wireguard-java_amd/csrc/wg_stitch.h"

using namespace wgd;

#define QRC(a, b, c, d)                                            \
  a += b; d ^= a; d = (d << 16) | (d >> 16);                        \
  c += d; b ^= c; b = (b << 12) | (b >> 20);                        \
  a += b; d ^= a; d = (d << 8) | (d >> 24);                         \
  c += d; b ^= c; b = (b << 7) | (b >> 25);

template <int G>
__global__ void k_check(const uint32_t* in, uint32_t* out, uint32_t* bad) {
  __shared__ uint32_t lds[64 * 4 * 4 * 2];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 64 * 4 * 4 * 2; i += 64) lds[i] = in[1024 + i];
  __syncthreads();
  uint32_t x[16], acc[5], R[5], Rs[4];
  for (int i = 0; i < 16; ++i) x[i] = in[lane * 16 + i];
  for (int i = 0; i < 5; ++i) {
    acc[i] = in[4096 + lane * 5 + i] & ((1u << 27) - 1u);
    R[i] = in[8192 + lane * 5 + i] & ((1u << 26) - 1u);
  }
  for (int i = 0; i < 4; ++i) Rs[i] = 5u * R[i + 1];
  // lane's first chunk: a lane-dependent place in the LDS image (16-B aligned), steps 4 G bytes apart
  const uint32_t base = (lane & 31u) * 16u;
  uint32_t xr[16], ar[5];
  for (int i = 0; i < 16; ++i) xr[i] = x[i];
  for (int i = 0; i < 5; ++i) ar[i] = acc[i];
  const uint32_t addr = (uint32_t)(uintptr_t)&lds[base / 4u];
  chacha20_rounds_stitch_asm<G>(x, acc, R, Rs, addr, 1u << 24);
  // reference
  for (int dr = 0; dr < kStitchDR; ++dr) {
    if (dr == 0) {
      QRC(xr[0], xr[4], xr[8], xr[12])
    } else {
      QRC(xr[0], xr[4], xr[8], xr[12]) QRC(xr[1], xr[5], xr[9], xr[13]) QRC(xr[2], xr[6], xr[10], xr[14])
      QRC(xr[3], xr[7], xr[11], xr[15])
    }
    QRC(xr[0], xr[5], xr[10], xr[15]) QRC(xr[1], xr[6], xr[11], xr[12]) QRC(xr[2], xr[7], xr[8], xr[13])
    QRC(xr[3], xr[4], xr[9], xr[14])
  }
  uint32_t S5[5] = {0u, Rs[0], Rs[1], Rs[2], Rs[3]};
  for (int t = 0; t < 4; ++t) {
    poly_mul<false>(ar, R, S5);
    const uint32_t* w = &lds[(base + 4u * G * t) / 4u];
    uint32_t c[5];
    poly_block_limbs(w[0], w[1], w[2], w[3], 1u << 24, c);
    for (int i = 0; i < 5; ++i) ar[i] += c[i];
  }
  uint32_t nbad = 0;
  for (int i = 0; i < 16; ++i) nbad += x[i] != xr[i];
  for (int i = 0; i < 5; ++i) nbad += (acc[i] != ar[i]) ? 100u : 0u;
  for (int i = 0; i < 5; ++i) {
    out[lane * 10 + i] = acc[i];
    out[lane * 10 + 5 + i] = ar[i];
  }
  atomicAdd(bad, nbad);
}

template <int G>
static int run(const uint32_t* d_in, uint32_t* d_out, uint32_t* d_bad) {
  hipMemset(d_bad, 0, 4);
  hipLaunchKernelGGL(k_check<G>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_bad);
  uint32_t bad = 0, o[640];
  hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost);
  hipMemcpy(o, d_out, sizeof o, hipMemcpyDeviceToHost);
  printf("{\"G\": %d, \"bad\": %u, \"lane0_acc\": [%u, %u, %u, %u, %u], \"lane0_ref\": [%u, %u, %u, %u, %u]}\n", G, bad,
         o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9]);
  return bad != 0;
}

int main() {
  const size_t n = 16384;
  uint32_t* h = (uint32_t*)malloc(n * 4);
  uint64_t s = 0x1234567;
  for (size_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (uint32_t)(s >> 32);
  }
  uint32_t *d_in, *d_out, *d_bad;
  hipMalloc(&d_in, n * 4);
  hipMalloc(&d_out, 640 * 4);
  hipMalloc(&d_bad, 4);
  hipMemcpy(d_in, h, n * 4, hipMemcpyHostToDevice);
  int rc = run<4>(d_in, d_out, d_bad) | run<8>(d_in, d_out, d_bad) | run<16>(d_in, d_out, d_bad);
  return rc;
}
