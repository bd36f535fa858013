// microbench20 — the Poly1305 Horner step of k_transport in isolation (round-4 study):
// issue cost vs dependency stalls of the v_mad_u64_u32 chains at 8 waves per SIMD, and the
// alternatives that fold several chunks into one reduction.
//
//   A  k_transport's step: acc = (acc + m) * R, one 25-mad chain (each limb's carry seeds the next
//      limb's chain, wgd::poly_mul), one chunk per step
//   B  two chunks per reduction: acc = acc*R^2 + m0*R + m1 as 5 independent 10-mad limb chains,
//      then one 64-bit carry pass (needs R and R^2, 5R and 5R^2)
//   C  the same two-chunk step with the carry-seeded chain (one 50-mad chain)
//   D  four chunks per reduction (R..R^4), 5 independent 20-mad chains, one carry pass
//   E  A's single step with five independent chains and the 64-bit carry pass (no seeding)
//
// Every wave evaluates the same 48-chunk polynomial (lane-dependent data) with each variant; the
// canonical results must agree (checked on the host). Time: HIP events around the launch; 8192 waves
// (8 per SIMD, 64 VGPRs or fewer), cycles per chunk per wave = duration * 2.4 GHz * 1024 SIMDs /
// (waves * chunks).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../wireguard-java_amd/csrc -o microbench20 microbench20.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#include "wg_device.h"

using namespace wgd;

constexpr int CH = 48;   // chunks per evaluation
constexpr int REPS = 8;  // evaluations per wave

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, cc;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return d;
}

// d_k = sum over products a_i * b_j (i + j = k) + 5 a_i b_j (i + j = k + 5), accumulated into d
__device__ __forceinline__ void prod_acc(const uint32_t a[5], const uint32_t b[5], const uint32_t b5[5],
                                         uint64_t d[5]) {
  d[0] = mad(a[0], b[0], mad(a[1], b5[4], mad(a[2], b5[3], mad(a[3], b5[2], mad(a[4], b5[1], d[0])))));
  d[1] = mad(a[0], b[1], mad(a[1], b[0], mad(a[2], b5[4], mad(a[3], b5[3], mad(a[4], b5[2], d[1])))));
  d[2] = mad(a[0], b[2], mad(a[1], b[1], mad(a[2], b[0], mad(a[3], b5[4], mad(a[4], b5[3], d[2])))));
  d[3] = mad(a[0], b[3], mad(a[1], b[2], mad(a[2], b[1], mad(a[3], b[0], mad(a[4], b5[4], d[3])))));
  d[4] = mad(a[0], b[4], mad(a[1], b[3], mad(a[2], b[2], mad(a[3], b[1], mad(a[4], b[0], d[4])))));
}
// 64-bit limb sums (< 2^63) -> limbs < 2^26 + small
__device__ __forceinline__ void carry64(uint64_t d[5], uint32_t h[5]) {
  uint64_t c;
  c = d[0] >> 26; h[0] = (uint32_t)d[0] & M26; d[1] += c;
  c = d[1] >> 26; h[1] = (uint32_t)d[1] & M26; d[2] += c;
  c = d[2] >> 26; h[2] = (uint32_t)d[2] & M26; d[3] += c;
  c = d[3] >> 26; h[3] = (uint32_t)d[3] & M26; d[4] += c;
  c = d[4] >> 26; h[4] = (uint32_t)d[4] & M26;
  const uint64_t t = (uint64_t)h[0] + c * 5u;  // c < 2^32 (D: 20 products per limb)
  h[0] = (uint32_t)t & M26;
  h[1] += (uint32_t)(t >> 26);
}

__device__ __forceinline__ void chunk(uint32_t seed, uint32_t k, uint32_t m[5]) {
  const uint32_t w0 = seed * 0x9E3779B9u + k, w1 = w0 ^ 0x85EBCA6Bu, w2 = w0 * 3u, w3 = w0 + 0x1234567u;
  poly_block_limbs(w0, w1, w2, w3, 1u << 24, m);
}

struct Pw {  // R^1..R^4 and their 5x forms
  uint32_t r[4][5], r5[4][5];
};

template <int V>
__global__ void __launch_bounds__(256) k(const Pw* pw, uint32_t* out) {
  const uint32_t seed = blockIdx.x * 256u + threadIdx.x;
  uint32_t acc_all = 0;
  uint32_t R[5], R5[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    R[i] = pw->r[0][i];
    R5[i] = pw->r5[0][i];
  }
  uint32_t h[5];
  for (int rep = 0; rep < REPS; ++rep) {
#pragma unroll
    for (int i = 0; i < 5; ++i) h[i] = 0;
    if constexpr (V == 0 || V == 4) {  // one chunk per step
      for (int c = 0; c < CH; ++c) {
        uint32_t m[5];
        chunk(seed + rep, c, m);
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] += m[i];
        if constexpr (V == 0) {
          poly_mul(h, R, R5);
        } else {
          uint64_t d[5] = {0, 0, 0, 0, 0};
          prod_acc(h, R, R5, d);
          carry64(d, h);
        }
      }
    } else if constexpr (V == 1 || V == 2) {  // two chunks per reduction
      uint32_t Q[5], Q5[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        Q[i] = pw->r[1][i];
        Q5[i] = pw->r5[1][i];
      }
      for (int c = 0; c < CH; c += 2) {
        uint32_t m0[5], m1[5];
        chunk(seed + rep, c, m0);
        chunk(seed + rep, c + 1, m1);
        // (h + m0) R^2 + m1 R
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] += m0[i];
        if constexpr (V == 1) {
          uint64_t d[5] = {0, 0, 0, 0, 0};
          prod_acc(h, Q, Q5, d);
          prod_acc(m1, R, R5, d);
          carry64(d, h);
        } else {
          // carry-seeded: limb k of both products in one chain started from limb k-1's carry
          uint64_t d = mad(h[0], Q[0], mad(h[1], Q5[4], mad(h[2], Q5[3], mad(h[3], Q5[2], (uint64_t)h[4] * Q5[1]))));
          d = mad(m1[0], R[0], mad(m1[1], R5[4], mad(m1[2], R5[3], mad(m1[3], R5[2], mad(m1[4], R5[1], d)))));
          const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
          uint32_t o[5];
          o[0] = (uint32_t)d & M26;
          d = mad(h4, Q5[2], mad(h3, Q5[3], mad(h2, Q5[4], mad(h1, Q[0], mad(h0, Q[1], d >> 26)))));
          d = mad(m1[4], R5[2], mad(m1[3], R5[3], mad(m1[2], R5[4], mad(m1[1], R[0], mad(m1[0], R[1], d)))));
          o[1] = (uint32_t)d & M26;
          d = mad(h4, Q5[3], mad(h3, Q5[4], mad(h2, Q[0], mad(h1, Q[1], mad(h0, Q[2], d >> 26)))));
          d = mad(m1[4], R5[3], mad(m1[3], R5[4], mad(m1[2], R[0], mad(m1[1], R[1], mad(m1[0], R[2], d)))));
          o[2] = (uint32_t)d & M26;
          d = mad(h4, Q5[4], mad(h3, Q[0], mad(h2, Q[1], mad(h1, Q[2], mad(h0, Q[3], d >> 26)))));
          d = mad(m1[4], R5[4], mad(m1[3], R[0], mad(m1[2], R[1], mad(m1[1], R[2], mad(m1[0], R[3], d)))));
          o[3] = (uint32_t)d & M26;
          d = mad(h4, Q[0], mad(h3, Q[1], mad(h2, Q[2], mad(h1, Q[3], mad(h0, Q[4], d >> 26)))));
          d = mad(m1[4], R[0], mad(m1[3], R[1], mad(m1[2], R[2], mad(m1[1], R[3], mad(m1[0], R[4], d)))));
          o[4] = (uint32_t)d & M26;
          uint32_t cc = (uint32_t)(d >> 26);
          o[0] += cc * 5u;
          cc = o[0] >> 26;
          o[0] &= M26;
          o[1] += cc;
#pragma unroll
          for (int i = 0; i < 5; ++i) h[i] = o[i];
        }
      }
    } else {  // V == 3: four chunks per reduction
      for (int c = 0; c < CH; c += 4) {
        uint32_t m[5];
        chunk(seed + rep, c, m);
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] += m[i];
        uint64_t d[5] = {0, 0, 0, 0, 0};
        prod_acc(h, pw->r[3], pw->r5[3], d);
#pragma unroll
        for (int t = 1; t < 4; ++t) {
          chunk(seed + rep, c + t, m);
          prod_acc(m, pw->r[3 - t], pw->r5[3 - t], d);
        }
        carry64(d, h);
      }
    }
    uint32_t tag[4];
    poly_finish(h, 0, 0, 0, 0, tag);
    acc_all ^= tag[0] ^ tag[1] ^ tag[2] ^ tag[3];
  }
  out[seed] = acc_all;
}

static void mulmod(const uint32_t a[5], const uint32_t b[5], uint32_t o[5]) {  // host, radix 2^26
  unsigned __int128 d[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      const unsigned __int128 p = (unsigned __int128)a[i] * b[j];
      if (i + j < 5) d[i + j] += p;
      else d[i + j - 5] += p * 5;
    }
  unsigned __int128 c = 0;
  for (int k = 0; k < 5; ++k) {
    d[k] += c;
    o[k] = (uint32_t)(d[k] & 0x3ffffff);
    c = d[k] >> 26;
  }
  uint64_t cc = (uint64_t)c * 5 + o[0];
  o[0] = (uint32_t)(cc & 0x3ffffff);
  o[1] += (uint32_t)(cc >> 26);
}

int main() {
  Pw pw;
  const uint32_t r[5] = {0x0123456 & 0x3ffffff, 0x2345678 & 0x3ffff03, 0x1b2c3d4 & 0x3ffc0ff, 0x0fedcba & 0x3f03fff,
                         0x00abcde & 0x00fffff};
  for (int i = 0; i < 5; ++i) pw.r[0][i] = r[i];
  for (int p = 1; p < 4; ++p) mulmod(pw.r[p - 1], r, pw.r[p]);
  for (int p = 0; p < 4; ++p)
    for (int i = 0; i < 5; ++i) pw.r5[p][i] = i ? pw.r[p][i] * 5u : 0u;
  Pw* dpw;
  uint32_t* dout;
  const uint32_t blocks = 2048, n = blocks * 256;
  hipMalloc(&dpw, sizeof pw);
  hipMalloc(&dout, n * 4);
  hipMemcpy(dpw, &pw, sizeof pw, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<uint32_t> ref(n), got(n);
  const char* names[5] = {"A one chunk, carry-seeded 25-mad chain (k_transport)",
                          "B two chunks per reduction, 5 independent 10-mad chains",
                          "C two chunks per reduction, carry-seeded 50-mad chain",
                          "D four chunks per reduction, 5 independent 20-mad chains",
                          "E one chunk, 5 independent chains + 64-bit carry pass"};
  auto run = [&](int v, void (*kern)(const Pw*, uint32_t*)) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, dpw, dout);
    hipEventRecord(a);
    const int it = 10;
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, dpw, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= it;
    hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
    if (v == 0) ref = got;
    const bool same = got == ref;
    const double waves = n / 64.0, chunks = (double)CH * REPS;
    const double cyc = ms * 1e-3 * 2.4e9 * 1024 / (waves * chunks);
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"cycles_per_chunk_per_wave\": %.1f, \"same_result\": %s}\n",
           names[v], ms, cyc, same ? "true" : "false");
  };
  run(0, k<0>);
  run(1, k<1>);
  run(2, k<2>);
  run(3, k<3>);
  run(4, k<4>);
  return 0;
}
