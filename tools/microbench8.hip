// Memory-pattern probe for the transport kernels: how fast can the chip read and
// write N packets of 1424 B (89 x 16-B chunks) at a 1440-B stride, as a function of
// how many lanes share a packet (G) and how many 16-B chunks a lane moves per step (C)?
// Lane j of a packet group moves chunks t*G*C + i*G + j (i < C) in step t, so one wave
// instruction covers G*16 contiguous bytes of each of its 64/G packets.
// out = in ^ 0x5a... (every byte read once, written once). No compute.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench8 tools/microbench8.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint32_t STRIDE = 1440, CHUNKS = 89;

// IL: lane j of the group moves chunks base + i*G + j (interleaved: one instruction
// covers G*16 contiguous bytes); !IL: chunks base + j*C + i (each lane C contiguous
// chunks, k_wave's layout: one instruction covers G chunks at a C*16-byte stride)
template <int G, int C, bool IL = true>
__global__ void __launch_bounds__(256) k_pat(const uint8_t* in, uint8_t* out, uint32_t npkt) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  const uint32_t pkt = gid / G, j = gid % G;
  if (pkt >= npkt) return;
  const uint4* src = (const uint4*)(in + (uint64_t)pkt * STRIDE);
  uint4* dst = (uint4*)(out + (uint64_t)pkt * STRIDE);
  for (uint32_t base = 0; base < CHUNKS; base += G * C) {
    uint4 v[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const uint32_t c = IL ? base + i * G + j : base + j * C + i;
      v[i] = c < CHUNKS ? src[c] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const uint32_t c = IL ? base + i * G + j : base + j * C + i;
      if (c < CHUNKS) dst[c] = make_uint4(v[i].x ^ 0x5a5a5a5au, v[i].y, v[i].z, v[i].w);
    }
  }
}

// contiguous streaming copy of the same byte count (the ceiling)
__global__ void __launch_bounds__(256) k_stream_copy(const uint4* in, uint4* out, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256u) {
    uint4 v = in[i];
    out[i] = make_uint4(v.x ^ 0x5a5a5a5au, v.y, v.z, v.w);
  }
}

template <typename F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

template <int G, int C, bool IL = true>
void run(const uint8_t* in, uint8_t* out, uint32_t npkt) {
  const uint32_t threads = npkt * G;
  const float ms = time_it([&] { hipLaunchKernelGGL((k_pat<G, C, IL>), dim3((threads + 255) / 256), dim3(256), 0, 0, in, out, npkt); }, 10);
  const double bytes = 2.0 * npkt * CHUNKS * 16.0;
  printf("G=%2d C=%2d %s %8.1f us  %6.2f TB/s  (per 64K packets %.1f us)\n", G, C, IL ? "il " : "blk", ms * 1e3, bytes / (ms * 1e-3) / 1e12,
         ms * 1e3 * 65536.0 / npkt);
}

int main() {
  const uint32_t npkt = 1u << 20;
  uint8_t *in, *out;
  (void)hipMalloc(&in, (size_t)npkt * STRIDE);
  (void)hipMalloc(&out, (size_t)npkt * STRIDE);
  (void)hipMemset(in, 1, (size_t)npkt * STRIDE);
  const uint64_t n16 = (uint64_t)npkt * STRIDE / 16;
  const float ms = time_it([&] { hipLaunchKernelGGL(k_stream_copy, dim3(4096), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n16); }, 10);
  printf("stream copy  %8.1f us  %6.2f TB/s (whole 1440-B strides)\n", ms * 1e3, 2.0 * n16 * 16 / (ms * 1e-3) / 1e12);
  run<1, 4>(in, out, npkt);
  run<1, 8>(in, out, npkt);
  run<1, 16>(in, out, npkt);
  run<2, 4>(in, out, npkt);
  run<4, 1>(in, out, npkt);
  run<4, 4>(in, out, npkt);
  run<4, 8>(in, out, npkt);
  run<8, 1>(in, out, npkt);
  run<8, 4>(in, out, npkt);
  run<16, 2>(in, out, npkt);
  run<32, 1>(in, out, npkt);
  run<64, 1>(in, out, npkt);
  run<8, 4, false>(in, out, npkt);
  run<8, 8, false>(in, out, npkt);
  run<4, 4, false>(in, out, npkt);
  run<2, 4, false>(in, out, npkt);
  return 0;
}
