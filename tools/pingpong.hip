// pingpong — host <-> persistent-kernel round trip, the per-packet server's floor.
//
// One wave polls a mailbox word for the value the host last wrote, then writes that value into a
// reply word in pinned host memory; the host writes i, polls the reply for i, N times. Two mailbox
// placements:
//   host    the mailbox in pinned, device-mapped host memory (the per-packet server's ring today):
//           every device poll is a PCIe read
//   device  the mailbox in fine-grained device memory written by the host through the BAR (posted
//           PCIe writes): the device polls its own memory
// The kernel's loop is bounded (a poll budget per round trip and N round trips), so it always ends.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o pingpong pingpong.hip
// Run:   pingpong [round_trips=20000]  -> one JSON line per placement
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_pong(const uint32_t* mailbox, uint32_t* reply, uint32_t n, uint32_t* timeouts) {
  if (threadIdx.x != 0) return;
  for (uint32_t i = 1; i <= n; ++i) {
    uint32_t spins = 0;
    while (__hip_atomic_load(mailbox, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
      if (++spins > (1u << 22)) {  // about a second: the host is gone
        atomicAdd(timeouts, 1u);
        return;
      }
    }
    __hip_atomic_store(reply, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void run(const char* name, uint32_t* mbox_host_view, const uint32_t* mbox_dev_view, uint32_t n) {
  uint32_t *reply, *reply_dev, *timeouts;
  CHECK(hipHostMalloc((void**)&reply, 64, hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer((void**)&reply_dev, reply, 0));
  CHECK(hipMalloc((void**)&timeouts, 4));
  CHECK(hipMemset(timeouts, 0, 4));
  *reply = 0;
  __atomic_store_n(mbox_host_view, 0u, __ATOMIC_SEQ_CST);
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, s, mbox_dev_view, reply_dev, n, timeouts);
  CHECK(hipGetLastError());
  std::vector<double> lat;
  lat.reserve(n);
  bool ok = true;
  for (uint32_t i = 1; i <= n && ok; ++i) {
    const double t0 = now_us();
    __atomic_store_n(mbox_host_view, i, __ATOMIC_SEQ_CST);
    for (uint64_t spin = 0; __atomic_load_n((volatile uint32_t*)reply, __ATOMIC_ACQUIRE) != i; ++spin)
      if (spin > (1ull << 28)) {
        ok = false;
        break;
      }
    lat.push_back(now_us() - t0);
  }
  if (!ok) __atomic_store_n(mbox_host_view, ~0u, __ATOMIC_SEQ_CST);
  CHECK(hipStreamSynchronize(s));
  uint32_t to = 0;
  CHECK(hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost));
  std::sort(lat.begin(), lat.end());
  const size_t m = lat.size();
  printf("{\"mailbox\": \"%s\", \"round_trips\": %zu, \"ok\": %s, \"device_timeouts\": %u, "
         "\"rtt_us\": {\"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f, \"max\": %.2f}}\n",
         name, m, ok ? "true" : "false", to, lat[m / 2], lat[m * 9 / 10], lat[m * 99 / 100], lat[m - 1]);
  fflush(stdout);
  CHECK(hipStreamDestroy(s));
  CHECK(hipHostFree(reply));
  CHECK(hipFree(timeouts));
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 20000u;
  // mailbox in pinned host memory
  uint32_t *hm, *hm_dev;
  CHECK(hipHostMalloc((void**)&hm, 64, hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer((void**)&hm_dev, hm, 0));
  run("host", hm, hm_dev, n);
  // mailbox in fine-grained device memory, written by the host through the BAR
  uint32_t* dm = nullptr;
  if (hipExtMallocWithFlags((void**)&dm, 64, hipDeviceMallocFinegrained) != hipSuccess || !dm) {
    printf("{\"mailbox\": \"device\", \"ok\": false, \"error\": \"no fine-grained device memory\"}\n");
    return 0;
  }
  // one virtual address space: the host stores to the same address (a large-BAR mapping of VRAM);
  // run last, since a host without that mapping faults here (a host fault, not a device one)
  hipPointerAttribute_t attr;
  uint32_t* hv = dm;
  if (hipPointerGetAttributes(&attr, dm) == hipSuccess && attr.hostPointer) hv = (uint32_t*)attr.hostPointer;
  run("device", hv, dm, n);
  return 0;
}
