// Round-trip latency of the small-launch shapes the drop-in path uses
// (mg_search's synchronisation took ~80 us more than its
// kernel).  Median over 2000 round trips of each shape, on one non-blocking
// stream:
//   k          empty kernel, hipStreamSynchronize
//   h2d+k+d2h  64-byte pinned copy in, kernel, 64-byte copy out, sync
//   +events    the same with two timing events around the kernel
//   poll       the h2d+k+d2h shape, waiting by polling hipEventQuery on an
//              event recorded last (no blocking wait)
//   zc         kernel reads its input from and writes its result to pinned
//              host memory (no copies), sync
//   zc+poll    the same, waiting by polling
// Build: hipcc --offload-arch=gfx950 -O2 tools/exp/sync_probe.hip -o tools/exp/sync_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void k_empty(unsigned* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] += 1u;
}
extern __shared__ unsigned lds_buf[];
// a search-shaped launch: many blocks, large dynamic LDS, ~iters dependent ALU steps per lane
__global__ __launch_bounds__(256, 2) void k_big(unsigned* out, unsigned iters) {
  unsigned x = threadIdx.x;
  lds_buf[threadIdx.x] = x;
  for (unsigned i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) out[blockIdx.x] = x + lds_buf[threadIdx.x];
}
__global__ void k_rw(const unsigned long long* in, unsigned long long* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = in[0] + 1ull;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, 4096, hipHostMallocDefault));
  CK(hipMalloc(&d, 4096));
  hipEvent_t e0, e1, ef;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  const int N = 2000;
  auto run = [&](const char* name, auto body) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i) {
      const double a = now_us();
      body();
      const double b = now_us();
      if (i >= 50) t.push_back(b - a);
    }
    std::sort(t.begin(), t.end());
    std::printf("%-12s median %7.1f us  p10 %7.1f  p90 %7.1f\n", name, t[t.size() / 2], t[t.size() / 10],
                t[t.size() * 9 / 10]);
  };
  run("k", [&] {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (unsigned*)d);
    (void)hipStreamSynchronize(s);
  });
  run("h2d+k+d2h", [&] {
    (void)hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, d, d + 16);
    (void)hipMemcpyAsync(h + 16, d + 16, 64, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
  });
  run("+events", [&] {
    (void)hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s);
    (void)hipEventRecord(e0, s);
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, d, d + 16);
    (void)hipEventRecord(e1, s);
    (void)hipMemcpyAsync(h + 16, d + 16, 64, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
  });
  run("poll", [&] {
    (void)hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, d, d + 16);
    (void)hipMemcpyAsync(h + 16, d + 16, 64, hipMemcpyDeviceToHost, s);
    (void)hipEventRecord(ef, s);
    while (hipEventQuery(ef) == hipErrorNotReady) {
    }
  });
  run("zc", [&] {
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, h, h + 16);
    (void)hipStreamSynchronize(s);
  });
  run("zc+poll", [&] {
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, h, h + 16);
    (void)hipEventRecord(ef, s);
    while (hipEventQuery(ef) == hipErrorNotReady) {
    }
  });
  run("zc+2k", [&] {
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, h, d);
    hipLaunchKernelGGL(k_rw, dim3(1), dim3(64), 0, s, d, h + 16);
    (void)hipStreamSynchronize(s);
  });
  (void)hipFuncSetAttribute((const void*)k_big, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  unsigned long long* hb = nullptr;
  CK(hipHostMalloc(&hb, 1 << 16, hipHostMallocDefault));
  for (unsigned iters : {0u, 2000u, 8000u}) {
    for (unsigned blocks : {256u, 2048u}) {
      char nm[64];
      std::snprintf(nm, sizeof nm, "big%u/%u", blocks, iters);
      run(nm, [&] {
        hipLaunchKernelGGL(k_big, dim3(blocks), dim3(256), 80 * 1024, s, (unsigned*)d, iters);
        (void)hipStreamSynchronize(s);
      });
      std::snprintf(nm, sizeof nm, "big%u/%u+ev+cp", blocks, iters);
      float kms = 0.f;
      run(nm, [&] {
        (void)hipMemcpyAsync(d, hb, 1024, hipMemcpyHostToDevice, s);
        (void)hipEventRecord(e0, s);
        hipLaunchKernelGGL(k_big, dim3(blocks), dim3(256), 80 * 1024, s, (unsigned*)d, iters);
        (void)hipEventRecord(e1, s);
        (void)hipMemcpyAsync(hb + 1024, d, 8320, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipEventElapsedTime(&kms, e0, e1);
      });
      std::printf("   (kernel by events: %.1f us)\n", kms * 1e3);
    }
  }
  std::printf("check %llu\n", h[16]);
  return 0;
}
