// Experiment: exact 2-by-1 reciprocal floor((2^64-1)/d) - 2^32 (d >= 2^31) on
// gfx950 via an f64 reciprocal + Newton steps + one integer correction, vs
// LLVM's u64 division.  Checks every lane's result for equality and times both.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32;
typedef uint64_t u64;

__device__ __forceinline__ u32 recip_ref(u32 d) { return (u32)(~0ull / (u64)d - (1ull << 32)); }

__device__ __forceinline__ u32 recip_f64(u32 d) {
  const u32 nh = ~d;                                  // (2^64-1) - 2^32 d = nh:ffffffff
  const double dd = (double)d;
  double r = __builtin_amdgcn_rcp(dd);
  double e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double n = __builtin_fma((double)nh, 4294967296.0, 4294967295.0);
  u32 v = (u32)(n * r);
  const u64 nx = ((u64)nh << 32) | 0xffffffffu;
  const u64 p = (u64)v * d;
  if (p > nx) v -= 1u;
  else if (nx - p >= d) v += 1u;
  return v;
}

__global__ void check(u64 seed, u32 iters, unsigned long long* bad, u32* sink, int mode) {
  u32 x = (u32)(seed ^ (blockIdx.x * 256u + threadIdx.x) * 2654435761u);
  u32 acc = 0, nbad = 0;
  for (u32 i = 0; i < iters; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    u32 d = x | 0x80000000u;
    if (i & 7) d = (i & 1) ? (0x80000000u + (i & 255)) : (0xffffffffu - (i & 255));
    if (mode == 0) { nbad += recip_f64(d) != recip_ref(d); acc ^= recip_f64(d); }
    else if (mode == 1) acc ^= recip_ref(d);
    else acc ^= recip_f64(d);
  }
  if (nbad) atomicAdd(bad, nbad);
  sink[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main() {
  unsigned long long* bad; u32* sink;
  hipMalloc(&bad, 8); hipMemset(bad, 0, 8);
  hipMalloc(&sink, 2048 * 256 * 4);
  hipLaunchKernelGGL(check, dim3(2048), dim3(256), 0, 0, 12345ull, 4096u, bad, sink, 0);
  unsigned long long h = 0;
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  printf("mismatches over %llu divisors: %llu\n", 2048ull * 256 * 4096, h);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int mode = 1; mode <= 2; ++mode) {
    hipEventRecord(a);
    hipLaunchKernelGGL(check, dim3(2048), dim3(256), 0, 0, 777ull, 4096u, bad, sink, mode);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%s: %.2f ms\n", mode == 1 ? "u64 division" : "f64 reciprocal", ms);
  }
  return h ? 1 : 0;
}
