#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>
typedef uint32_t u32; typedef uint64_t u64;
extern "C" __global__ void asm_kernel(const u32* code, u64 n, u32* out);
int main() {
  const int L = 4096; std::vector<u32> code(L + 8, 0);
  std::mt19937 rng(1);
  for (int i = 0; i < L; i++) {
    u32 op = 1 + (i & 1), d = rng() % 16, a = rng() % 16, b = rng() % 16;
    code[i] = op | d << 8 | a << 16 | b << 24;
  }
  u32 *dcode, *dout; u64 n = 1ull << 22;
  hipMalloc(&dcode, code.size() * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(dcode, code.data(), code.size() * 4, hipMemcpyHostToDevice);
  int ncu = 256; hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int grid : {ncu * 8, ncu * 16}) {
    hipLaunchKernelGGL(asm_kernel, dim3(grid), dim3(256), 0, 0, dcode, n, dout);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(asm_kernel, dim3(grid), dim3(256), 0, 0, dcode, n, dout);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
    printf("grid %d: %.3f ms, %.1f G lane-insn/s (err=%s)\n", grid, ms, (double)n * L / (ms * 1e-3) / 1e9,
           hipGetErrorString(hipGetLastError()));
  }
  // CPU check of a few lanes
  std::vector<u32> out(n); hipMemcpy(out.data(), dout, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (u64 c = 0; c < 1000; c += 37) {
    u32 W[16][8];
    for (int i = 0; i < 128; i++) W[i / 8][i % 8] = i < 32 ? i + (u32)c : i < 64 ? (i ^ (u32)c) : 0;
    for (int i = 0; i < L; i++) {
      u32 op = code[i] & 255, d = code[i] >> 8 & 255, a = code[i] >> 16 & 255, b = code[i] >> 24;
      u32 r[8];
      if (op == 1) { u64 cy = 0; for (int k = 0; k < 8; k++) { u64 s = (u64)W[a][k] + W[b][k] + cy; r[k] = (u32)s; cy = s >> 32; } }
      else for (int k = 0; k < 8; k++) r[k] = W[a][k] ^ W[b][k];
      for (int k = 0; k < 8; k++) W[d][k] = r[k];
    }
    if ((W[0][0] ^ W[0][7]) != out[c]) bad++;
  }
  printf("mismatches: %d\n", bad);
}
