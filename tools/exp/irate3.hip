// Experiment: issue rates of more instruction forms (see tools/exp/irate.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/exp/irate3 tools/exp/irate3.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32;
typedef uint64_t u64;
#define ITERS 4096

__global__ void k0(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_cmp_lt_u32_e32 vcc, %8, %9\n s_nop 4\n" "v_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43", "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k1(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("s_mov_b64 vcc, 0x5555\n" "v_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\nv_cndmask_b32_e32 %0, %0, %8, vcc\nv_cndmask_b32_e32 %1, %1, %8, vcc\nv_cndmask_b32_e32 %2, %2, %8, vcc\nv_cndmask_b32_e32 %3, %3, %8, vcc\nv_cndmask_b32_e32 %4, %4, %8, vcc\nv_cndmask_b32_e32 %5, %5, %8, vcc\nv_cndmask_b32_e32 %6, %6, %8, vcc\nv_cndmask_b32_e32 %7, %7, %8, vcc\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43", "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k2(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_cmp_lt_u32_e32 vcc, %8, %9\n s_nop 4\n" "v_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\nv_cndmask_b32_e64 %0, %0, %8, vcc\nv_cndmask_b32_e64 %1, %1, %8, vcc\nv_cndmask_b32_e64 %2, %2, %8, vcc\nv_cndmask_b32_e64 %3, %3, %8, vcc\nv_cndmask_b32_e64 %4, %4, %8, vcc\nv_cndmask_b32_e64 %5, %5, %8, vcc\nv_cndmask_b32_e64 %6, %6, %8, vcc\nv_cndmask_b32_e64 %7, %7, %8, vcc\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43", "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k3(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("s_mov_b64 s[40:41], 0x5555\n" "v_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\nv_cndmask_b32_e64 %0, %0, %8, s[40:41]\nv_cndmask_b32_e64 %1, %1, %8, s[40:41]\nv_cndmask_b32_e64 %2, %2, %8, s[40:41]\nv_cndmask_b32_e64 %3, %3, %8, s[40:41]\nv_cndmask_b32_e64 %4, %4, %8, s[40:41]\nv_cndmask_b32_e64 %5, %5, %8, s[40:41]\nv_cndmask_b32_e64 %6, %6, %8, s[40:41]\nv_cndmask_b32_e64 %7, %7, %8, s[40:41]\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k4(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\nv_cmp_lt_u32_e32 vcc, %0, %8\nv_cmp_lt_u32_e32 vcc, %1, %8\nv_cmp_lt_u32_e32 vcc, %2, %8\nv_cmp_lt_u32_e32 vcc, %3, %8\nv_cmp_lt_u32_e32 vcc, %4, %8\nv_cmp_lt_u32_e32 vcc, %5, %8\nv_cmp_lt_u32_e32 vcc, %6, %8\nv_cmp_lt_u32_e32 vcc, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43", "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k5(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\nv_sub_u32_e32 %0, %0, %8\nv_sub_u32_e32 %1, %1, %8\nv_sub_u32_e32 %2, %2, %8\nv_sub_u32_e32 %3, %3, %8\nv_sub_u32_e32 %4, %4, %8\nv_sub_u32_e32 %5, %5, %8\nv_sub_u32_e32 %6, %6, %8\nv_sub_u32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k6(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\nv_or_b32_e32 %0, %0, %8\nv_or_b32_e32 %1, %1, %8\nv_or_b32_e32 %2, %2, %8\nv_or_b32_e32 %3, %3, %8\nv_or_b32_e32 %4, %4, %8\nv_or_b32_e32 %5, %5, %8\nv_or_b32_e32 %6, %6, %8\nv_or_b32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k7(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\nv_and_b32_e32 %0, %0, %8\nv_and_b32_e32 %1, %1, %8\nv_and_b32_e32 %2, %2, %8\nv_and_b32_e32 %3, %3, %8\nv_and_b32_e32 %4, %4, %8\nv_and_b32_e32 %5, %5, %8\nv_and_b32_e32 %6, %6, %8\nv_and_b32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k8(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\nv_not_b32_e32 %0, %0\nv_not_b32_e32 %1, %1\nv_not_b32_e32 %2, %2\nv_not_b32_e32 %3, %3\nv_not_b32_e32 %4, %4\nv_not_b32_e32 %5, %5\nv_not_b32_e32 %6, %6\nv_not_b32_e32 %7, %7\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k9(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\nv_lshrrev_b32_e32 %0, %8, %0\nv_lshrrev_b32_e32 %1, %8, %1\nv_lshrrev_b32_e32 %2, %8, %2\nv_lshrrev_b32_e32 %3, %8, %3\nv_lshrrev_b32_e32 %4, %8, %4\nv_lshrrev_b32_e32 %5, %8, %5\nv_lshrrev_b32_e32 %6, %8, %6\nv_lshrrev_b32_e32 %7, %8, %7\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k10(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\nv_lshrrev_b32_e32 %0, 7, %0\nv_lshrrev_b32_e32 %1, 7, %1\nv_lshrrev_b32_e32 %2, 7, %2\nv_lshrrev_b32_e32 %3, 7, %3\nv_lshrrev_b32_e32 %4, 7, %4\nv_lshrrev_b32_e32 %5, 7, %5\nv_lshrrev_b32_e32 %6, 7, %6\nv_lshrrev_b32_e32 %7, 7, %7\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k11(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\nv_bfe_u32 %0, %0, %8, %9\nv_bfe_u32 %1, %1, %8, %9\nv_bfe_u32 %2, %2, %8, %9\nv_bfe_u32 %3, %3, %8, %9\nv_bfe_u32 %4, %4, %8, %9\nv_bfe_u32 %5, %5, %8, %9\nv_bfe_u32 %6, %6, %8, %9\nv_bfe_u32 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k12(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\nv_bfi_b32 %0, %0, %8, %9\nv_bfi_b32 %1, %1, %8, %9\nv_bfi_b32 %2, %2, %8, %9\nv_bfi_b32 %3, %3, %8, %9\nv_bfi_b32 %4, %4, %8, %9\nv_bfi_b32 %5, %5, %8, %9\nv_bfi_b32 %6, %6, %8, %9\nv_bfi_b32 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k13(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\nv_perm_b32 %0, %0, %8, %9\nv_perm_b32 %1, %1, %8, %9\nv_perm_b32 %2, %2, %8, %9\nv_perm_b32 %3, %3, %8, %9\nv_perm_b32 %4, %4, %8, %9\nv_perm_b32 %5, %5, %8, %9\nv_perm_b32 %6, %6, %8, %9\nv_perm_b32 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k14(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\nv_lshl_or_b32 %0, %0, %8, %9\nv_lshl_or_b32 %1, %1, %8, %9\nv_lshl_or_b32 %2, %2, %8, %9\nv_lshl_or_b32 %3, %3, %8, %9\nv_lshl_or_b32 %4, %4, %8, %9\nv_lshl_or_b32 %5, %5, %8, %9\nv_lshl_or_b32 %6, %6, %8, %9\nv_lshl_or_b32 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k15(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\nv_or3_b32 %0, %0, %8, %9\nv_or3_b32 %1, %1, %8, %9\nv_or3_b32 %2, %2, %8, %9\nv_or3_b32 %3, %3, %8, %9\nv_or3_b32 %4, %4, %8, %9\nv_or3_b32 %5, %5, %8, %9\nv_or3_b32 %6, %6, %8, %9\nv_or3_b32 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k16(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\nv_min_u32_e32 %0, %0, %8\nv_min_u32_e32 %1, %1, %8\nv_min_u32_e32 %2, %2, %8\nv_min_u32_e32 %3, %3, %8\nv_min_u32_e32 %4, %4, %8\nv_min_u32_e32 %5, %5, %8\nv_min_u32_e32 %6, %6, %8\nv_min_u32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k17(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\nv_max_u32_e32 %0, %0, %8\nv_max_u32_e32 %1, %1, %8\nv_max_u32_e32 %2, %2, %8\nv_max_u32_e32 %3, %3, %8\nv_max_u32_e32 %4, %4, %8\nv_max_u32_e32 %5, %5, %8\nv_max_u32_e32 %6, %6, %8\nv_max_u32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k18(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\nv_sub_co_u32_e32 %0, vcc, %0, %8\nv_sub_co_u32_e32 %1, vcc, %1, %8\nv_sub_co_u32_e32 %2, vcc, %2, %8\nv_sub_co_u32_e32 %3, vcc, %3, %8\nv_sub_co_u32_e32 %4, vcc, %4, %8\nv_sub_co_u32_e32 %5, vcc, %5, %8\nv_sub_co_u32_e32 %6, vcc, %6, %8\nv_sub_co_u32_e32 %7, vcc, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43", "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k19(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\nv_mul_u32_u24_e32 %0, %0, %8\nv_mul_u32_u24_e32 %1, %1, %8\nv_mul_u32_u24_e32 %2, %2, %8\nv_mul_u32_u24_e32 %3, %3, %8\nv_mul_u32_u24_e32 %4, %4, %8\nv_mul_u32_u24_e32 %5, %5, %8\nv_mul_u32_u24_e32 %6, %6, %8\nv_mul_u32_u24_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k20(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\nv_mad_u32_u24 %0, %0, %8, %9\nv_mad_u32_u24 %1, %1, %8, %9\nv_mad_u32_u24 %2, %2, %8, %9\nv_mad_u32_u24 %3, %3, %8, %9\nv_mad_u32_u24 %4, %4, %8, %9\nv_mad_u32_u24 %5, %5, %8, %9\nv_mad_u32_u24 %6, %6, %8, %9\nv_mad_u32_u24 %7, %7, %8, %9\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k21(u32* out, u32 s) {
  u64 p0 = threadIdx.x, p1 = p0 * 3, p2 = p0 * 5, p3 = p0 * 7, q0 = p0 ^ 9, q1 = p0 ^ 11, q2 = p0 ^ 13, q3 = p0 ^ 15;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\nv_lshlrev_b64 %[p0], 3, %[q1]\nv_lshlrev_b64 %[p1], 3, %[q2]\nv_lshlrev_b64 %[p2], 3, %[q3]\nv_lshlrev_b64 %[p3], 3, %[q0]\n" : [p0]"+v"(p0), [p1]"+v"(p1), [p2]"+v"(p2), [p3]"+v"(p3), [q0]"+v"(q0), [q1]"+v"(q1), [q2]"+v"(q2), [q3]"+v"(q3) : : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)(p0 ^ p1 ^ p2 ^ p3 ^ q0 ^ q1 ^ q2 ^ q3);
}

__global__ void k22(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\nv_add_f32_e32 %0, %0, %8\nv_add_f32_e32 %1, %1, %8\nv_add_f32_e32 %2, %2, %8\nv_add_f32_e32 %3, %3, %8\nv_add_f32_e32 %4, %4, %8\nv_add_f32_e32 %5, %5, %8\nv_add_f32_e32 %6, %6, %8\nv_add_f32_e32 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k23(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\nv_pk_add_u16 %0, %0, %8\nv_pk_add_u16 %1, %1, %8\nv_pk_add_u16 %2, %2, %8\nv_pk_add_u16 %3, %3, %8\nv_pk_add_u16 %4, %4, %8\nv_pk_add_u16 %5, %5, %8\nv_pk_add_u16 %6, %6, %8\nv_pk_add_u16 %7, %7, %8\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k24(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u, c = threadIdx.x * 5u + 3u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\nv_alignbit_b32 %0, %0, %8, 7\nv_alignbit_b32 %1, %1, %8, 7\nv_alignbit_b32 %2, %2, %8, 7\nv_alignbit_b32 %3, %3, %8, 7\nv_alignbit_b32 %4, %4, %8, 7\nv_alignbit_b32 %5, %5, %8, 7\nv_alignbit_b32 %6, %6, %8, 7\nv_alignbit_b32 %7, %7, %8, 7\n"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(c) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(u32*, u32);
struct K { const char* name; kfn f; int n; };
int main() {
  K ks[] = {
    {"cndmask_e32 vcc(valu)", k0, 64},
    {"cndmask_e32 vcc(salu)", k1, 64},
    {"cndmask_e64 vcc", k2, 64},
    {"cndmask_e64 sgpr(salu)", k3, 64},
    {"cmp_lt_e32 -> vcc", k4, 64},
    {"sub_u32_e32", k5, 64},
    {"or_b32_e32", k6, 64},
    {"and_b32_e32", k7, 64},
    {"not_b32", k8, 64},
    {"lshrrev_e32", k9, 64},
    {"lshrrev imm", k10, 64},
    {"bfe_u32", k11, 64},
    {"bfi_b32", k12, 64},
    {"perm_b32", k13, 64},
    {"lshl_or_b32", k14, 64},
    {"or3_b32", k15, 64},
    {"min_u32_e32", k16, 64},
    {"max_u32_e32", k17, 64},
    {"sub_co_e32 (vcc out)", k18, 64},
    {"mul_u32_u24", k19, 64},
    {"mad_u32_u24", k20, 64},
    {"lshlrev_b64", k21, 64},
    {"add_f32", k22, 64},
    {"pk_add_u16", k23, 64},
    {"alignbit imm", k24, 64}};
  u32* out;
  (void)hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("%-24s %6s %10s %16s\n", "form", "w/SIMD", "ms", "wave-ins/CU-clk");
  for (auto& k : ks) {
    for (int wps : {2, 8}) {
      const int blocks = 256 * wps;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double wins = blocks * 4.0 * ITERS * k.n;
      printf("%-24s %6d %10.3f %16.3f\n", k.name, wps, ms, wins / (ms * 1e-3 * 2.4e9 * 256));
    }
  }
  return 0;
}