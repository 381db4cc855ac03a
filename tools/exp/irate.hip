// Experiment: per-instruction issue rates on gfx950 for the multi-limb ALU.
// Each kernel runs ITERS loop trips of an unrolled body of K instructions per
// lane over independent accumulators (or one dependent chain where named), at
// a given waves/SIMD (block size x blocks).  Reports wave-instructions per
// CU-cycle (2.0 = the guide's VALU peak: 4 SIMD x 1 wave64 op per 2 cycles).
// Hazards inside inline asm are padded by hand (VALU SGPR write -> VALU read:
// 2 wait states).  Build: hipcc --offload-arch=gfx950 -O3 -o tools/exp/irate tools/exp/irate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32;
typedef uint64_t u64;

#define ITERS 4096

#define R8(X) X X X X X X X X
// v_add_u32: 8 independent chains
__global__ void k_add(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                    "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "s"(s));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// v_mad_u64_u32: 8 independent accumulators (carry out to an unused SGPR pair)
__global__ void k_mad(u32* out, u32 s) {
  u64 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 m = threadIdx.x * 2654435761u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n v_mad_u64_u32 %1, s[40:41], %8, %9, %1\n"
                    "v_mad_u64_u32 %2, s[40:41], %8, %9, %2\n v_mad_u64_u32 %3, s[40:41], %8, %9, %3\n"
                    "v_mad_u64_u32 %4, s[40:41], %8, %9, %4\n v_mad_u64_u32 %5, s[40:41], %8, %9, %5\n"
                    "v_mad_u64_u32 %6, s[40:41], %8, %9, %6\n v_mad_u64_u32 %7, s[40:41], %8, %9, %7\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(m), "s"(s)
                 : "s40", "s41");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
// v_mul_hi_u32: 8 independent chains
__global__ void k_mulhi(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
                    "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "s"(s));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// v_lshl_add_u64: 8 independent 64-bit accumulators
__global__ void k_lshladd(u32* out, u32 s) {
  u64 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u64 m = threadIdx.x * 2654435761ull;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_lshl_add_u64 %0, %0, 0, %8\n v_lshl_add_u64 %1, %1, 0, %8\n v_lshl_add_u64 %2, %2, 0, %8\n"
                    "v_lshl_add_u64 %3, %3, 0, %8\n v_lshl_add_u64 %4, %4, 0, %8\n v_lshl_add_u64 %5, %5, 0, %8\n"
                    "v_lshl_add_u64 %6, %6, 0, %8\n v_lshl_add_u64 %7, %7, 0, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(m));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
// 256-bit add as add_co + 7 addc through VCC, s_nop 1 between links (one chain)
__global__ void k_addc_nop(u32* out, u32 s) {
  u32 a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_co_u32 %0, vcc, %0, %8\n s_nop 1\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n s_nop 1\n"
                    "v_addc_co_u32 %2, vcc, %2, %8, vcc\n s_nop 1\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n s_nop 1\n"
                    "v_addc_co_u32 %4, vcc, %4, %8, vcc\n s_nop 1\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n s_nop 1\n"
                    "v_addc_co_u32 %6, vcc, %6, %8, vcc\n s_nop 1\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n")
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                 : "v"(s)
                 : "vcc");
  }
  u32 x = 0;
  for (int k = 0; k < 8; ++k) x ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// two 256-bit add chains interleaved through s[40:41] / s[42:43] with one wait state between
__global__ void k_addc_x2(u32* out, u32 s) {
  u32 a[8], b[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k, b[k] = a[k] ^ 5u;
#define L2(K) "v_addc_co_u32 %" #K ", s[40:41], %" #K ", %16, s[40:41]\n s_nop 0\n v_addc_co_u32 %" #K "+8, s[42:43], %" #K "+8, %16, s[42:43]\n s_nop 0\n"
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_co_u32 %0, s[40:41], %0, %16\n v_add_co_u32 %8, s[42:43], %8, %16\n s_nop 0\n"
                    "v_addc_co_u32 %1, s[40:41], %1, %16, s[40:41]\n v_addc_co_u32 %9, s[42:43], %9, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %2, s[40:41], %2, %16, s[40:41]\n v_addc_co_u32 %10, s[42:43], %10, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %3, s[40:41], %3, %16, s[40:41]\n v_addc_co_u32 %11, s[42:43], %11, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %4, s[40:41], %4, %16, s[40:41]\n v_addc_co_u32 %12, s[42:43], %12, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %5, s[40:41], %5, %16, s[40:41]\n v_addc_co_u32 %13, s[42:43], %13, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %6, s[40:41], %6, %16, s[40:41]\n v_addc_co_u32 %14, s[42:43], %14, %16, s[42:43]\n s_nop 0\n"
                    "v_addc_co_u32 %7, s[40:41], %7, %16, s[40:41]\n v_addc_co_u32 %15, s[42:43], %15, %16, s[42:43]\n s_nop 0\n")
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
                   "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7])
                 : "v"(s)
                 : "s40", "s41", "s42", "s43");
  }
  u32 x = 0;
  for (int k = 0; k < 8; ++k) x ^= a[k] ^ b[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// 256-bit add with no flags: 4 x v_lshl_add_u64 per 64-bit limb pair... (sum only, carries via v_add3 of compare results)
__global__ void k_nop(u32* out, u32 s) {
  u32 a0 = threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n") : "+v"(a0));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
// v_cndmask_b32 with an SGPR mask written long before: 8 independent chains
__global__ void k_cnd(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = a0 * 7u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_cmp_lt_u32 s[40:41], %8, %9\n s_nop 1\n" R8(
                     "v_cndmask_b32 %0, %0, %8, s[40:41]\n v_cndmask_b32 %1, %1, %8, s[40:41]\n"
                     "v_cndmask_b32 %2, %2, %8, s[40:41]\n v_cndmask_b32 %3, %3, %8, s[40:41]\n"
                     "v_cndmask_b32 %4, %4, %8, s[40:41]\n v_cndmask_b32 %5, %5, %8, s[40:41]\n"
                     "v_cndmask_b32 %6, %6, %8, s[40:41]\n v_cndmask_b32 %7, %7, %8, s[40:41]\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b), "v"(s)
                 : "s40", "s41");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// dependent v_add_u32 chain (latency): one accumulator
__global__ void k_dep(u32* out, u32 s) {
  u32 a0 = threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                    "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
                 : "+v"(a0)
                 : "s"(s));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
// dependent v_mad_u64_u32 chain (latency): one accumulator
__global__ void k_maddep(u32* out, u32 s) {
  u64 a0 = threadIdx.x;
  u32 m = threadIdx.x * 2654435761u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                    "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                    "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                    "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n")
                 : "+v"(a0)
                 : "v"(m), "s"(s)
                 : "s40", "s41");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)a0;
}


// v_add_u32 (VOP2, 4-byte encoding) with a VGPR operand: 8 independent chains
__global__ void k_add_e32(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_u32_e32 %0, %0, %8\n v_add_u32_e32 %1, %1, %8\n v_add_u32_e32 %2, %2, %8\n v_add_u32_e32 %3, %3, %8\n"
                    "v_add_u32_e32 %4, %4, %8\n v_add_u32_e32 %5, %5, %8\n v_add_u32_e32 %6, %6, %8\n v_add_u32_e32 %7, %7, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// the same add in the VOP3 (8-byte) encoding with VGPR operands
__global__ void k_add_e64(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_add_u32_e64 %0, %0, %8\n v_add_u32_e64 %1, %1, %8\n v_add_u32_e64 %2, %2, %8\n v_add_u32_e64 %3, %3, %8\n"
                    "v_add_u32_e64 %4, %4, %8\n v_add_u32_e64 %5, %5, %8\n v_add_u32_e64 %6, %6, %8\n v_add_u32_e64 %7, %7, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// v_xor_b32 (VOP2) with a VGPR operand
__global__ void k_xor_e32(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 b = blockIdx.x | 1u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_xor_b32_e32 %0, %0, %8\n v_xor_b32_e32 %1, %1, %8\n v_xor_b32_e32 %2, %2, %8\n v_xor_b32_e32 %3, %3, %8\n"
                    "v_xor_b32_e32 %4, %4, %8\n v_xor_b32_e32 %5, %5, %8\n v_xor_b32_e32 %6, %6, %8\n v_xor_b32_e32 %7, %7, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// v_mad_u64_u32 with VGPR operands only
__global__ void k_mad_v(u32* out, u32 s) {
  u64 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  u32 m = threadIdx.x * 2654435761u, b = blockIdx.x | 1u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n v_mad_u64_u32 %1, s[40:41], %8, %9, %1\n"
                    "v_mad_u64_u32 %2, s[40:41], %8, %9, %2\n v_mad_u64_u32 %3, s[40:41], %8, %9, %3\n"
                    "v_mad_u64_u32 %4, s[40:41], %8, %9, %4\n v_mad_u64_u32 %5, s[40:41], %8, %9, %5\n"
                    "v_mad_u64_u32 %6, s[40:41], %8, %9, %6\n v_mad_u64_u32 %7, s[40:41], %8, %9, %7\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(m), "v"(b)
                 : "s40", "s41");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
// v_mov_b32 (VOP1) VGPR to VGPR
__global__ void k_mov(u32* out, u32 s) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(R8("v_mov_b32_e32 %0, %1\n v_mov_b32_e32 %1, %2\n v_mov_b32_e32 %2, %3\n v_mov_b32_e32 %3, %4\n"
                    "v_mov_b32_e32 %4, %5\n v_mov_b32_e32 %5, %6\n v_mov_b32_e32 %6, %7\n v_mov_b32_e32 %7, %0\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(u32*, u32);
struct K {
  const char* name;
  kfn f;
  int insns_per_iter;  // wave instructions per loop trip (VALU + s_nop)
};

int main() {
  K ks[] = {{"v_add_u32 x8", k_add, 64},        {"v_mad_u64_u32 x8", k_mad, 64},
            {"v_mul_hi_u32 x8", k_mulhi, 64},   {"v_lshl_add_u64 x8", k_lshladd, 64},
            {"addc chain+nop1 (8 VALU+7 nop)", k_addc_nop, 120},
            {"2 addc chains+nop0 (16 VALU+8 nop)", k_addc_x2, 192},
            {"s_nop 0", k_nop, 64},               {"v_cndmask x8", k_cnd, 66},
            {"dep v_add_u32", k_dep, 64},         {"dep v_mad_u64_u32", k_maddep, 64},
            {"v_add_u32_e32 (vgpr) x8", k_add_e32, 64}, {"v_add_u32_e64 (vgpr) x8", k_add_e64, 64},
            {"v_xor_b32_e32 x8", k_xor_e32, 64},      {"v_mad_u64_u32 (vgpr) x8", k_mad_v, 64},
            {"v_mov_b32_e32 x8", k_mov, 64}};
  u32* out;
  hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int cus = 256;
  printf("%-38s %6s %12s %14s %14s\n", "kernel", "w/SIMD", "ms", "wave-ins/CU-clk", "cyc/ins/wave");
  for (auto& k : ks) {
    for (int wps : {1, 2, 4, 8}) {
      const int blocks = cus * wps;  // 256-thread blocks: 4 waves = one per SIMD
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double waves = blocks * 4.0;
      const double wins = waves * (double)ITERS * k.insns_per_iter;
      const double clk = ms * 1e-3 * 2.4e9;
      const double per_cu = wins / (clk * cus);
      // cycles between a wave's instructions: SIMD clocks x resident waves / instructions issued
      const double cpi = clk * wps / ((double)ITERS * k.insns_per_iter);
      printf("%-38s %6d %12.3f %14.3f %14.2f\n", k.name, wps, ms, per_cu, cpi);
    }
  }
  hipFree(out);
  return 0;
}
