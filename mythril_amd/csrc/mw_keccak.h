// mw_keccak.h — Keccak-256 (original 0x01 padding, rate 136 B) for one message
// per lane.  Replaces _pysha3.keccak_256 on the concrete-hash path
// (mythril/support/support_utils.py:50-59; keccak_function_manager.py:57-69).
// State: 25 x u64 lanes in VGPRs, fully unrolled permutation (static indices).
#pragma once
#include "mw_alu.h"

namespace mw {

// 64-bit rotate by a constant 0 < n < 64 on 32-bit halves: two v_alignbit_b32
// (LLVM otherwise emits two 64-bit shifts and two ORs)
MW_HD u64 rotl64(u64 x, int n) {
  u32 lo = (u32)x, hi = (u32)(x >> 32);
  if (n >= 32) {
    const u32 t = lo;
    lo = hi;
    hi = t;
    n -= 32;
  }
  if (n == 0) return (u64)lo | ((u64)hi << 32);
  const u32 nh = alignbit(hi, lo, 32u - (u32)n), nl = alignbit(lo, hi, 32u - (u32)n);
  return (u64)nl | ((u64)nh << 32);
}

// gfx950 3-input logic (v_bitop3_b32; truth table over src0=0xF0, src1=0xCC,
// src2=0xAA): a^b^c = 0x96, a^(~b&c) = 0xD2.  One instruction per 32-bit half
// where plain C takes two (theta's column parity, chi).
#if defined(__HIP_DEVICE_COMPILE__)
template <unsigned TT>
__device__ __forceinline__ u64 bitop3_64(u64 a, u64 b, u64 c) {
  const u32 lo = __builtin_amdgcn_bitop3_b32((u32)a, (u32)b, (u32)c, TT);
  const u32 hi = __builtin_amdgcn_bitop3_b32((u32)(a >> 32), (u32)(b >> 32), (u32)(c >> 32), TT);
  return (u64)lo | ((u64)hi << 32);
}
MW_HD u64 xor3_64(u64 a, u64 b, u64 c) { return bitop3_64<0x96>(a, b, c); }
MW_HD u64 chi_64(u64 a, u64 b, u64 c) { return bitop3_64<0xD2>(a, b, c); }
#else
MW_HD u64 xor3_64(u64 a, u64 b, u64 c) { return a ^ b ^ c; }
MW_HD u64 chi_64(u64 a, u64 b, u64 c) { return a ^ (~b & c); }
#endif

MW_HD void keccak_f1600(u64 A[25]) {
  const u64 RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
      0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
      0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  // rho offsets and pi lane order along the (x,y) -> (y, 2x+3y) cycle starting at lane 1
  const int RHO[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                       27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
  const int PI[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                      15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
#pragma unroll 4
  for (int rnd = 0; rnd < 24; ++rnd) {
    u64 C[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = xor3_64(xor3_64(A[x], A[x + 5], A[x + 10]), A[x + 15], A[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      const u64 c1 = C[(x + 4) % 5], r1 = rotl64(C[(x + 1) % 5], 1);
#pragma unroll
      for (int y = 0; y < 25; y += 5) A[y + x] = xor3_64(A[y + x], c1, r1);
    }
    u64 t = A[1];
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      int j = PI[i];
      u64 tmp = A[j];
      A[j] = rotl64(t, RHO[i]);
      t = tmp;
    }
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      u64 r0 = A[y], r1 = A[y + 1], r2 = A[y + 2], r3 = A[y + 3], r4 = A[y + 4];
      A[y] = chi_64(r0, r1, r2);
      A[y + 1] = chi_64(r1, r2, r3);
      A[y + 2] = chi_64(r2, r3, r4);
      A[y + 3] = chi_64(r3, r4, r0);
      A[y + 4] = chi_64(r4, r0, r1);
    }
    A[0] ^= RC[rnd];
  }
}

// absorb + squeeze one message; out = 32 digest bytes as 4 little-endian u64 lanes.
// Whole 8-byte state lanes of a 4-byte-aligned message are read as two dwords;
// only the lane that straddles the end of the message (and unaligned messages)
// goes byte by byte.  Padding (0x01 ... 0x80, rate 136) is XORed in afterwards.
MW_HD void keccak256_msg(const uint8_t* __restrict__ msg, u32 len, u64 out[4]) {
  u64 A[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) A[i] = 0;
  const bool aligned = (((uintptr_t)msg) & 3u) == 0u;
  const u32 nblk = len / 136u + 1u;
  for (u32 blk = 0; blk < nblk; ++blk) {
    const u32 base = blk * 136u;
#pragma unroll
    for (int lane = 0; lane < 17; ++lane) {
      const u32 p0 = base + (u32)(lane * 8);
      u64 v = 0;
      if (aligned && p0 + 8u <= len) {
        const u32* w = (const u32*)(msg + p0);
        v = (u64)w[0] | ((u64)w[1] << 32);
      } else if (p0 < len) {
        for (u32 b = 0; b < 8u && p0 + b < len; ++b) v |= (u64)msg[p0 + b] << (8 * b);
      }
      A[lane] ^= v;
    }
    if (blk + 1u == nblk) {  // pad10*1 with Keccak's domain byte 0x01
      const u32 r = len - base;  // 0..135 message bytes in this block
#pragma unroll
      for (int lane = 0; lane < 17; ++lane) {
        u64 pad = ((u32)lane == r / 8u) ? (0x01ull << (8u * (r % 8u))) : 0ull;
        if (lane == 16) pad ^= 0x80ull << 56;
        A[lane] ^= pad;
      }
    }
    keccak_f1600(A);
  }
  out[0] = A[0];
  out[1] = A[1];
  out[2] = A[2];
  out[3] = A[3];
}

}  // namespace mw
