// mw_leaf.h — on-device candidate generation (never materialised in HBM).
//
// Candidate index c (u64) -> value of each free variable ("leaf": sender_N,
// call_valueN, N_calldata bytes, calldatasize, storage/balance reads,
// keccak UF results — the leaf schema of SURVEY.md §8a row A8,
// mythril/laser/ethereum/transaction/symbolic.py:118-136, calldata.py:214-215).
//   random leaf: w > 32: Philox4x32-10(key=(seed_lo ^ id, seed_hi), ctr=(c_lo, c_hi, blk, 0)),
//                blk 0 -> limbs 0..3, blk 1 -> limbs 4..7, masked to width;
//                w <= 32: fmix64(c ^ seed ^ id * 0xC2B2AE3D27D4EB4F), masked to width
//   pool leaf:   digit = (c >> shift) & (2^bits - 1); entry = pool[digit];
//                entry flag RANDOM -> random value above, else the constant.
//   interleaved: digit bit b = index bit (shift + b*stride)  (Morton order: indices
//                below 2^(n*k) cover every combination of the first 2^k entries
//                of n pools, so the strongest proposals are tried together first)
//   hashed pool: digit = fmix64(c ^ (salt * 0x9E3779B97F4A7C15)) & (2^bits - 1)
//                (MurmurHash3 finalizer), then as a pool leaf: samples large
//                pools when the index bits cannot enumerate every leaf.
// Restated independently in oracle/philox.py (pinned by Random123 KATs).
#pragma once
#include "mw_alu.h"
#include "mw_isa.h"

// Hook for specialised kernels (mw_jit.h): pins a leaf's Philox key where the
// leaf is generated, so LLVM cannot hoist every leaf's key schedule to the
// top of a straight-line kernel and spill it.  No-op for the interpreter.
#ifndef MW_LEAF_KEY_FENCE
#define MW_LEAF_KEY_FENCE(k) ((void)0)
#endif

namespace mw {

MW_HD void philox4x32_10(u32 c[4], u32 k0, u32 k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    u64 p0 = (u64)0xD2511F53u * c[0];
    u64 p1 = (u64)0xCD9E8D57u * c[2];
    u32 hi0 = (u32)(p0 >> 32), lo0 = (u32)p0;
    u32 hi1 = (u32)(p1 >> 32), lo1 = (u32)p1;
    u32 n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

MW_HD u64 fmix64(u64 h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

// MW_ABLATE_* (timing experiments only, tools/leaf_ablate.py; wrong values):
//   LEAF    every leaf is (u32)cand ^ id in limb 0 (no digit, gather or Philox)
//   PHILOX  random leaves are one multiply-xor of the index (no Philox rounds)
//   DIGIT   interleaved digits read as a plain bit-field (no per-bit loop)
//
// Random leaf value: w > 32 Philox4x32-10 blocks 0 and (w > 128) 1; w <= 32
// (calldata bytes, Bools) one MurmurHash3 finalizer of index ^ seed ^ salt,
// a tenth of Philox's work (oracle/philox.py random_leaf restates both).
MW_HD void random_leaf(u32 id, u32 w, u64 seed, u64 cand, u32 out[8]) {
#if defined(MW_ABLATE_PHILOX)
  out[0] = ((u32)cand ^ id) * 0x9E3779B9u;
  out[1] = ((u32)(cand >> 32) ^ id) * 0x85EBCA6Bu;
#pragma unroll
  for (int k = 2; k < 8; ++k) out[k] = out[k - 2] ^ (u32)seed;
  canon(out, w);
  return;
#endif
  if (w <= 32u) {
    out[0] = (u32)fmix64(cand ^ seed ^ ((u64)id * 0xC2B2AE3D27D4EB4Full));
#pragma unroll
    for (int k = 1; k < 8; ++k) out[k] = 0u;
    canon(out, w);
    return;
  }
  u32 k0 = (u32)seed ^ id, k1 = (u32)(seed >> 32);
  MW_LEAF_KEY_FENCE(k0);
  MW_LEAF_KEY_FENCE(k1);
  u32 c[4] = {(u32)cand, (u32)(cand >> 32), 0u, 0u};
  philox4x32_10(c, k0, k1);
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
  if (w > 128) {
    u32 d[4] = {(u32)cand, (u32)(cand >> 32), 1u, 0u};
    philox4x32_10(d, k0, k1);
    out[4] = d[0]; out[5] = d[1]; out[6] = d[2]; out[7] = d[3];
  } else {
    out[4] = out[5] = out[6] = out[7] = 0u;
  }
  canon(out, w);
}


// Candidate value of one leaf from its descriptor fields (the interpreter
// reads them from the leaf table below; specialised kernels, mw_jit.h, pass
// them as literals).
MW_HD void leaf_fields(u32 w, u32 kind, u32 id, u32 shift, u32 bits, u32 poff, u32 stride,
                       const u32* __restrict__ pool, u64 seed, u64 cand, u32 out[8]) {
#if defined(MW_ABLATE_LEAF)
  out[0] = (u32)cand ^ id;
#pragma unroll
  for (int k = 1; k < 8; ++k) out[k] = 0u;
  canon(out, w);
  return;
#endif
#if defined(MW_ABLATE_DIGIT)
  if (kind == 3u) kind = 1u;
#endif
  if (kind >= 1u && kind <= 3u) {
    u32 digit;
    if (kind == 3u) {
      digit = 0;
      for (u32 b = 0; b < bits; ++b) digit |= (u32)((cand >> (shift + b * stride)) & 1u) << b;
    } else {
      const u64 src = kind == 1u ? (cand >> shift) : fmix64(cand ^ ((u64)id * 0x9E3779B97F4A7C15ull));
      digit = (u32)src & ((bits >= 32) ? 0xffffffffu : ((1u << bits) - 1u));
    }
    const u32* e = pool + poff + (u64)digit * MW_POOL_ENTRY_WORDS_OF(w);
    if (w < 32u) {   // one-word narrow entry
      const u32 x = e[0];
      if (x & MW_POOL_NARROW_RANDOM) {
        random_leaf(id, w, seed, cand, out);
      } else {
        out[0] = x;
#pragma unroll
        for (int k = 1; k < 8; ++k) out[k] = 0u;
      }
    } else if (e[0] & 1u) {
      random_leaf(id, w, seed, cand, out);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = e[1 + k];
      canon(out, w);
    }
  } else {
    random_leaf(id, w, seed, cand, out);
  }
}

// leaf: MW_LEAF_WORDS words (uniform); pool: per-lane gather
MW_HD void leaf_value(const u32* __restrict__ leaf_, const u32* __restrict__ pool, u64 seed,
                      u64 cand, u32 out[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __attribute__((address_space(4))) u32* leaf = (const __attribute__((address_space(4))) u32*)leaf_;
#else
  const u32* leaf = leaf_;
#endif
  const u32 w = leaf[MW_LEAF_WIDTH];
  const u32 id = leaf[MW_LEAF_ID];
#if defined(MW_ABLATE_LEAF)
  out[0] = (u32)cand ^ id;
#pragma unroll
  for (int k = 1; k < 8; ++k) out[k] = 0u;
  canon(out, w);
  return;
#endif
#if defined(MW_ABLATE_DIGIT)
  const u32 kind = leaf[MW_LEAF_KIND] == 3u ? 1u : leaf[MW_LEAF_KIND];
#else
  const u32 kind = leaf[MW_LEAF_KIND];
#endif
  if (kind >= 1u && kind <= 3u) {
    const u32 bits = leaf[MW_LEAF_BITS];
    u32 digit;
    if (kind == 3u) {
      const u32 sh = leaf[MW_LEAF_SHIFT], st = leaf[MW_LEAF_STRIDE];
      digit = 0;
      for (u32 b = 0; b < bits; ++b) digit |= (u32)((cand >> (sh + b * st)) & 1u) << b;
    } else {
      const u64 src = kind == 1u ? (cand >> leaf[MW_LEAF_SHIFT])
                                 : fmix64(cand ^ ((u64)id * 0x9E3779B97F4A7C15ull));
      digit = (u32)src & ((bits >= 32) ? 0xffffffffu : ((1u << bits) - 1u));
    }
    const u32* e = pool + leaf[MW_LEAF_POOL] + (u64)digit * MW_POOL_ENTRY_WORDS_OF(w);
    if (w < 32u) {  // narrow leaf (calldata bytes, Bools): one-word entry
      const u32 x = e[0];
      if (x & MW_POOL_NARROW_RANDOM) {
        random_leaf(id, w, seed, cand, out);
      } else {
        out[0] = x;
#pragma unroll
        for (int k = 1; k < 8; ++k) out[k] = 0u;
      }
    } else if (e[0] & 1u) {
      random_leaf(id, w, seed, cand, out);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = e[1 + k];
      canon(out, w);
    }
  } else {
    random_leaf(id, w, seed, cand, out);
  }
}

}  // namespace mw
