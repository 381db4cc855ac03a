// mw_jit.h — support header for specialised (per-program) search kernels.
//
// mythril_amd/jit.py emits one straight-line function per program from the
// compiler's SSA machine IR (mythril_amd/compiler.py, before slot
// allocation): every value is a register array, every constant a literal and
// every leaf descriptor folded into the call.  There is no dispatch, no
// register-file indexing and no spill area: LLVM schedules and allocates the
// whole program for gfx950.
//
// Each helper below has exactly the semantics of the matching interpreter case
// in mw_interp.h (same ALU, same canonicalisation), and the candidate
// generator is the interpreter's (mw_leaf.h), so a specialised kernel returns
// the interpreter's verdict for every candidate index.  tests/test_jit.py
// checks both against the oracle on the CPU (a host build of the generated
// source) and tests/test_gpu_jit.py on gfx950.
#pragma once
#if defined(__HIP_DEVICE_COMPILE__)
#define MW_LEAF_KEY_FENCE(k) asm volatile("" : "+s"(k))
#endif
#include "mw_alu.h"
#include "mw_isa.h"
#include "mw_leaf.h"

namespace mw {
namespace jit {
MW_HD void xor8(const u32 x[8], const u32 y[8], u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = x[k] ^ y[k];
}

// ------------------------------------------------------------------ wide
// MW_ABLATE_*: timing experiments only (tools/ab_c5.py): the op class becomes an
// XOR (wrong results, same data flow), so the time it saves is that class's cost
#if defined(MW_ABLATE_ADD)
#define add8(x, y, r) ((void)xor8(x, y, r), 0u)
#define sub8(x, y, r) ((void)xor8(x, y, r), 0u)
#endif
#if defined(MW_ABLATE_MUL)
#define mul8(x, y, r) xor8(x, y, r)
#endif
MW_HD void w_add(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { add8(x, y, r); canon(r, w); }
MW_HD void w_sub(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { sub8(x, y, r); canon(r, w); }
MW_HD void w_mul(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { mul8(x, y, r); canon(r, w); }
MW_HD void w_and(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = x[k] & y[k];
  canon(r, w);
}
MW_HD void w_or(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = x[k] | y[k];
  canon(r, w);
}
MW_HD void w_xor(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = x[k] ^ y[k];
  canon(r, w);
}
MW_HD void w_not(const u32 x[8], u32 w, u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = ~x[k];
  canon(r, w);
}
#if defined(MW_ABLATE_SHIFT)
MW_HD void w_shl(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { xor8(x, y, r); }
MW_HD void w_lshr(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { xor8(x, y, r); }
MW_HD void w_ashr(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { xor8(x, y, r); }
#else
MW_HD void w_shl(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { wshl(x, y, w, r); canon(r, w); }
MW_HD void w_lshr(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { wlshr(x, y, w, r); canon(r, w); }
MW_HD void w_ashr(const u32 x[8], const u32 y[8], u32 w, u32 r[8]) { washr(x, y, w, r); canon(r, w); }
#endif
// kind: 0 udiv, 1 urem, 2 sdiv, 3 srem, 4 smod (wdiv consumes its operands);
// dc counts the wave's division paths and digit steps (udivrem8)
MW_HD void w_div(int kind, const u32 x[8], const u32 y[8], u32 w, u32 r[8], DivCount& dc) {
#if defined(MW_ABLATE_DIV)
  xor8(x, y, r);
  return;
#endif
  u32 a[8], b[8];
  copy8(a, x);
  copy8(b, y);
  wdiv(kind, a, b, w, r, &dc);
  canon(r, w);
}
MW_HD void w_ite(u32 c, const u32 x[8], const u32 y[8], u32 w, u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = c ? x[k] : y[k];
  canon(r, w);
}
MW_HD void w_shli(const u32 x[8], u32 imm, u32 w, u32 r[8]) { shl8(x, imm, r); canon(r, w); }
MW_HD void w_lshri(const u32 x[8], u32 imm, u32 w, u32 r[8]) { shr8(x, imm, 0u, r); canon(r, w); }
MW_HD void w_zextn(u32 v, u32 w, u32 r[8]) {
  zero8(r);
  r[0] = v;
  canon(r, w);
}
MW_HD void w_sext(const u32 x[8], u32 imm, u32 w, u32 r[8]) {
  copy8(r, x);
  sext8(r, imm);
  canon(r, w);
}
MW_HD void w_sextn(u32 v, u32 imm, u32 w, u32 r[8]) {
  zero8(r);
  r[0] = v;
  sext8(r, imm);
  canon(r, w);
}
MW_HD void w_insn(const u32 x[8], u32 v, u32 imm, u32 w, u32 r[8]) {
  u32 y[8];
  zero8(y);
  y[0] = v;
  shl8(y, imm, r);
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] |= x[k];
  canon(r, w);
}
MW_HD void w_mov(const u32 x[8], u32 w, u32 r[8]) {
  copy8(r, x);
  canon(r, w);
}

// ------------------------------------------------------------------ wide -> narrow
MW_HD u32 n_extractw(const u32 x[8], u32 imm, u32 w) {
  u32 r[8];
  shr8(x, imm, 0u, r);
  return r[0] & nmask(w);
}
MW_HD u32 n_ult(const u32 x[8], const u32 y[8]) { return ult8(x, y) ? 1u : 0u; }
MW_HD u32 n_ule(const u32 x[8], const u32 y[8]) { return ult8(y, x) ? 0u : 1u; }
// signed compare at width w: flip the sign bit (bit w-1) of both, compare unsigned
MW_HD u32 n_scmp(const u32 x_[8], const u32 y_[8], u32 w, bool le) {
  u32 x[8], y[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bit = (int)w - 1 - 32 * k;
    const u32 m = (bit >= 0 && bit < 32) ? (1u << bit) : 0u;
    x[k] = x_[k] ^ m;
    y[k] = y_[k] ^ m;
  }
  return (le ? !ult8(y, x) : ult8(x, y)) ? 1u : 0u;
}
MW_HD u32 n_eq(const u32 x[8], const u32 y[8]) { return eq8(x, y) ? 1u : 0u; }
MW_HD u32 n_umulno(const u32 x[8], const u32 y[8], u32 w) {
  u32 lo[8], hi[8];
  mulhi8(x, y, lo, hi);
  u32 ov = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) ov |= (lo[k] & ~limb_mask(w, k)) | hi[k];
  return ov ? 0u : 1u;
}
MW_HD u32 n_addc(const u32 x[8], const u32 y[8], u32 w) {
  u32 r[8];
  const u32 c = add8(x, y, r);
  u32 bit = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int b = (int)w - 32 * k;
    bit |= (b >= 0 && b < 32) ? ((r[k] >> b) & 1u) : 0u;
  }
  return (w >= 256) ? c : bit;
}

// ------------------------------------------------------------------ narrow (<= 32 bit)
MW_HD u32 nn_add(u32 a, u32 b, u32 w) { return (a + b) & nmask(w); }
MW_HD u32 nn_sub(u32 a, u32 b, u32 w) { return (a - b) & nmask(w); }
MW_HD u32 nn_mul(u32 a, u32 b, u32 w) { return (a * b) & nmask(w); }
MW_HD u32 nn_not(u32 a, u32 w) { return (~a) & nmask(w); }
MW_HD u32 nn_shli(u32 a, u32 imm, u32 w) { return (imm >= 32 ? 0u : (a << imm)) & nmask(w); }
MW_HD u32 nn_lshri(u32 a, u32 imm, u32 w) { return (imm >= 32 ? 0u : (a >> imm)) & nmask(w); }
MW_HD u32 nn_sext(u32 a, u32 imm, u32 w) { return n_sext(a, imm) & nmask(w); }
MW_HD u32 nn_addc(u32 a, u32 b, u32 w) { return (u32)((((u64)a + b) >> w) & 1u); }

// ------------------------------------------------------------------ leaves kept in LDS
// jit.py (lds_leaves > 0) stores the most-used wide leaves of a program in LDS
// at their definition and reloads them at every use, so they occupy no
// registers between uses: at 2 waves/SIMD a lane has 256 registers, and C5's
// 16 leaves alone would take 128.  Layout [slot][half][lane] x 16 B: each
// ds_read_b128 of a wave reads 1 KiB of consecutive 16-byte lane records
// (conflict-free).  Volatile accesses: LLVM may not merge the reloads of one
// leaf into one long-lived copy.  Budget: slots x 8 KiB per 256-thread block.
#ifndef MW_JIT_LDS_SLOTS
#define MW_JIT_LDS_SLOTS 0
#endif
#if MW_JIT_LDS_SLOTS > 0
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ u32x4 mw_jit_lds[MW_JIT_LDS_SLOTS * 2 * 256];
// through an LDS (address space 3) pointer: ds_read/ds_write_b128 with 32-bit
// addresses; a generic pointer would make them flat_load/store (64-bit address
// registers, and sc0 sc1 for the volatile accesses)
typedef volatile __attribute__((address_space(3))) u32x4 lds_u32x4;
MW_HD void lds_put8(u32 slot, const u32 v[8]) {
  lds_u32x4* p = (lds_u32x4*)mw_jit_lds + slot * 512u + threadIdx.x;
  u32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
  p[0] = a;
  p[256] = b;
}
MW_HD void lds_get8(u32 slot, u32 r[8]) {
  lds_u32x4* p = (lds_u32x4*)mw_jit_lds + slot * 512u + threadIdx.x;
  const u32x4 a = p[0], b = p[256];
  r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
  r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
}
#else
static u32 mw_jit_host_lds[MW_JIT_LDS_SLOTS * 8];  // host build: one candidate at a time
MW_HD void lds_put8(u32 slot, const u32 v[8]) {
  for (int k = 0; k < 8; ++k) mw_jit_host_lds[slot * 8 + k] = v[k];
}
MW_HD void lds_get8(u32 slot, u32 r[8]) {
  for (int k = 0; k < 8; ++k) r[k] = mw_jit_host_lds[slot * 8 + k];
}
#endif
#endif

// ------------------------------------------------------------------ control
// wave-wide "no lane alive" (per candidate in the host build)
MW_HD bool none(bool alive) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(alive) == 0ull;
#else
  return !alive;
#endif
}

// Opaque copy of a value: a recomputed term (compiler.py remat) reads its
// operands through it, so LLVM cannot CSE the recomputation with the copy of
// an earlier conjunct and stretch that copy's live range back across both.
MW_HD void fence8(const u32 x[8], u32 r[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r[k] = x[k];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(r[k]));
#endif
  }
}
MW_HD u32 fence1(u32 x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}

// alive &= (v != 0), materialised at this point: without the fence LLVM sinks
// every comparison of an exhaustive body to its single use (the final return),
// keeping all compared wide values live to the end of the program.
MW_HD bool check(bool alive, u32 v) {
  u32 a = (alive && v != 0u) ? 1u : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(a));
#endif
  return a != 0u;
}

// trace rows (host build only; device bodies are instantiated with trace == nullptr)
MW_HD void tstore(u32* trace, u64 stride, u64 idx, u32 row, const u32* v, int n) {
  if (trace)
    for (int k = 0; k < n; ++k) trace[((u64)row + k) * stride + idx] = v[k];
}

// Basic-block boundary for straight-line bodies (jit.py SPLIT_EVERY): a branch
// on a control bit the host never sets (ctl is the launch's flags word), around
// a side effect the compiler must keep.  The empty asm re-defines ctl at every
// boundary, so jump threading cannot prove the later tests false from the first
// one and fold the blocks back together.  Costs one scalar test and branch;
// stops LLVM from scheduling the whole program as one region.
#define MW_JIT_NEVER 0x80000000u
#if defined(__HIP_DEVICE_COMPILE__)
#define JIT_SPLIT()                                        \
  do {                                                     \
    asm volatile("" : "+s"(ctl));                          \
    if (__builtin_expect((ctl & MW_JIT_NEVER) != 0u, 0))   \
      asm volatile("s_nop 0");                             \
  } while (0)
#else
#define JIT_SPLIT() ((void)ctl)
#endif

typedef bool (*body_fn)(const u32* __restrict__, u64, u64, bool, u32, u32*, u64, u64, DivCount&);

// stage bits of a launch: a program is one part (FIRST|LAST) or several parts
// launched in order over the same candidates, passing each candidate's alive
// bit through a buffer (jit.py split_ssa: parts end at conjunct boundaries)
#define MW_JIT_FIRST 1u
#define MW_JIT_LAST 2u

#if !defined(MW_JIT_HOST)
// One 256-candidate chunk per block (chunk = chunk0 + blockIdx.x), with the
// interpreter's result protocol (mw_search_kernel): per-wave ballot -> lowest
// satisfying lane -> atomicMin on the program's witness index; optional
// per-candidate verdicts (mg_eval_generated).  No grid-stride loop on purpose:
// inside a loop LLVM hoists every leaf's Philox key schedule (uniform, loop
// invariant) into SGPRs and spills hundreds of them into VGPR lanes.
// A part that is not LAST stores alive bits (index cand - begin) instead; a
// part that is not FIRST starts from them.
template <body_fn BODY>
__device__ __attribute__((always_inline)) inline void search(const u32* __restrict__ pool, u64 seed, u64 begin,
                                                             u64 count, u64 chunk0, u32 flags,
                                                             u64* __restrict__ out_min, u64* __restrict__ counter,
                                                             u32* __restrict__ verdict, u32* __restrict__ alivebuf,
                                                             u32 stage) {
  const u64 base = begin + (chunk0 + blockIdx.x) * 256;
  if ((flags & MW_FLAG_STOP_AFTER_HIT) && stage == (MW_JIT_FIRST | MW_JIT_LAST)) {
    const u64 m = __hip_atomic_load(out_min, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (m <= base) return;
  }
  const u32 lane = threadIdx.x & 63u;
  const u64 cand = base + threadIdx.x;
  const bool valid = cand < begin + count;
  bool in = valid;
  if (!(stage & MW_JIT_FIRST) && valid) in = alivebuf[cand - begin] != 0u;
  DivCount dc;
  const bool ok = BODY(pool, seed, cand, in, flags, nullptr, 0, 0, dc);
  const u64 nvalid = (u64)__popcll(__ballot(valid));
  // MW_FLAG_NO_COUNT (a timed exhaustive launch): no counter atomics at all
  const bool counting = !(flags & MW_FLAG_NO_COUNT);
  // this block's counter stripe (mw_alu.h MW_CTR_STRIPES)
  counter += MW_CTR_STRIPE_WORDS * (1u + (blockIdx.x & (MW_CTR_STRIPES - 1u)));
  if (counting && lane == 0 && nvalid)   // division paths x lanes (mg_stats.lane_div_*)
    add_div_counts(counter, dc, nvalid);
  if (!(stage & MW_JIT_LAST)) {
    if (valid) alivebuf[cand - begin] = ok ? 1u : 0u;
    return;
  }
  if (verdict && valid) verdict[cand - begin] = ok ? 1u : 0u;
  const u64 hit = __ballot(ok);
  if (hit) {
    const u32 first = (u32)__ffsll((unsigned long long)hit) - 1u;
    // the atomic only when it can lower the minimum: exhaustive searches of
    // dense programs would otherwise queue one per wave on this one address
    if (lane == first && cand < __hip_atomic_load(out_min, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin((unsigned long long*)out_min, (unsigned long long)cand);
  }
  if (counting && lane == 0 && nvalid) atomicAdd((unsigned long long*)counter, (unsigned long long)nvalid);
}

// <name>_x: exhaustive; <name>_e: per-wave early exit after a failing CHECK.
// <name>_sig: FNV-1a 64 of the whole program's words, checked by
// mg_prog_attach_kernel; <name>_part / <name>_nparts: this module's part.
// waves per SIMD the kernel is compiled for: 2 (<= 256 registers per lane) by
// default, 1 gives 512 registers (AGPRs as spill space).
#ifndef MW_JIT_WAVES
#define MW_JIT_WAVES 2
#endif
#define MW_JIT_KERNEL(NAME, SUFFIX, BODY, EARLY)                                                     \
  extern "C" __global__ __launch_bounds__(256, MW_JIT_WAVES) void NAME##SUFFIX(                      \
      const mw::u32* __restrict__ pool, mw::u64 seed, mw::u64 begin, mw::u64 count, mw::u64 chunk0,  \
      mw::u32 flags, mw::u64* __restrict__ out_min, mw::u64* __restrict__ counter,                   \
      mw::u32* __restrict__ verdict, mw::u32* __restrict__ alivebuf, mw::u32 stage) {                \
    mw::jit::search<BODY<EARLY>>(pool, seed, begin, count, chunk0, flags, out_min, counter, verdict, \
                                 alivebuf, stage);                                                   \
  }
#define MW_JIT_SIG(NAME, SIG) extern "C" __device__ const mw::u64 NAME##_sig = SIG;
#define MW_JIT_PART(NAME, K, N)                                \
  extern "C" __device__ const mw::u32 NAME##_part = K;         \
  extern "C" __device__ const mw::u32 NAME##_nparts = N;
#else
#define MW_JIT_KERNEL(NAME, SUFFIX, BODY, EARLY)
#define MW_JIT_SIG(NAME, SIG)
#define MW_JIT_PART(NAME, K, N)
#endif

// host build (tests only): verdicts (+ trace rows) of candidates [begin, begin+count)
#if defined(MW_JIT_HOST)
#define MW_JIT_HOST_ENTRY(NAME, BODY)                                                                \
  extern "C" int NAME##_host(const mw::u32* pool, mw::u64 seed, mw::u64 begin, mw::u64 count,        \
                             mw::u32 early, mw::u32* verdict, mw::u32* trace) {                      \
    for (mw::u64 i = 0; i < count; ++i) {                                                            \
      mw::DivCount ds;                                                                               \
      verdict[i] = (early ? BODY<true>(pool, seed, begin + i, true, 0u, trace, count, i, ds)             \
                          : BODY<false>(pool, seed, begin + i, true, 0u, trace, count, i, ds)) ? 1u : 0u; \
    }                                                                                                \
    return 0;                                                                                        \
  }
#else
#define MW_JIT_HOST_ENTRY(NAME, BODY)
#endif

}  // namespace jit
}  // namespace mw
