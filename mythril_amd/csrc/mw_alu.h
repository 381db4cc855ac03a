// mw_alu.h — multi-limb bitvector ALU for the witness interpreter.
//
// One candidate per lane: a <=256-bit value is 8 x u32 limbs held in VGPRs
// (limb 0 least significant); <=32-bit values are a single u32.  Semantics are
// SMT-LIB 2.6 (z3 hi_div0=true), i.e. what z3 gives the terms Mythril builds:
//   bvadd/bvsub/bvmul/bvsdiv     mythril/laser/smt/bitvec.py:126-166
//   bvand/bvor/bvxor             bitvec.py:168-199
//   bvslt/bvsgt/bvsle/bvsge      bitvec.py:201-243
//   bvshl/bvashr, LShR           bitvec.py:295-309, bitvec_helper.py:30-31
//   UDiv/URem/SRem               bitvec_helper.py:153-180
//   BVMulNoOverflow(unsigned)    bitvec_helper.py:211-224
// Division by zero: udiv -> all-ones, urem -> dividend, sdiv -> (s<0 ? 1 : -1),
// srem/smod -> dividend.  Shifts by >= width: shl/lshr -> 0, ashr -> sign fill.
//
// Written as portable C++ (__host__ __device__) so the identical code is
// checked on the CPU by tests/test_host_emulator.py before it runs on gfx950.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define MW_HD __host__ __device__ __attribute__((always_inline)) inline

// wave-wide "any lane": guards rarely needed corrections so the wave branches
// over them instead of issuing them under an all-zero exec mask (LLVM only
// skips masked blocks longer than ~12 instructions)
#if defined(__HIP_DEVICE_COMPILE__)
#define MW_ANY(c) (__ballot(c) != 0ull)
#else
#define MW_ANY(c) (c)
#endif
// Branch weights for the division's rare paths (short and limb-aligned
// divisors, add-backs): LLVM then places them after the kernel's hot code
// instead of in line, so the straight-line code the waves stream through
// holds about a third of the instructions it would (C5: 384 inlined
// divisions, two thirds of the code object in their cold paths).
#if defined(MW_DIV_NO_HINTS)
#define MW_RARE(c) (c)
#define MW_USUAL(c) (c)
#else
#define MW_RARE(c) __builtin_expect(!!(c), 0)
#define MW_USUAL(c) __builtin_expect(!!(c), 1)
#endif

namespace mw {
typedef uint32_t u32;
typedef uint64_t u64;

MW_HD u32 addc(u32 a, u32 b, u32& c) {
  u32 co;
  u32 r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
}
MW_HD u32 subb(u32 a, u32 b, u32& br) {
  u32 bo;
  u32 r = __builtin_subc(a, b, br, &bo);
  br = bo;
  return r;
}

// mask of limb k of a w-bit value (branch-free, so a uniform w stays on the SALU)
MW_HD u32 limb_mask(u32 w, int k) {
  const int lo = 32 * k;
  const int rem = (int)w - lo;  // bits of this limb that belong to the value
  const u32 part = 0xffffffffu >> ((32 - (rem > 0 ? (rem < 32 ? rem : 32) : 32)) & 31);
  return rem >= 32 ? 0xffffffffu : (rem > 0 ? part : 0u);
}
MW_HD u32 nmask(u32 w) { return w >= 32 ? 0xffffffffu : ((1u << w) - 1u); }

MW_HD void canon(u32 r[8], u32 w) {
  if (w < 256) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] &= limb_mask(w, k);
  }
}

MW_HD void copy8(u32 d[8], const u32 s[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = s[k];
}
MW_HD void zero8(u32 d[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = 0;
}

// ---------------------------------------------------------------- add / sub
MW_HD u32 add8(const u32 a[8], const u32 b[8], u32 r[8]) {
  u32 c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = addc(a[k], b[k], c);
  return c;
}
MW_HD u32 sub8(const u32 a[8], const u32 b[8], u32 r[8]) {
  u32 br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = subb(a[k], b[k], br);
  return br;
}
// borrow of a - b  ==  a <u b
MW_HD bool ult8(const u32 a[8], const u32 b[8]) {
  u32 br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) (void)subb(a[k], b[k], br);
  return br != 0;
}
MW_HD bool eq8(const u32 a[8], const u32 b[8]) {
  u32 x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x |= a[k] ^ b[k];
  return x == 0;
}
MW_HD bool is_zero8(const u32 a[8]) {
  u32 x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x |= a[k];
  return x == 0;
}

// ---------------------------------------------------------------- multiply
// low 256 bits of a*b (product scanning by rows)
MW_HD void mul8(const u32 a[8], const u32 b[8], u32 r[8]) {
  u32 acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u32 carry = 0;
#pragma unroll
    for (int j = 0; j < 8 - i; ++j) {
      if (i + j < 7) {
        u64 p = (u64)a[i] * b[j] + acc[i + j] + carry;
        acc[i + j] = (u32)p;
        carry = (u32)(p >> 32);
      } else {
        acc[i + j] += a[i] * b[j] + carry;
      }
    }
  }
  copy8(r, acc);
}
// full 512-bit product high half (limbs 8..15)
MW_HD void mulhi8(const u32 a[8], const u32 b[8], u32 lo[8], u32 hi[8]) {
  u32 acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u32 carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u64 p = (u64)a[i] * b[j] + acc[i + j] + carry;
      acc[i + j] = (u32)p;
      carry = (u32)(p >> 32);
    }
    acc[i + 8] = carry;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    lo[k] = acc[k];
    hi[k] = acc[k + 8];
  }
}

// ---------------------------------------------------------------- shifts
// funnel shifts on 32-bit limbs, b in [0,31]: one v_alignbit_b32 each (no
// 64-bit register pairs).  fshl32 with b == 0 must return hi, which the
// alignbit by (32 - b) & 31 == 0 would not: one select covers it.
MW_HD u32 alignbit(u32 hi, u32 lo, u32 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, b);
#else
  return (u32)((((u64)hi << 32) | lo) >> (b & 31u));
#endif
}
MW_HD u32 fshr32(u32 hi, u32 lo, u32 b) { return alignbit(hi, lo, b); }
MW_HD u32 fshl32(u32 hi, u32 lo, u32 b) { return b ? alignbit(hi, lo, 32u - b) : hi; }

// r = a << s for s in [0,255] (bits shifted past 256 dropped)
MW_HD void shl8(const u32 a[8], u32 s, u32 r[8]) {
  u32 t[8];
  copy8(t, a);
  u32 q = s >> 5, b = s & 31;
#pragma unroll
  for (int st = 0; st < 3; ++st) {
    int n = 1 << st;
    bool c = (q >> st) & 1;
#pragma unroll
    for (int k = 7; k >= 0; --k) t[k] = c ? (k >= n ? t[k - n] : 0u) : t[k];
  }
#pragma unroll
  for (int k = 7; k >= 1; --k) r[k] = fshl32(t[k], t[k - 1], b);
  r[0] = t[0] << b;
}
// r = a >> s (fill = 0 or all-ones for arithmetic), s in [0,255]
MW_HD void shr8(const u32 a[8], u32 s, u32 fill, u32 r[8]) {
  u32 t[8];
  copy8(t, a);
  u32 q = s >> 5, b = s & 31;
#pragma unroll
  for (int st = 0; st < 3; ++st) {
    int n = 1 << st;
    bool c = (q >> st) & 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = c ? (k + n < 8 ? t[k + n] : fill) : t[k];
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) r[k] = fshr32(t[k + 1], t[k], b);
  r[7] = fshr32(fill, t[7], b);
}

// amount >= w ?  (amount is a w-bit canonical value held in 8 limbs)
MW_HD bool amount_ge(const u32 b[8], u32 w) {
  u32 hi = b[1] | b[2] | b[3] | b[4] | b[5] | b[6] | b[7];
  return hi != 0 || b[0] >= w;
}

// sign bit of a w-bit value (w in 33..256) / sign fill word
MW_HD bool signbit8(const u32 a[8], u32 w) {
  u32 x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int bit = (int)w - 1 - 32 * k;
    x |= (bit >= 0 && bit < 32) ? ((a[k] >> bit) & 1u) : 0u;
  }
  return x != 0;
}
// sign-extend a w_from-bit value in place to 256 bits
MW_HD void sext8(u32 a[8], u32 w_from) {
  bool s = signbit8(a, w_from);
  if (w_from < 256) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] |= s ? ~limb_mask(w_from, k) : 0u;
  }
}

MW_HD void wshl(const u32 a[8], const u32 b[8], u32 w, u32 r[8]) {
  if (amount_ge(b, w)) {
    zero8(r);
  } else {
    shl8(a, b[0], r);
    canon(r, w);
  }
}
MW_HD void wlshr(const u32 a[8], const u32 b[8], u32 w, u32 r[8]) {
  if (amount_ge(b, w)) {
    zero8(r);
  } else {
    shr8(a, b[0], 0u, r);
  }
}
MW_HD void washr(const u32 a[8], const u32 b[8], u32 w, u32 r[8]) {
  u32 t[8];
  copy8(t, a);
  sext8(t, w);
  u32 fill = signbit8(a, w) ? 0xffffffffu : 0u;
  u32 s = amount_ge(b, w) ? 255u : b[0];
  shr8(t, s, fill, r);
  canon(r, w);
}

// ---------------------------------------------------------------- division
MW_HD u32 clz32(u32 x) { return x ? (u32)__builtin_clz(x) : 32u; }
// Moller-Granlund reciprocal of a normalized divisor d (top bit set):
// floor((2^64 - 1) / d) - 2^32, i.e. the 2-by-1 quotient (~d : 0xffffffff) / d.
// On the device an f64 reciprocal (two Newton steps) gives the quotient to
// within one, and one integer correction makes it exact (tools/exp/recip_check.hip
// checks it against the u64 division on 2^31 divisors): ~20 instructions where
// LLVM's generic u64 division expands to ~350 (about 100 executed).
MW_HD u32 recip32(u32 d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32 nh = ~d;
  const double dd = (double)d;
  double r = __builtin_amdgcn_rcp(dd);
  double e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double n = __builtin_fma((double)nh, 4294967296.0, 4294967295.0);
  // n * r reaches 2^32 for d = 2^31 (the reciprocal is 2^32 - 1): an out-of-range
  // double -> u32 conversion is undefined, and when d is a compile-time constant
  // (a specialised kernel dividing by a known limb) LLVM folds it to poison.
  // The hardware conversion saturates; say so explicitly.
  const double t = n * r;
  u32 v = t >= 4294967295.0 ? 0xffffffffu : (u32)t;
  const u64 nx = ((u64)nh << 32) | 0xffffffffu;
  const u64 p = (u64)v * d;
  if (p > nx) v -= 1u;
  else if (nx - p >= d) v += 1u;
  return v;
#else
  return (u32)(~0ull / (u64)d - (1ull << 32));
#endif
}

// Quotient digit estimate for a full-width divisor (y7 != 0): from the top 64
// bits of both operands, xh = x7:x6 and yh = y7:y6 >= 2^32, never below the true
// quotient floor(x / y) (< 2^32) and at most 2 above it:
//   x / y < (xh + 1) 2^192 / (yh 2^192) = (xh + 1) / yh  <=  estimate,
//   (xh + 1) / yh - x / y <= (xh + yh + 1) / (yh (yh + 1)) ~ 1 + 2^-32.
// Device: f64 with every rounding biased upwards (numerator rounded up by
// 2^-51, denominator down by 2^-51, reciprocal by two Newton steps, quotient
// up by 2^-48).  Host: the exact 64-bit quotient.
MW_HD u32 qdigit_est(u32 x7, u32 x6, u32 y7, u32 y6) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double two32 = 4294967296.0;
  const double xd = __builtin_fma((double)x7, two32, (double)x6);
  const double yd = __builtin_fma((double)y7, two32, (double)y6);
  const double A = (xd + 1.0) * (1.0 + 0x1p-51);
  const double B = yd * (1.0 - 0x1p-51);
  double rc = __builtin_amdgcn_rcp(B);
  double e = __builtin_fma(-B, rc, 1.0);
  rc = __builtin_fma(rc, e, rc);
  e = __builtin_fma(-B, rc, 1.0);
  rc = __builtin_fma(rc, e, rc);
  const double Q = A * rc * (1.0 + 0x1p-48);
  return Q >= 4294967295.0 ? 0xffffffffu : (u32)Q;
#else
  const u64 xh = ((u64)x7 << 32) | x6, yh = ((u64)y7 << 32) | y6;
  const u64 qe = xh == ~0ull ? xh / yh + 1u : (xh + 1u) / yh;
  return qe > 0xffffffffull ? 0xffffffffu : (u32)qe;
#endif
}

// The same estimate for a three-limb window (w2:w1:w0) over a divisor whose top
// limb y7 is nonzero (not necessarily normalised), when the window's digit is
// below 2^32: (w2:w1:w0) is rounded up by 2^-50 (three roundings).
MW_HD u32 qdigit_est3(u32 w2, u32 w1, u32 w0, u32 y7, u32 y6) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double two32 = 4294967296.0;
  const double wd = __builtin_fma(__builtin_fma((double)w2, two32, (double)w1), two32, (double)w0);
  const double yd = __builtin_fma((double)y7, two32, (double)y6);
  const double A = (wd + 1.0) * (1.0 + 0x1p-50);
  const double B = yd * (1.0 - 0x1p-51);
  double rc = __builtin_amdgcn_rcp(B);
  double e = __builtin_fma(-B, rc, 1.0);
  rc = __builtin_fma(rc, e, rc);
  e = __builtin_fma(-B, rc, 1.0);
  rc = __builtin_fma(rc, e, rc);
  const double Q = A * rc * (1.0 + 0x1p-48);
  return Q >= 4294967295.0 ? 0xffffffffu : (u32)Q;
#else
  const unsigned __int128 W = ((unsigned __int128)w2 << 64) | ((unsigned __int128)w1 << 32) | w0;
  const u64 yh = ((u64)y7 << 32) | y6;
  const unsigned __int128 qe = (W + 1u) / yh;
  return qe > 0xffffffffu ? 0xffffffffu : (u32)qe;
#endif
}

// q = x / y, r = x % y when y's top limb is nonzero (y >= 2^224, so q < 2^32):
// one estimated digit (qdigit_est, never too small), one multiply-subtract over
// 9 limbs, and an add-back loop for the (rare) overestimate, run by a wave only
// if one of its lanes needs it.  No shifts and no digit loop: tools/ab_c5.py
// measured division at half of the C5 kernel's time before this path.
MW_HD void udivrem8_full(const u32 x[8], const u32 y[8], u32 q[8], u32 r[8]) {
  u32 qd = qdigit_est(x[7], x[6], y[7], y[6]);
  u32 carry = 0, br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u64 p = (u64)qd * y[k] + carry;
    carry = (u32)(p >> 32);
    r[k] = subb(x[k], (u32)p, br);
  }
  u32 hi = 0u - carry - br;  // limb 8 of x - qd*y: 0, or -1/-2 when qd is too large
  while (MW_RARE(MW_ANY(hi != 0u))) {
    if (hi != 0u) {
      u32 c = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = addc(r[k], y[k], c);
      hi += c;
      qd -= 1u;
    }
  }
  q[0] = qd;
#pragma unroll
  for (int k = 1; k < 8; ++k) q[k] = 0u;
}

// q = x / y, r = x % y for a one-limb divisor (0 < y < 2^32): short division,
// eight 2-by-1 steps (Moller & Granlund 2011, Alg. 4) with one reciprocal of
// the normalised divisor; the remainder stays one limb throughout.  C5 divides
// by such values (quotients of earlier divisions) in 42 of its 384 divisions,
// where the general loop ran all eight steps.
// The eight steps are unrolled.  MW_SHORT_ROLLED runs them as a rolled loop
// over a sliding window (w[7] the current limb, w[6] the next lower one), the
// digits shifting into qq: 90 KB less code over C5's 384 division sites, but
// 0.2 ms slower per 2^22 launch (tools/ab_c5.py "shortroll", profiles/r4h).
MW_HD void udivrem8_short(const u32 x[8], u32 y0, u32 q[8], u32 r[8]) {
  const u32 s = clz32(y0);
  const u32 d = y0 << s;
  const u32 v = recip32(d);
  u32 rem = fshl32(0u, x[7], s);  // < 2^s <= d
#if defined(MW_SHORT_ROLLED)
  u32 w[8], qq[8];
  copy8(w, x);
  zero8(qq);
#pragma unroll 1
  for (int it = 0; it < 8; ++it) {
    const u32 u0 = fshl32(w[7], w[6], s);   // it == 7: x[0] << s (w[6] is 0 by then)
    const u64 qp = (u64)v * rem + ((((u64)rem) << 32) | u0);
    u32 q1 = (u32)(qp >> 32) + 1u;
    const u32 q0 = (u32)qp;
    u32 rr = u0 - q1 * d;
    const bool adj1 = rr > q0;
    q1 = adj1 ? q1 - 1u : q1;
    rr = adj1 ? rr + d : rr;
    const bool adj2 = rr >= d;  // unlikely
    q1 = adj2 ? q1 + 1u : q1;
    rr = adj2 ? rr - d : rr;
#pragma unroll
    for (int k = 7; k > 0; --k) qq[k] = qq[k - 1];
    qq[0] = q1;
#pragma unroll
    for (int k = 7; k > 0; --k) w[k] = w[k - 1];
    w[0] = 0u;
    rem = rr;
  }
  copy8(q, qq);
#else
#pragma unroll
  for (int k = 7; k >= 0; --k) {
    const u32 u0 = k > 0 ? fshl32(x[k], x[k - 1], s) : (x[0] << s);
    const u64 qq = (u64)v * rem + ((((u64)rem) << 32) | u0);
    u32 q1 = (u32)(qq >> 32) + 1u;
    const u32 q0 = (u32)qq;
    u32 rr = u0 - q1 * d;
    const bool adj1 = rr > q0;
    q1 = adj1 ? q1 - 1u : q1;
    rr = adj1 ? rr + d : rr;
    const bool adj2 = rr >= d;  // unlikely
    q1 = adj2 ? q1 + 1u : q1;
    rr = adj2 ? rr - d : rr;
    q[k] = q1;
    rem = rr;
  }
#endif
  r[0] = rem >> s;
#pragma unroll
  for (int k = 1; k < 8; ++k) r[k] = 0u;
}

// q = x / y, r = x % y for y != 0, base-2^32 schoolbook division with one of
// three paths per wave: a single estimated digit when every lane's divisor is
// full width (udivrem8_full), short division when every lane's divisor is one
// limb (udivrem8_short), and otherwise limb-aligned digits with the same
// estimate (below).  Digit estimates are never too small and at most 2 too
// large; the add-back runs under a wave-uniform branch that is almost never
// taken.  Zero digits are skipped per wave: when the window's top limb is 0 and
// the next one is below the divisor's top limb, the window is below the
// divisor.  *dc (optional) counts the path the wave took and the digit steps
// it ran, for the executed-work roofline (bench.py).
// Per-wave division path counts for the executed-work roofline (bench.py,
// compiler.Program.executed_ops): each field is incremented once per wave
// (wave-uniform), and the kernels add nvalid x count to mg_stats.
struct DivCount {
  u32 full = 0;   // one-digit path (every lane's divisor full width)
  u32 shrt = 0;   // short division (every lane's divisor one limb)
  u32 gen = 0;    // limb-aligned schoolbook entries
  u32 steps = 0;  // digit positions the schoolbook path ran (some lane's digit nonzero)
};

// The launch counters (evals, then the DivCount fields x lanes) are striped:
// stripe 0 is the interpreters' (one atomic per wave per launch), stripes
// 1..MW_CTR_STRIPES the specialised kernels' (one 256-candidate block each,
// so one set of atomics per wave per chunk: on a single address those
// serialise across the 8 XCDs, ~12 ns each, and capped small programs at
// ~5 G evals/s).  Each stripe is a 128-byte line; the host sums them.
#define MW_CTR_STRIPES 64
#define MW_CTR_STRIPE_WORDS 16

#if defined(__HIP_DEVICE_COMPILE__)
// counter[1..4] += nvalid x (steps, full, short, general): one lane per wave
__device__ inline void add_div_counts(u64* counter, const DivCount& dc, u64 nvalid) {
  if (dc.steps) atomicAdd((unsigned long long*)(counter + 1), (unsigned long long)(nvalid * dc.steps));
  if (dc.full) atomicAdd((unsigned long long*)(counter + 2), (unsigned long long)(nvalid * dc.full));
  if (dc.shrt) atomicAdd((unsigned long long*)(counter + 3), (unsigned long long)(nvalid * dc.shrt));
  if (dc.gen) atomicAdd((unsigned long long*)(counter + 4), (unsigned long long)(nvalid * dc.gen));
}
#endif

MW_HD void udivrem8(const u32 x[8], const u32 y[8], u32 q[8], u32 r[8], DivCount* dc = nullptr) {
  if (MW_USUAL(!MW_ANY(y[7] == 0u))) {  // every lane's divisor is full width: one digit
    udivrem8_full(x, y, q, r);
    if (dc) dc->full += 1u;
    return;
  }
  if (MW_RARE(!MW_ANY((y[1] | y[2] | y[3] | y[4] | y[5] | y[6] | y[7]) != 0u))) {  // one-limb divisors
    udivrem8_short(x, y[0], q, r);
    if (dc) dc->shrt += 1u;
    return;
  }
  // Any other divisor: schoolbook division on limb-aligned operands.  Both are
  // shifted left by whole limbs (n = the divisor's zero top limbs, per lane)
  // so the divisor's top limb is nonzero; no bit normalisation is needed,
  // because each digit comes from the same upward-biased f64 estimate as the
  // full-width path (qdigit_est3: never too small, at most 2 too large),
  // followed by one multiply-subtract over 9 limbs and a wave-skipped
  // add-back loop.  A digit position runs only if some lane of the wave has a
  // nonzero digit there.  (Knuth's loop with 3-by-2 estimates, used until
  // round 2, needed bit normalisation and cost about 1.5x as much per digit;
  // tools/ab_c5.py put those 25 of C5's 384 divisions at 13 % of the kernel.)
  if (dc) dc->gen += 1u;
  u32 v[8], u[16];
  copy8(v, y);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    u[k] = x[k];
    u[k + 8] = 0u;
  }
#if defined(MW_GEN_ROLLED_SHIFT)
  // v <<= 32n, u <<= 32n (n: the lane's zero top limbs of y) as a rolled loop
  // of one-limb moves under selects, run as often as the wave's largest n:
  // 90 KB less code than the three select stages below, but 1.8 ms slower per
  // 2^22 C5 launch (tools/ab_c5.py "genroll", profiles/r4h): the loop's exit
  // test and its serial chain run at every division site a wave reaches
  u32 n = 0u;
#pragma unroll 1
  for (int st = 0; st < 7; ++st) {
    const bool c = v[7] == 0u;
    if (!MW_ANY(c)) break;
    n += c ? 1u : 0u;
#pragma unroll
    for (int k = 7; k > 0; --k) v[k] = c ? v[k - 1] : v[k];
    v[0] = c ? 0u : v[0];
#pragma unroll
    for (int k = 15; k > 0; --k) u[k] = c ? u[k - 1] : u[k];
    u[0] = c ? 0u : u[0];
  }
#else
  const u32 n = y[7] ? 0u : y[6] ? 1u : y[5] ? 2u : y[4] ? 3u : y[3] ? 4u : y[2] ? 5u : y[1] ? 6u : 7u;
#pragma unroll
  for (int st = 0; st < 3; ++st) {  // v <<= 32n, u <<= 32n (limb moves under selects)
    const int m = 1 << st;
    const bool c = (n >> st) & 1u;
#pragma unroll
    for (int k = 7; k >= 0; --k) v[k] = c ? (k >= m ? v[k - m] : 0u) : v[k];
#pragma unroll
    for (int k = 15; k >= 0; --k) u[k] = c ? (k >= m ? u[k - m] : 0u) : u[k];
  }
#endif
  // The eight digit positions as a rolled loop over a sliding window
  // w = u[j..j+8] (j = 7 - it), the untouched low limbs feeding it from lo[]
  // and the digits shifting into qq[]: unrolled, this path was ~1 000
  // instructions at each of C5's 384 division sites, most of the kernel's
  // code, although a site runs it on every wave or on none.
  u32 w[9], lo[7], qq[8];
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = u[7 + k];
#pragma unroll
  for (int k = 0; k < 7; ++k) lo[k] = u[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) qq[k] = 0u;
#pragma unroll 1
  for (int it = 0; it < 8; ++it) {
    u32 qd = 0u;
    if (MW_ANY(w[8] != 0u || w[7] >= v[7])) {  // else digit 0 in every lane
      if (dc) dc->steps += 1u;
      qd = qdigit_est3(w[8], w[7], w[6], v[7], v[6]);
      u32 carry = 0, br = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const u64 p = (u64)qd * v[k] + carry;
        carry = (u32)(p >> 32);
        w[k] = subb(w[k], (u32)p, br);
      }
      u32 hi = w[8] - carry - br;  // 0, or the negative top limb when qd is too large
      while (MW_RARE(MW_ANY(hi != 0u))) {
        if (hi != 0u) {
          u32 c = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) w[k] = addc(w[k], v[k], c);
          hi += c;
          qd -= 1u;
        }
      }
      w[8] = 0u;
    }
#pragma unroll
    for (int k = 7; k > 0; --k) qq[k] = qq[k - 1];
    qq[0] = qd;
    if (it < 7) {  // the next window u[j-1 .. j+7]
#pragma unroll
      for (int k = 8; k > 0; --k) w[k] = w[k - 1];
      w[0] = lo[6];
#pragma unroll
      for (int k = 6; k > 0; --k) lo[k] = lo[k - 1];
      lo[0] = 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    q[k] = qq[k];
    u[k] = w[k];
    u[k + 8] = 0u;
  }
#if defined(MW_GEN_ROLLED_SHIFT)
#pragma unroll 1
  for (int st = 0; st < 7; ++st) {  // r = u[0..7] >> 32n, one limb per pass
    const bool c = n > (u32)st;
    if (!MW_ANY(c)) break;
#pragma unroll
    for (int k = 0; k < 7; ++k) u[k] = c ? u[k + 1] : u[k];
    u[7] = c ? 0u : u[7];
  }
#else
#pragma unroll
  for (int st = 0; st < 3; ++st) {  // r = u[0..7] >> 32n
    const int m = 1 << st;
    const bool c = (n >> st) & 1u;
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = c ? (k + m < 16 ? u[k + m] : 0u) : u[k];
  }
#endif
  copy8(r, u);
}

MW_HD void neg8(const u32 a[8], u32 r[8]) {
  u32 br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = subb(0u, a[k], br);
}
MW_HD void cneg8(u32 a[8], bool c, u32 w) {  // a = c ? -a mod 2^w : a
  u32 br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u32 t = subb(0u, a[k], br);
    a[k] = c ? t : a[k];
  }
  canon(a, w);
}

// kind: 0 udiv, 1 urem, 2 sdiv, 3 srem, 4 smod.  x, y are consumed (overwritten).
MW_HD void wdiv(int kind, u32 x[8], u32 y[8], u32 w, u32 r[8], DivCount* dc = nullptr) {
  bool sa = false, sb = false;
  if (kind >= 2) {
    sa = signbit8(x, w);
    sb = signbit8(y, w);
    cneg8(x, sa, w);  // |s|
    cneg8(y, sb, w);  // |t|
  }
  const bool yz = is_zero8(y);
  y[0] |= yz ? 1u : 0u;  // divide by 1 instead; result replaced below
  u32 q[8];
  udivrem8(x, y, q, r, dc);  // r = |s| mod |t|
  if (yz) {  // SMT-LIB: q = all ones, r = dividend magnitude
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      q[k] = limb_mask(w, k);
      r[k] = x[k];
    }
  }
  switch (kind) {
    case 0:
      copy8(r, q);
      break;
    case 1:
      break;
    case 2:  // quotient negated when the signs differ
      copy8(r, q);
      cneg8(r, sa != sb, w);
      break;
    case 3:  // remainder takes the dividend's sign
      cneg8(r, sa, w);
      break;
    default: {  // smod: u = |s| mod |t|; result follows the divisor's sign
      const bool uz = is_zero8(r);
      // t (the signed divisor) = sb ? -|t| : |t|  (y still holds |t|, or 1 if t == 0)
      if (yz) y[0] = 0u;
      cneg8(y, sb, w);
      // sa & !sb : t - u ; !sa & sb : u + t ; sa & sb : -u
      const bool negu = sa;
      cneg8(r, negu, w);  // r = sa ? -u : u
      const bool addt = !uz && (sa != sb);
      u32 c = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const u32 t = addc(r[k], y[k], c);
        r[k] = addt ? t : r[k];
      }
      break;
    }
  }
  canon(r, w);
}

// ---------------------------------------------------------------- narrow (<= 32 bit)
MW_HD u32 n_sext(u32 a, u32 wfrom) {
  if (wfrom >= 32) return a;
  u32 s = (a >> (wfrom - 1)) & 1u;
  return s ? (a | ~nmask(wfrom)) : a;
}
MW_HD u32 n_div(int kind, u32 a, u32 b, u32 w) {
  u32 m = nmask(w);
  bool sa = false, sb = false;
  u32 x = a, y = b;
  if (kind >= 2) {
    sa = (a >> (w - 1)) & 1u;
    sb = (b >> (w - 1)) & 1u;
    x = sa ? ((0u - a) & m) : a;
    y = sb ? ((0u - b) & m) : b;
  }
  u32 q, rm;
  if (y == 0) {
    q = m;
    rm = x;
  } else {
    q = x / y;
    rm = x - q * y;
  }
  u32 r;
  switch (kind) {
    case 0: r = q; break;
    case 1: r = rm; break;
    case 2: r = (sa != sb) ? (0u - q) : q; break;
    case 3: r = sa ? (0u - rm) : rm; break;
    default: {
      if (rm == 0) r = 0;
      else if (!sa && !sb) r = rm;
      else if (sa && !sb) r = (0u - rm) + b;
      else if (!sa && sb) r = rm + b;
      else r = 0u - rm;
      break;
    }
  }
  return r & m;
}
MW_HD u32 n_shl(u32 a, u32 b, u32 w) { return b >= w ? 0u : ((a << b) & nmask(w)); }
MW_HD u32 n_lshr(u32 a, u32 b, u32 w) { return b >= w ? 0u : (a >> b); }
MW_HD u32 n_ashr(u32 a, u32 b, u32 w) {
  int32_t sa = (int32_t)n_sext(a, w);
  u32 s = b >= w ? 31u : b;
  return ((u32)(sa >> s)) & nmask(w);
}
MW_HD bool n_slt(u32 a, u32 b, u32 w) { return (int32_t)n_sext(a, w) < (int32_t)n_sext(b, w); }
MW_HD bool n_sle(u32 a, u32 b, u32 w) { return (int32_t)n_sext(a, w) <= (int32_t)n_sext(b, w); }
MW_HD bool n_umulno(u32 a, u32 b, u32 w) {
  u64 p = (u64)a * b;
  return w >= 32 ? (p >> 32) == 0 : (p >> w) == 0;
}

}  // namespace mw
