/* ORACLE (test infrastructure only) — C restatement of the DAG semantics.
 *
 * Plain C99 + OpenMP.  Evaluates a constraint DAG (serialised by oracle/cdag.py
 * from the IR) for candidate indices [begin, begin+n): leaves drawn with
 * Philox4x32-10 exactly as oracle/philox.py specifies, every op with SMT-LIB
 * 2.6 semantics (oracle/bvsem.py is the reference for this file; both restate
 * z3's bitvector theory as Mythril uses it, mythril/laser/smt/bitvec.py,
 * bitvec_helper.py, bool.py).  Widths 1..256; values are 8 x u32 limbs,
 * canonical (bits >= width are zero).  Written independently of the product
 * ALU (mythril_amd/csrc): simple schoolbook arithmetic, bit-serial division.
 *
 * Used by bench.py's cpu_baseline leg and by tests for large parity sweeps.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef uint32_t u32;
typedef uint64_t u64;

enum {
  O_CONST = 0, O_VAR, O_ADD, O_SUB, O_MUL, O_UDIV, O_UREM, O_SDIV, O_SREM, O_SMOD,
  O_AND, O_OR, O_XOR, O_NOT, O_NEG, O_SHL, O_LSHR, O_ASHR, O_CONCAT, O_EXTRACT,
  O_ZEXT, O_SEXT, O_ITE, O_EQ, O_ULT, O_ULE, O_SLT, O_SLE, O_UMULNO, O_ROTL, O_ROTR, O_ADDC
};

/* node record: op, width, a, b, c, p0, p1, salt (8 x i32) */
typedef struct { int32_t op, w, a, b, c, p0, p1, salt; } onode;

static void mask(u32* v, int w) {
  for (int k = 0; k < 8; ++k) {
    int lo = 32 * k;
    if (w >= lo + 32) continue;
    if (w <= lo) v[k] = 0;
    else v[k] &= (1u << (w - lo)) - 1u;
  }
}
static int bit(const u32* v, int i) { return (v[i >> 5] >> (i & 31)) & 1; }
static int iszero(const u32* v) { for (int k = 0; k < 8; ++k) if (v[k]) return 0; return 1; }
static int cmpu(const u32* a, const u32* b) {
  for (int k = 7; k >= 0; --k) { if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1; }
  return 0;
}
static void add(const u32* a, const u32* b, u32* r) {
  u64 c = 0;
  for (int k = 0; k < 8; ++k) { c += (u64)a[k] + b[k]; r[k] = (u32)c; c >>= 32; }
}
static void sub(const u32* a, const u32* b, u32* r) {
  u64 br = 0;
  for (int k = 0; k < 8; ++k) { u64 t = (u64)a[k] - b[k] - br; r[k] = (u32)t; br = (t >> 63) & 1; }
}
static void neg(const u32* a, u32* r, int w) { u32 z[8] = {0}; sub(z, a, r); mask(r, w); }
static void mul(const u32* a, const u32* b, u32* r) {
  u32 t[16]; memset(t, 0, sizeof t);
  for (int i = 0; i < 8; ++i) {
    u64 c = 0;
    for (int j = 0; j < 8; ++j) { c += (u64)a[i] * b[j] + t[i + j]; t[i + j] = (u32)c; c >>= 32; }
    t[i + 8] = (u32)c;
  }
  memcpy(r, t, 32);
}
static void shl1(u32* v) { for (int k = 7; k > 0; --k) v[k] = (v[k] << 1) | (v[k - 1] >> 31); v[0] <<= 1; }
static void shl(const u32* a, int s, u32* r) {  /* 0 <= s < 256 */
  u32 t[8] = {0}; int q = s >> 5, b = s & 31;
  for (int k = 7; k >= 0; --k) {
    if (k - q < 0) continue;
    u32 v = a[k - q] << b;
    if (b && k - q - 1 >= 0) v |= a[k - q - 1] >> (32 - b);
    t[k] = v;
  }
  memcpy(r, t, 32);
}
static void shr(const u32* a, int s, u32 fill, u32* r) { /* 0 <= s < 256, fill = 0 or ~0 */
  u32 t[8]; int q = s >> 5, b = s & 31;
  for (int k = 0; k < 8; ++k) {
    u32 lo = (k + q < 8) ? a[k + q] : fill;
    u32 hi = (k + q + 1 < 8) ? a[k + q + 1] : fill;
    t[k] = b ? (lo >> b) | (hi << (32 - b)) : lo;
  }
  memcpy(r, t, 32);
}
/* bit-serial restoring division, y != 0 */
static void udivrem(const u32* x, const u32* y, u32* q, u32* r) {
  u32 rr[8] = {0}, qq[8] = {0};
  int top = 255;
  while (top >= 0 && !bit(x, top)) --top;
  for (int i = top; i >= 0; --i) {
    shl1(rr);
    rr[0] |= (u32)bit(x, i);
    if (cmpu(rr, y) >= 0) { sub(rr, y, rr); qq[i >> 5] |= 1u << (i & 31); }
  }
  memcpy(q, qq, 32); memcpy(r, rr, 32);
}
static int sgnbit(const u32* a, int w) { return bit(a, w - 1); }
static void sext_to256(u32* a, int w) {
  if (w < 256 && sgnbit(a, w)) {
    for (int i = w; i < 256; ++i) a[i >> 5] |= 1u << (i & 31);
  }
}
static void ones(u32* r, int w) { for (int k = 0; k < 8; ++k) r[k] = 0xffffffffu; mask(r, w); }
static int amount_ge(const u32* b, int w) {
  for (int k = 1; k < 8; ++k) if (b[k]) return 1;
  return b[0] >= (u32)w;
}

static void divop(int op, const u32* s, const u32* t, int w, u32* r) {
  u32 q[8], m[8], x[8], y[8], tmp[8];
  if (op == O_UDIV || op == O_UREM) {
    if (iszero(t)) { if (op == O_UDIV) ones(r, w); else memcpy(r, s, 32); return; }
    udivrem(s, t, q, m);
    memcpy(r, op == O_UDIV ? q : m, 32);
    return;
  }
  int ms = sgnbit(s, w), mt = sgnbit(t, w);
  if (ms) neg(s, x, w); else memcpy(x, s, 32);
  if (mt) neg(t, y, w); else memcpy(y, t, 32);
  if (iszero(y)) { ones(q, w); memcpy(m, x, 32); } else udivrem(x, y, q, m);
  if (op == O_SDIV) {
    if (ms != mt) neg(q, r, w); else memcpy(r, q, 32);
  } else if (op == O_SREM) {
    if (ms) neg(m, r, w); else memcpy(r, m, 32);
  } else { /* smod: sign follows the divisor */
    if (iszero(m)) { memset(r, 0, 32); }
    else if (!ms && !mt) memcpy(r, m, 32);
    else if (ms && !mt) { neg(m, tmp, w); add(tmp, t, r); }
    else if (!ms && mt) add(m, t, r);
    else neg(m, r, w);
  }
  mask(r, w);
}

static void philox(u32 c[4], u32 k0, u32 k1) {
  for (int i = 0; i < 10; ++i) {
    u64 p0 = (u64)0xD2511F53u * c[0], p1 = (u64)0xCD9E8D57u * c[2];
    u32 n0 = (u32)(p1 >> 32) ^ c[1] ^ k0, n2 = (u32)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (u32)p1; c[3] = (u32)p0; c[0] = n0; c[2] = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
static u64 fmix64(u64 h) {
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  return h;
}

/* Random leaf (oracle/philox.py random_leaf): w > 32 Philox4x32-10 blocks 0
 * and 1; w <= 32 one fmix64 of the index, seed and salt. */
static void leaf(u64 seed, u32 salt, u64 cand, int w, u32* out) {
  if (w <= 32) {
    const u64 h = fmix64(cand ^ seed ^ ((u64)salt * 0xC2B2AE3D27D4EB4Full));
    out[0] = (u32)h;
    for (int k = 1; k < 8; ++k) out[k] = 0;
    mask(out, w);
    return;
  }
  u32 k0 = (u32)seed ^ salt, k1 = (u32)(seed >> 32);
  for (u32 blk = 0; blk < 2; ++blk) {
    u32 c[4] = {(u32)cand, (u32)(cand >> 32), blk, 0};
    philox(c, k0, k1);
    for (int i = 0; i < 4; ++i) out[4 * blk + i] = c[i];
  }
  mask(out, w);
}

/* Candidate-leaf spec (oracle/philox.py leaf_value; DESIGN.md "Candidate space"):
 * kind 0 random, 1 pool digit = index bit-field, 2 hashed digit, 3 bit-interleaved
 * digit.  Pool entries are 9 words: flags (bit 0 = RANDOM) + 8 limbs. */
typedef struct { int32_t kind, shift, bits, stride, pool; } ospec;

static void spec_leaf(const ospec* sp, const u32* pool, u64 seed, u32 salt, u64 cand, int w, u32* out) {
  if (sp && sp->kind >= 1 && sp->kind <= 3) {
    u64 d = 0;
    u64 m = sp->bits >= 64 ? ~0ull : ((1ull << sp->bits) - 1);
    if (sp->kind == 1) d = (cand >> sp->shift) & m;
    else if (sp->kind == 2) d = fmix64(cand ^ ((u64)salt * 0x9E3779B97F4A7C15ull)) & m;
    else for (int b = 0; b < sp->bits; ++b) d |= ((cand >> (sp->shift + b * sp->stride)) & 1ull) << b;
    const u32* e = pool + sp->pool + 9 * d;
    if (!(e[0] & 1u)) {
      for (int k = 0; k < 8; ++k) out[k] = e[1 + k];
      mask(out, w);
      return;
    }
  }
  leaf(seed, salt, cand, w, out);
}

static const ospec* g_specs;   /* set per call (read-only while the OpenMP region runs) */
static const u32* g_pool;

static void eval1(const onode* g, const u32* consts, int i, u32* V, u64 seed, u64 cand) {
  const onode* n = &g[i];
  u32* r = V + 8 * (size_t)i;
  const u32* a = n->a >= 0 ? V + 8 * (size_t)n->a : 0;
  const u32* b = n->b >= 0 ? V + 8 * (size_t)n->b : 0;
  const u32* c = n->c >= 0 ? V + 8 * (size_t)n->c : 0;
  int w = n->w;
  int aw = n->a >= 0 ? g[n->a].w : w;
  u32 t[8], u[8];
  switch (n->op) {
    case O_CONST: memcpy(r, consts + 8 * (size_t)n->p0, 32); break;
    case O_VAR: spec_leaf(g_specs && n->p0 >= 0 ? &g_specs[n->p0] : 0, g_pool, seed, (u32)n->salt, cand, w, r); break;
    case O_ADD: add(a, b, r); mask(r, w); break;
    case O_SUB: sub(a, b, r); mask(r, w); break;
    case O_MUL: mul(a, b, r); mask(r, w); break;
    case O_UDIV: case O_UREM: case O_SDIV: case O_SREM: case O_SMOD: divop(n->op, a, b, w, r); break;
    case O_AND: for (int k = 0; k < 8; ++k) r[k] = a[k] & b[k]; break;
    case O_OR: for (int k = 0; k < 8; ++k) r[k] = a[k] | b[k]; break;
    case O_XOR: for (int k = 0; k < 8; ++k) r[k] = a[k] ^ b[k]; break;
    case O_NOT: for (int k = 0; k < 8; ++k) r[k] = ~a[k]; mask(r, w); break;
    case O_NEG: neg(a, r, w); break;
    case O_SHL: if (amount_ge(b, w)) memset(r, 0, 32); else { shl(a, (int)b[0], r); mask(r, w); } break;
    case O_LSHR: if (amount_ge(b, w)) memset(r, 0, 32); else shr(a, (int)b[0], 0, r); break;
    case O_ASHR: {
      memcpy(t, a, 32); sext_to256(t, w);
      u32 fill = sgnbit(a, w) ? 0xffffffffu : 0u;
      shr(t, amount_ge(b, w) ? 255 : (int)b[0], fill, r); mask(r, w); break;
    }
    case O_CONCAT: /* a = high part, b = low part of width g[b].w */
      shl(a, g[n->b].w, t); for (int k = 0; k < 8; ++k) r[k] = t[k] | b[k]; mask(r, w); break;
    case O_EXTRACT: shr(a, n->p1, 0, r); mask(r, w); break;
    case O_ZEXT: memcpy(r, a, 32); break;
    case O_SEXT: memcpy(r, a, 32); sext_to256(r, aw); mask(r, w); break;
    case O_ITE: memcpy(r, a[0] ? b : c, 32); break;
    case O_EQ: memset(r, 0, 32); r[0] = cmpu(a, b) == 0; break;
    case O_ULT: memset(r, 0, 32); r[0] = cmpu(a, b) < 0; break;
    case O_ULE: memset(r, 0, 32); r[0] = cmpu(a, b) <= 0; break;
    case O_SLT: case O_SLE: {
      memcpy(t, a, 32); memcpy(u, b, 32);
      t[(aw - 1) >> 5] ^= 1u << ((aw - 1) & 31); u[(aw - 1) >> 5] ^= 1u << ((aw - 1) & 31);
      int cmp = cmpu(t, u);
      memset(r, 0, 32); r[0] = n->op == O_SLT ? cmp < 0 : cmp <= 0; break;
    }
    case O_UMULNO: { /* full product < 2^aw */
      u32 full[16]; memset(full, 0, sizeof full);
      for (int i2 = 0; i2 < 8; ++i2) {
        u64 cc = 0;
        for (int j = 0; j < 8; ++j) { cc += (u64)a[i2] * b[j] + full[i2 + j]; full[i2 + j] = (u32)cc; cc >>= 32; }
        full[i2 + 8] = (u32)cc;
      }
      int ok = 1;
      for (int bi = aw; bi < 512; ++bi) if ((full[bi >> 5] >> (bi & 31)) & 1) { ok = 0; break; }
      memset(r, 0, 32); r[0] = ok; break;
    }
    case O_ROTL: case O_ROTR: {
      int s = n->p0 % w; if (n->op == O_ROTR) s = (w - s) % w;
      if (!s) { memcpy(r, a, 32); break; }
      shl(a, s, t); mask(t, w); shr(a, w - s, 0, u);
      for (int k = 0; k < 8; ++k) r[k] = t[k] | u[k];
      break;
    }
    case O_ADDC: { /* carry out of the aw-bit sum a + b (operands < 2^aw) */
      u64 cc = 0;
      for (int k = 0; k < 8; ++k) { cc += (u64)a[k] + b[k]; t[k] = (u32)cc; cc >>= 32; }
      int co = aw >= 256 ? (int)cc : (int)((t[aw >> 5] >> (aw & 31)) & 1u);
      memset(r, 0, 32); r[0] = (u32)co; break;
    }
    default: memset(r, 0, 32); break;
  }
}

/* Evaluate candidates [begin, begin+n); roots are Bool nodes (conjuncts).
 * verdict (may be NULL) receives 0/1; returns the number satisfied, or -1. */
long long odag_eval(const int32_t* nodes, int nn, const u32* consts, const int32_t* roots, int nroots,
                    u64 seed, u64 begin, u64 n, uint8_t* verdict, int nthreads, u64* first_sat) {
  const onode* g = (const onode*)nodes;
  long long total = 0;
  u64 best = ~0ull;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : total)
  {
    u32* V = (u32*)malloc(sizeof(u32) * 8 * (size_t)nn);
    u64 mybest = ~0ull;
#pragma omp for schedule(dynamic, 64)
    for (long long j = 0; j < (long long)n; ++j) {
      u64 cand = begin + (u64)j;
      for (int i = 0; i < nn; ++i) eval1(g, consts, i, V, seed, cand);
      int ok = 1;
      for (int k = 0; k < nroots; ++k) ok &= (V[8 * (size_t)roots[k]] & 1u) != 0;
      if (verdict) verdict[j] = (uint8_t)ok;
      total += ok;
      if (ok && cand < mybest) mybest = cand;
    }
#pragma omp critical
    { if (mybest < best) best = mybest; }
    free(V);
  }
  if (first_sat) *first_sat = best;
  return total;
}

/* As odag_eval, with pool/hashed/interleaved leaves: VAR node p0 indexes specs
 * (-1 = random leaf); pool holds the 9-word entries the specs point into. */
long long odag_eval_spec(const int32_t* nodes, int nn, const u32* consts, const int32_t* roots, int nroots,
                         const int32_t* specs, const u32* pool, u64 seed, u64 begin, u64 n, uint8_t* verdict,
                         int nthreads, u64* first_sat) {
  g_specs = (const ospec*)specs;
  g_pool = pool;
  long long r = odag_eval(nodes, nn, consts, roots, nroots, seed, begin, n, verdict, nthreads, first_sat);
  g_specs = 0;
  g_pool = 0;
  return r;
}

/* ---------------------------------------------------------------------------
 * Division path counts (checks mg_stats.lane_div_* of the product kernels).
 * The product's wide division (mythril_amd/csrc/mw_alu.h udivrem8, called as
 * mw_alu.h wdiv does: dividend |s|, divisor |t| or 1 when t = 0, at the op's
 * width) picks its path per wave of 64 lanes from these documented rules:
 *   full    every lane's divisor has its top limb (7) nonzero
 *   short   otherwise, every lane's divisor is one limb
 *   general otherwise: both operands move up by n = (zero top limbs of the
 *           divisor) limbs, and digit position j = 7..0 runs when some lane
 *           has u[j+8] != 0 or u[j+7] >= v[7] for its current remainder u.
 * Restated here from those rules (not from the product's code): the remainder
 * above position j is R_j = (x << 32n >> 32(j+1)) mod v, so u[j+8] = R_j[7]
 * and u[j+7] = R_j[6]; R is advanced one limb at a time by bit-serial
 * reduction.  Waves are `wave` consecutive candidates from begin (the kernels'
 * lane -> index map); out = {digit steps, full, short, general}, each x lanes. */
static void div_operands(const onode* g, int i, const u32* V, u32* x, u32* y) {
  const onode* nd = &g[i];
  const u32* s = V + 8 * (size_t)nd->a;
  const u32* t = V + 8 * (size_t)nd->b;
  int w = nd->w;
  if (nd->op == O_SDIV || nd->op == O_SREM || nd->op == O_SMOD) {
    if (sgnbit(s, w)) neg(s, x, w); else memcpy(x, s, 32);
    if (sgnbit(t, w)) neg(t, y, w); else memcpy(y, t, 32);
  } else {
    memcpy(x, s, 32);
    memcpy(y, t, 32);
  }
  if (iszero(y)) y[0] = 1;
}

/* conds bit j: digit position j runs for this lane (general path) */
static u32 general_conds(const u32* x, const u32* y) {
  int n = 0;
  while (n < 7 && y[7 - n] == 0) ++n;
  u32 v[8] = {0}, u[16] = {0}, R[8];
  for (int k = 0; k + n < 8; ++k) v[k + n] = y[k];
  for (int k = 0; k < 8; ++k) u[k + n] = x[k];
  memcpy(R, u + 8, 32);
  u32 conds = 0;
  for (int j = 7; j >= 0; --j) {
    if (R[7] != 0 || R[6] >= v[7]) conds |= 1u << j;
    for (int b = 31; b >= 0; --b) {   /* R = (R * 2^32 + u[j]) mod v, one bit at a time */
      u32 carry = R[7] >> 31;
      shl1(R);
      R[0] |= (u[j] >> b) & 1u;
      if (carry || cmpu(R, v) >= 0) sub(R, v, R);
    }
  }
  return conds;
}

long long odag_div_paths(const int32_t* nodes, int nn, const u32* consts, const int32_t* specs, const u32* pool,
                         u64 seed, u64 begin, u64 n, int wave, int nthreads, u64* out) {
  const onode* g = (const onode*)nodes;
  int ndiv = 0;
  int* divs = (int*)malloc(sizeof(int) * (size_t)(nn + 1));
  for (int i = 0; i < nn; ++i)
    if (g[i].op >= O_UDIV && g[i].op <= O_SMOD && g[i].w > 32) divs[ndiv++] = i;
  if (wave < 1) wave = 1;
  g_specs = (const ospec*)specs;
  g_pool = pool;
  u64 steps = 0, full = 0, shrt = 0, gen = 0;
  const long long nwaves = (long long)((n + (u64)wave - 1) / (u64)wave);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : steps, full, shrt, gen)
  {
    u32* V = (u32*)malloc(sizeof(u32) * 8 * (size_t)nn);
    u32* X = (u32*)malloc(sizeof(u32) * 8 * (size_t)(ndiv + 1) * (size_t)wave);
    u32* Y = (u32*)malloc(sizeof(u32) * 8 * (size_t)(ndiv + 1) * (size_t)wave);
#pragma omp for schedule(dynamic, 4)
    for (long long wv = 0; wv < nwaves; ++wv) {
      const u64 first = begin + (u64)wv * (u64)wave;
      u64 lanes = n - (u64)wv * (u64)wave;
      if (lanes > (u64)wave) lanes = (u64)wave;
      /* every lane of the wave runs (lanes past the range too: their index is
       * evaluated, only valid lanes are counted) */
      for (int l = 0; l < wave; ++l) {
        const u64 cand = first + (u64)l;
        for (int i = 0; i < nn; ++i) eval1(g, consts, i, V, seed, cand);
        for (int d = 0; d < ndiv; ++d)
          div_operands(g, divs[d], V, X + 8 * ((size_t)d * wave + l), Y + 8 * ((size_t)d * wave + l));
      }
      for (int d = 0; d < ndiv; ++d) {
        const u32* Yd = Y + 8 * (size_t)d * wave;
        const u32* Xd = X + 8 * (size_t)d * wave;
        int all_full = 1, all_short = 1;
        for (int l = 0; l < wave; ++l) {
          const u32* yl = Yd + 8 * l;
          if (yl[7] == 0) all_full = 0;
          for (int k = 1; k < 8; ++k) if (yl[k]) all_short = 0;
        }
        if (all_full) { full += lanes; continue; }
        if (all_short) { shrt += lanes; continue; }
        gen += lanes;
        u32 any = 0;
        for (int l = 0; l < wave; ++l) any |= general_conds(Xd + 8 * l, Yd + 8 * l);
        steps += lanes * (u64)__builtin_popcount(any);
      }
    }
    free(V); free(X); free(Y);
  }
  g_specs = 0;
  g_pool = 0;
  free(divs);
  out[0] = steps; out[1] = full; out[2] = shrt; out[3] = gen;
  return ndiv;
}

int odag_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
