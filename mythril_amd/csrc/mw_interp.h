// mw_interp.h — bytecode interpreter for one candidate per lane.
//
// The instruction stream is wave-uniform: every lane of a wavefront executes
// the same program on its own candidate assignment, so `pc`, the opcode and
// every slot index live in SGPRs (s_load_dwordx4 per instruction) and the
// dispatch `switch` is a scalar branch tree.  The W file (MW_NW x 8 limbs) and
// N file (MW_NN x 1) are ext_vector values indexed by a uniform slot number,
// which hipcc lowers to `s_set_gpr_idx_on` + v_mov — the file never leaves the
// VGPRs (checked in tests/test_build.py against the gfx950 ISA: no scratch).
//
// Env policy (device kernel or host emulator) supplies:
//   void leaf(u32 idx, u32 out[8]);            candidate value of leaf `idx`
//   void store(u32 row, const u32* v, int n);  trace rows (mg_eval)
//   void spill(u32 slot, const u32* v, int n); void fill(u32 slot, u32* v, int n);
//   bool none(bool alive);                     wave-wide "no lane alive"
//   u32 dsteps;                                division digit steps run (mw_alu.h udivrem8)
#pragma once
#include "mw_alu.h"
#include "mw_isa.h"
#include "mw_prog.h"

namespace mw {

// The program and its constant pool are read through the constant address
// space on the device: with a uniform index that makes every instruction fetch
// an s_load into SGPRs and keeps the opcode, slot numbers and constants
// wave-uniform (a generic pointer read from a struct would compile to a vector
// load and a divergent, exec-masked dispatch with waterfall register indexing).
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) u32* kptr;
#else
typedef const u32* kptr;
#endif
#define MW_KPTR(p) ((kptr)(p))
typedef u32 u32x4v __attribute__((ext_vector_type(4), aligned(4)));   // SMEM needs only dword alignment
typedef u32 u32x8v __attribute__((ext_vector_type(8), aligned(4)));
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) u32x4v* kptr4;
typedef const __attribute__((address_space(4))) u32x8v* kptr8;
#else
typedef const u32x4v* kptr4;
typedef const u32x8v* kptr8;
#endif
// one instruction (4 words at a 16-byte-aligned word index) as ONE scalar load:
// with pc advanced on several paths, element-wise reads became four s_load_dword
#define MW_LOAD_INSN(at, a, b, c, d)                                          \
  do {                                                                        \
    const u32x4v _v = *(kptr4)(code + (at));                                  \
    a = _v.x; b = _v.y; c = _v.z; d = _v.w;                                   \
  } while (0)
#define MW_KPAD 72   // minimum constant-region words (>= MW_NN + 8, see MW_FETCH_N)

// W file: four vectors, F<k> holding limb k of every slot (elements 0..NW-1)
// and limb k+4 (elements NW..2NW-1).  A 16-element vector read or written at a
// uniform index is lowered to s_set_gpr_idx + v_mov; an 8-element one (one
// vector per limb) was expanded into compare + v_cndmask chains, ~16
// instructions per limb and ~250 per W operand fetch + write-back.
typedef u32 u32xW __attribute__((ext_vector_type(2 * MW_NW)));
typedef u32 u32xN __attribute__((ext_vector_type(32)));      // one half of the N file
// (the N file is two 32-slot halves: a single 64-element vector indexed at run
// time is lowered through scratch memory, two halves stay in VGPRs)
// slot numbers are validated on load (mw_validate.cpp); the clamp keeps an
// index inside its vector regardless (one scalar min on a uniform value)
#define MW_WSLOT(o) ((o) < (u32)MW_NW ? (o) : 0u)

#define MW_FETCH_W(opnd, x)                                                   \
  do {                                                                        \
    u32 _o = (opnd);                                                          \
    if (_o & MW_KBIT) {                                                       \
      kptr _p = cpool + (_o & 0x7fffu);                                       \
      x[0] = _p[0]; x[1] = _p[1]; x[2] = _p[2]; x[3] = _p[3];                 \
      x[4] = _p[4]; x[5] = _p[5]; x[6] = _p[6]; x[7] = _p[7];                 \
    } else {                                                                  \
      _o = MW_WSLOT(_o);                                                      \
      x[0] = F0[_o]; x[1] = F1[_o]; x[2] = F2[_o]; x[3] = F3[_o];             \
      x[4] = F0[_o + MW_NW]; x[5] = F1[_o + MW_NW];                           \
      x[6] = F2[_o + MW_NW]; x[7] = F3[_o + MW_NW];                           \
    }                                                                         \
  } while (0)

// Both N halves are read and one is selected (a uniform branch here costs
// ~10 scalar instructions of structurizer flow); the constant-pool load stays
// behind a branch, so register operands issue no scalar load (which would wait
// out the next instruction's prefetch).
#define MW_FETCH_N(opnd, v)                                                   \
  do {                                                                        \
    const u32 _o = (opnd);                                                    \
    const u32 _h = NH[_o & 31u], _f = NF[_o & 31u];                           \
    v = (_o & 32u) ? _h : _f;                                                 \
    if (_o & MW_KBIT) v = cpool[_o & 0x7fffu];                                \
  } while (0)

#define MW_WRITE_W(d, r)                                                      \
  do {                                                                        \
    u32 _d = MW_WSLOT((u32)(d));                                              \
    F0[_d] = r[0]; F1[_d] = r[1]; F2[_d] = r[2]; F3[_d] = r[3];               \
    F0[_d + MW_NW] = r[4]; F1[_d + MW_NW] = r[5];                             \
    F2[_d + MW_NW] = r[6]; F3[_d + MW_NW] = r[7];                             \
  } while (0)

#define MW_WRITE_N(d, v)                                                      \
  do {                                                                        \
    if ((d) & 32u) NH[(d) & 31u] = (v);                                       \
    else NF[(d) & 31u] = (v);                                                 \
  } while (0)

template <class Env>
MW_HD bool mw_run(const u32* __restrict__ code_, const u32* __restrict__ cpool_, Env& env,
                  bool alive, u32 flags) {
  const kptr code = MW_KPTR(code_);
  const kptr cpool = MW_KPTR(cpool_);
  u32xW F0 = 0, F1 = 0, F2 = 0, F3 = 0;
  u32xN NF = 0, NH = 0;   // N slots 0..31, 32..63
  // Instruction fetch is software-pipelined: the next instruction's s_load is in
  // flight while the current one executes (the words after END are always
  // readable: the constant pool follows the code in the program buffer).
  u32 w0 = code[0], w1 = code[1], w2 = code[2], w3 = code[3];
  bool stop = false;
  // ONE loop exit (END or a uniform early stop): a return inside the switch
  // would make LLVM's CFG structurizer thread flag variables and exec-mask
  // arithmetic through every iteration.
  for (u32 pc = 4;; pc += 4) {
    const u32 op = w0 & 0xffu;
    if (op == MW_END || stop) break;
    u32 w = w0 >> 16;   // w, dst, imm: a W_CDINS chain leaves its last instruction's here
    u32 dst = w1 & 0xffffu;
    const u32 oa = w1 >> 16, ob = w2 & 0xffffu, oc = w2 >> 16;
    u32 imm = w3;
    // decode above, prefetch below: scalar loads return out of order, so the
    // lgkmcnt(0) guarding this instruction's words must not also cover the
    // next instruction's load (the barrier stops the load being hoisted).
    asm volatile("" ::: "memory");
    u32 n0, n1, n2, n3;
    MW_LOAD_INSN(pc, n0, n1, n2, n3);
    u32 x[8], y[8];
    u32 r[8];   // the op's result; limbs an op does not set go to scratch slots only
    switch (op) {
      case MW_CHECK: {  // runs of CHECKs as above
        u32 fa = oa;
        for (;;) {
          u32 v;
          MW_FETCH_N(fa, v);
          alive = alive && (v != 0);
          if ((n0 & 0xffu) != MW_CHECK) break;
          fa = n1 >> 16;
          pc += 4;
          asm volatile("" ::: "memory");
          MW_LOAD_INSN(pc, n0, n1, n2, n3);
        }
        // wave-uniform: stop at the next loop top (keeps one loop exit)
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_CHECK_IMP: {
        u32 p, q;
        MW_FETCH_N(oa, p);
        MW_FETCH_N(ob, q);
        alive = alive && (p == 0u || q != 0u);
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_CHECK_IMPEQ: {  // a => (b = c): a congruence conjunct over narrow cells
        // Runs of CHECK_IMPEQ (C3: 2 176 congruence conjuncts in a row) stay in
        // this case, two instructions per scalar load (s_load_dwordx8),
        // without the dispatch tree and write-back (~150 scalar and vector
        // instructions per dispatch).  pc keeps indexing the next instruction.
#define MW_IMPEQ_STEP(fa, fb, fc)                                             \
  do {                                                                        \
    u32 _p, _b, _c;                                                           \
    MW_FETCH_N(fa, _p);                                                       \
    MW_FETCH_N(fb, _b);                                                       \
    MW_FETCH_N(fc, _c);                                                       \
    alive = alive && (_p == 0u || _b == _c);                                  \
  } while (0)
        MW_IMPEQ_STEP(oa, ob & 0xffffu, oc);
        while ((n0 & 0xffu) == MW_CHECK_IMPEQ) {
          asm volatile("" ::: "memory");
          const u32x8v q = *(kptr8)(code + pc + 4);  // the two instructions after n
          MW_IMPEQ_STEP(n1 >> 16, n2 & 0xffffu, n2 >> 16);
          pc += 4;
          if ((q[0] & 0xffu) != MW_CHECK_IMPEQ) { n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; break; }
          MW_IMPEQ_STEP(q[1] >> 16, q[2] & 0xffffu, q[2] >> 16);
          pc += 4;
          n0 = q[4]; n1 = q[5]; n2 = q[6]; n3 = q[7];
        }
#undef MW_IMPEQ_STEP
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_CHECK_IMPEQK: {  // (N[a] = imm) => (b = c): a keyed congruence premise, runs as above
#define MW_IMPEQK_STEP(fa, fb, fc, k)                                         \
  do {                                                                        \
    u32 _p, _b, _c;                                                           \
    MW_FETCH_N(fa, _p);                                                       \
    MW_FETCH_N(fb, _b);                                                       \
    MW_FETCH_N(fc, _c);                                                       \
    alive = alive && (_p != (k) || _b == _c);                                 \
  } while (0)
        MW_IMPEQK_STEP(oa, ob, oc, imm);
        while ((n0 & 0xffu) == MW_CHECK_IMPEQK) {
          asm volatile("" ::: "memory");
          const u32x8v q = *(kptr8)(code + pc + 4);
          MW_IMPEQK_STEP(n1 >> 16, n2 & 0xffffu, n2 >> 16, n3);
          pc += 4;
          if ((q[0] & 0xffu) != MW_CHECK_IMPEQK) { n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3]; break; }
          MW_IMPEQK_STEP(q[1] >> 16, q[2] & 0xffffu, q[2] >> 16, q[3]);
          pc += 4;
          n0 = q[4]; n1 = q[5]; n2 = q[6]; n3 = q[7];
        }
#undef MW_IMPEQK_STEP
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_CHECK_GRID: {  // one row of a congruence grid (compiler.py _form_grids)
        u32 key, v;
        MW_FETCH_N(oa, key);
        MW_FETCH_N(ob, v);
        const u32 j = imm - key;
        if (j <= ((oc >> 10) & 31u)) {
          env.fill((oc & 1023u) + j, x, 1);   // a per-lane word (fill writes x[0..7])
          alive = alive && x[0] == v;
        }
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_CHECK_IMPEQW: {
        u32 p;
        MW_FETCH_N(oa, p);
        MW_FETCH_W(ob, x);
        MW_FETCH_W(oc, y);
        alive = alive && (p == 0u || eq8(x, y));
        if (flags & MW_FLAG_EARLY_EXIT) stop = env.none(alive);
        break;
      }
      case MW_W_CDINS: {  // acc | (ite(K[c] <s size, leaf, 0) << off)
        // A calldata word is built by a chain of these (32 per ABI word: 22 %
        // of the LASER corpus's instructions).  MW_FLAG_CHAIN (set by the
        // compiler, checked by the validator) says the next instruction is a
        // W_CDINS whose only input from here is this result as its acc: the
        // chain runs inside this case with the word kept in registers, and the
        // last result goes through the common write-back (w, dst, imm are the
        // last instruction's).
        u32 fb = ob, fc = oc, fl = w0;
        MW_FETCH_W(oa, x);
        for (;;) {
          MW_FETCH_W(fb, y);   // size
          u32 k[8];
          MW_FETCH_W(fc, k);   // the constant index
          k[7] ^= 0x80000000u;
          y[7] ^= 0x80000000u;
          const bool in_range = ult8(k, y);   // signed 256-bit k < size
          env.leaf(imm & 0xffffu, r);
          u32 t[8];
          zero8(t);
          t[0] = in_range ? r[0] : 0u;
          shl8(t, imm >> 16, r);
#pragma unroll
          for (int q = 0; q < 8; ++q) r[q] |= x[q];
          if (!(fl & (MW_FLAG_CHAIN << 8))) break;
          if (w - 1u < 255u) canon(r, w);
          copy8(x, r);
          fl = n0;
          w = n0 >> 16;
          dst = n1 & 0xffffu;
          fb = n2 & 0xffffu;
          fc = n2 >> 16;
          imm = n3;
          pc += 4;
          asm volatile("" ::: "memory");
          MW_LOAD_INSN(pc, n0, n1, n2, n3);
        }
        break;
      }
      case MW_LEAF_W:
        env.leaf(imm, r);
        break;
      case MW_LEAF_N:
        env.leaf(imm, r);
        break;
      case MW_STORE_W:
        MW_FETCH_W(oa, x);
        env.store(imm, x, 8);
        break;
      case MW_STORE_N: {
        MW_FETCH_N(oa, x[0]);
        env.store(imm, x, 1);
        break;
      }
      case MW_SPILL_W:
        MW_FETCH_W(oa, x);
        env.spill(imm, x, 8);
        break;
      case MW_FILL_W:
        env.fill(imm, r, 8);
        break;
      case MW_SPILL_N:
        MW_FETCH_N(oa, x[0]);
        env.spill(imm, x, 1);
        break;
      case MW_FILL_N:
        env.fill(imm, r, 1);
        break;
      case MW_MOV_W:
        MW_FETCH_W(oa, x);
        copy8(r, x);
        break;
      case MW_MOV_N: {
        u32 v;
        MW_FETCH_N(oa, v);
        r[0] = v;
        break;
      }

      // ---------------------------------------------------------- wide
      case MW_W_ADD:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        add8(x, y, r);
        break;
      case MW_W_SUB:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        sub8(x, y, r);
        break;
      case MW_W_MUL:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        mul8(x, y, r);
        break;
      case MW_W_AND:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = x[k] & y[k];
        break;
      case MW_W_OR:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = x[k] | y[k];
        break;
      case MW_W_XOR:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = x[k] ^ y[k];
        break;
      case MW_W_NOT:
        MW_FETCH_W(oa, x);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = ~x[k];
        break;
      case MW_W_SHL:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        wshl(x, y, w, r);
        break;
      case MW_W_LSHR:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        wlshr(x, y, w, r);
        break;
      case MW_W_ASHR:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        washr(x, y, w, r);
        break;
      case MW_W_UDIV:
      case MW_W_UREM:
      case MW_W_SDIV:
      case MW_W_SREM:
      case MW_W_SMOD:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        wdiv((int)(op - MW_W_UDIV), x, y, w, r, &env.dsteps);
        break;
      case MW_W_ITE: {
        u32 c;
        MW_FETCH_N(oc, c);
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = c ? x[k] : y[k];
        break;
      }
      case MW_W_SHLI:
        MW_FETCH_W(oa, x);
        shl8(x, imm, r);
        break;
      case MW_W_LSHRI:
        MW_FETCH_W(oa, x);
        shr8(x, imm, 0u, r);
        break;
      case MW_W_ZEXTN: {
        u32 v;
        MW_FETCH_N(oa, v);
        zero8(r);
        r[0] = v;
        break;
      }
      case MW_W_SEXT:
        MW_FETCH_W(oa, x);
        sext8(x, imm);
        copy8(r, x);
        break;
      case MW_W_SEXTN: {
        u32 v;
        MW_FETCH_N(oa, v);
        zero8(r);
        r[0] = v;
        sext8(r, imm);
        break;
      }
      case MW_W_INSN: {
        u32 v;
        MW_FETCH_W(oa, x);
        MW_FETCH_N(ob, v);
        zero8(y);
        y[0] = v;
        shl8(y, imm, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] |= x[k];
        break;
      }

      // ---------------------------------------------------------- wide -> narrow
      case MW_N_EXTRACTW: {
        MW_FETCH_W(oa, x);
        shr8(x, imm, 0u, r);
        r[0] = r[0] & nmask(w);
        break;
      }
      case MW_N_ULT:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        r[0] = ult8(x, y) ? 1u : 0u;
        break;
      case MW_N_ULE:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        r[0] = ult8(y, x) ? 0u : 1u;
        break;
      case MW_N_SLT:
      case MW_N_SLE: {
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        // flip the sign bit (bit w-1) of both, then compare unsigned
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int bit = (int)w - 1 - 32 * k;
          u32 m = (bit >= 0 && bit < 32) ? (1u << bit) : 0u;
          x[k] ^= m;
          y[k] ^= m;
        }
        bool lt = (op == MW_N_SLT) ? ult8(x, y) : !ult8(y, x);
        r[0] = lt ? 1u : 0u;
        break;
      }
      case MW_N_EQ:
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        r[0] = eq8(x, y) ? 1u : 0u;
        break;
      case MW_N_UMULNO: {
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        u32 hi[8];
        mulhi8(x, y, r, hi);
        u32 ov = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) ov |= (r[k] & ~limb_mask(w, k)) | hi[k];
        r[0] = ov ? 0u : 1u;
        break;
      }
      case MW_N_ADDC: {
        MW_FETCH_W(oa, x);
        MW_FETCH_W(ob, y);
        u32 c = add8(x, y, r);
        u32 bit = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int b = (int)w - 32 * k;
          bit |= (b >= 0 && b < 32) ? ((r[k] >> b) & 1u) : 0u;
        }
        r[0] = (w >= 256) ? c : bit;
        break;
      }

      // ---------------------------------------------------------- narrow
      // one case per opcode in the single dispatch switch (a nested switch
      // under `default` doubled the scalar branch tree for every narrow op)
#define MW_N2(OPC, EXPR)                                                      \
  case OPC: {                                                                 \
    u32 a, b;                                                                 \
    MW_FETCH_N(oa, a);                                                        \
    MW_FETCH_N(ob, b);                                                        \
    const u32 m = nmask(w);                                                   \
    (void)m;                                                                  \
    r[0] = (EXPR);                                                            \
    break;                                                                    \
  }
#define MW_N1(OPC, EXPR)                                                      \
  case OPC: {                                                                 \
    u32 a;                                                                    \
    MW_FETCH_N(oa, a);                                                        \
    const u32 m = nmask(w);                                                   \
    (void)m;                                                                  \
    r[0] = (EXPR);                                                            \
    break;                                                                    \
  }
      MW_N2(MW_N_ADD, (a + b) & m)
      MW_N2(MW_N_SUB, (a - b) & m)
      MW_N2(MW_N_MUL, (a * b) & m)
      MW_N2(MW_N_AND, a & b)
      MW_N2(MW_N_OR, a | b)
      MW_N2(MW_N_XOR, a ^ b)
      MW_N1(MW_N_NOT, (~a) & m)
      MW_N2(MW_N_SHL, n_shl(a, b, w))
      MW_N2(MW_N_LSHR, n_lshr(a, b, w))
      MW_N2(MW_N_ASHR, n_ashr(a, b, w))
      MW_N2(MW_N_UDIV, n_div(0, a, b, w))
      MW_N2(MW_N_UREM, n_div(1, a, b, w))
      MW_N2(MW_N_SDIV, n_div(2, a, b, w))
      MW_N2(MW_N_SREM, n_div(3, a, b, w))
      MW_N2(MW_N_SMOD, n_div(4, a, b, w))
      case MW_N_ITE: {
        u32 a, b, c;
        MW_FETCH_N(oa, a);
        MW_FETCH_N(ob, b);
        MW_FETCH_N(oc, c);
        r[0] = c ? a : b;
        break;
      }
      MW_N1(MW_N_SHLI, (imm >= 32 ? 0u : (a << imm)) & m)
      MW_N1(MW_N_LSHRI, (imm >= 32 ? 0u : (a >> imm)) & m)
      MW_N1(MW_N_SEXT, n_sext(a, imm) & m)
      MW_N2(MW_N_ULTN, a < b ? 1u : 0u)
      MW_N2(MW_N_ULEN, a <= b ? 1u : 0u)
      MW_N2(MW_N_SLTN, n_slt(a, b, w))
      MW_N2(MW_N_SLEN, n_sle(a, b, w))
      MW_N2(MW_N_EQN, a == b ? 1u : 0u)
      MW_N2(MW_N_UMULNON, n_umulno(a, b, w))
      MW_N2(MW_N_ADDCN, (u32)((((u64)a + b) >> w) & 1u))
#undef MW_N1
#undef MW_N2
      default:
        break;  // unreachable: opcodes are validated on load
    }
    // Single, UNCONDITIONAL write-back to the targets the compiler encoded in
    // dst (mw_prog.h): W slot, N-low slot, N-high slot, each the reserved
    // scratch slot when the op does not write that file.  A conditional
    // indexed write leaves two versions of a file live at the loop latch and
    // the register allocator resolves that with a whole-file copy per dispatch
    // (32 v_mov_b64 for the N file); per-op write kinds cost ~35 scalar
    // instructions of selects and lane-mask flow.  Here: 8 + 2 indexed moves.
    // wide ops (16..38) of width 33..255: clear bits >= w (narrow ops mask their
    // result; leaves, fills and moves are canonical already)
    if (op - (u32)MW_W_ADD <= (u32)(MW_W_CDINS - MW_W_ADD) && w - 33u < 223u) canon(r, w);
    {
      const u32 dw = MW_DST_W(dst), dlo = MW_DST_NLO(dst), dhi = MW_DST_NHI(dst);
      F0[dw] = r[0]; F1[dw] = r[1]; F2[dw] = r[2]; F3[dw] = r[3];
      F0[dw + MW_NW] = r[4]; F1[dw + MW_NW] = r[5]; F2[dw + MW_NW] = r[6]; F3[dw + MW_NW] = r[7];
      NF[dlo] = r[0];
      NH[dhi] = r[0];
    }
    w0 = n0;
    w1 = n1;
    w2 = n2;
    w3 = n3;
  }
  return alive && !stop;
}

}  // namespace mw
