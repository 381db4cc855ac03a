// mw_validate.cpp — program validation and error reporting shared by the
// device library (libmythril_witness.so) and the host emulator.  Every program
// is checked before upload: opcodes, operand slots, constant-pool offsets,
// widths, leaf/pool/trace/spill ranges, and a terminating END — so the
// interpreter loop can never run off the stream or index out of its files.
#include <stdint.h>

#include <algorithm>
#include <string>

#include "../../include/mythril_witness.h"
#include "mw_asm_interp.inc"   // MW_ASM_NFUSED / MW_ASM_FUSED_SEQS (macros only here)
#include "mw_isa.h"
#include "mw_prog.h"

typedef uint32_t u32;
typedef uint64_t u64;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// operand classes per opcode: returns false for unknown opcodes
// kinds: 0 none, 1 W-or-K source, 2 N-or-K source, 3 W dst, 4 N dst
struct OpShape {
  int dst, a, b, c;
  bool wide;  // width rules: wide ops 1..256, narrow 1..32
};

bool op_shape(u32 op, OpShape& s) {
  s = OpShape{0, 0, 0, 0, false};
  switch (op) {
    case MW_END: return true;
    case MW_CHECK: s.a = 2; return true;
    case MW_CHECK_IMP: s.a = 2; s.b = 2; return true;
    case MW_CHECK_IMPEQ: s.a = 2; s.b = 2; s.c = 2; return true;
    case MW_CHECK_IMPEQW: s.a = 2; s.b = 1; s.c = 1; return true;
    case MW_CHECK_IMPEQK: s.a = 2; s.b = 2; s.c = 2; return true;
    case MW_CHECK_GRID: s.a = 2; s.b = 2; return true;   // c: the table's word and size, raw
    case MW_W_CDINS: s.dst = 3; s.a = 1; s.b = 1; s.c = 1; s.wide = true; return true;
    case MW_LEAF_W: s.dst = 3; return true;
    case MW_LEAF_N: s.dst = 4; return true;
    case MW_STORE_W: s.a = 1; return true;
    case MW_STORE_N: s.a = 2; return true;
    case MW_SPILL_W: s.a = 1; return true;
    case MW_FILL_W: s.dst = 3; return true;
    case MW_SPILL_N: s.a = 2; return true;
    case MW_FILL_N: s.dst = 4; return true;
    case MW_MOV_W: s.dst = 3; s.a = 1; return true;
    case MW_MOV_N: s.dst = 4; s.a = 2; return true;
    case MW_W_ADD: case MW_W_SUB: case MW_W_MUL: case MW_W_AND: case MW_W_OR: case MW_W_XOR:
    case MW_W_SHL: case MW_W_LSHR: case MW_W_ASHR: case MW_W_UDIV: case MW_W_UREM:
    case MW_W_SDIV: case MW_W_SREM: case MW_W_SMOD:
      s.dst = 3; s.a = 1; s.b = 1; s.wide = true; return true;
    case MW_W_NOT: case MW_W_SHLI: case MW_W_LSHRI: case MW_W_SEXT:
      s.dst = 3; s.a = 1; s.wide = true; return true;
    case MW_W_ITE: s.dst = 3; s.a = 1; s.b = 1; s.c = 2; s.wide = true; return true;
    case MW_W_ZEXTN: case MW_W_SEXTN: s.dst = 3; s.a = 2; s.wide = true; return true;
    case MW_W_INSN: s.dst = 3; s.a = 1; s.b = 2; s.wide = true; return true;
    case MW_N_EXTRACTW: s.dst = 4; s.a = 1; return true;
    case MW_N_ULT: case MW_N_ULE: case MW_N_SLT: case MW_N_SLE: case MW_N_EQ:
    case MW_N_UMULNO: case MW_N_ADDC:
      s.dst = 4; s.a = 1; s.b = 1; s.wide = true; return true;
    case MW_N_ADD: case MW_N_SUB: case MW_N_MUL: case MW_N_AND: case MW_N_OR: case MW_N_XOR:
    case MW_N_SHL: case MW_N_LSHR: case MW_N_ASHR: case MW_N_UDIV: case MW_N_UREM:
    case MW_N_SDIV: case MW_N_SREM: case MW_N_SMOD: case MW_N_ULTN: case MW_N_ULEN:
    case MW_N_SLTN: case MW_N_SLEN: case MW_N_EQN: case MW_N_UMULNON: case MW_N_ADDCN:
      s.dst = 4; s.a = 2; s.b = 2; return true;
    case MW_N_NOT: case MW_N_SHLI: case MW_N_LSHRI: case MW_N_SEXT:
      s.dst = 4; s.a = 2; return true;
    case MW_N_ITE: s.dst = 4; s.a = 2; s.b = 2; s.c = 2; return true;
    default: return false;
  }
}

bool w_slot_ok(u32 f) { return f < MW_NW && f != MW_W_RESERVED; }
bool n_slot_ok(u32 f) { return f < MW_NN && (f & 31u) != MW_N_RESERVED; }

bool check_operand(int kind, u32 f, size_t nconst) {
  if (kind == 0) return true;
  if (kind == 3) return w_slot_ok(f);
  if (kind == 4) return n_slot_ok(f);
  if (f & MW_KBIT) {
    size_t o = f & 0x7fffu;
    return o + (kind == 1 ? 8 : 1) <= nconst;
  }
  return kind == 1 ? w_slot_ok(f) : n_slot_ok(f);
}

}  // namespace

extern "C" {

int mw_fail(int code, const char* msg) {
  g_err = msg ? msg : "";
  return code;
}

const char* mg_last_error(void) { return g_err.c_str(); }

int mg_validate_desc(const mg_prog_desc* d) {
  if (!d || !d->code || d->ncode_words < 4 || d->ncode_words % 4)
    return fail(MG_E_PROG, "code must be a non-empty multiple of 4 words");
  if (d->nleaves && !d->leaves) return fail(MG_E_PROG, "leaf table missing");
  if (d->nconst_words > 0x8000) return fail(MG_E_PROG, "constant pool exceeds 32768 words");
  const size_t n = d->ncode_words / 4;
  if ((d->code[4 * (n - 1)] & 0xffu) != MW_END) return fail(MG_E_PROG, "program must end with END");
  for (size_t i = 0; i < n; ++i) {
    const u32* I = d->code + 4 * i;
    const u32 op = I[0] & 0xffu, w = I[0] >> 16;
    OpShape s;
    if (!op_shape(op, s)) return fail(MG_E_PROG, "unknown opcode " + std::to_string(op) + " at " + std::to_string(i));
    if (op == MW_END && i != n - 1) return fail(MG_E_PROG, "END before the last instruction");
    const u32 dst = I[1] & 0xffffu, a = I[1] >> 16, b = I[2] & 0xffffu, c = I[2] >> 16;
    const u32 iflags = (I[0] >> 8) & 0xffu;
    if (iflags) {   // only a W_CDINS chain link, followed by the W_CDINS that reads it as its acc
      const u32* N = I + 4;
      // the link's result stays in registers and is never written back, so the
      // consumer may read it only as its acc operand: a size operand naming the
      // same slot would read the stale slot
      if (iflags != MW_FLAG_CHAIN || op != MW_W_CDINS || i + 1 >= n || (N[0] & 0xffu) != MW_W_CDINS ||
          (N[1] >> 16) != MW_DST_W(dst) || (N[2] & 0xffffu) == MW_DST_W(dst))
        return fail(MG_E_PROG, "bad instruction flags at " + std::to_string(i));
    }
    // dst = write targets (mw_prog.h): the file the op writes names a real slot,
    // the others their scratch slot
    {
      const u32 dw = MW_DST_W(dst), dl = MW_DST_NLO(dst), dh = MW_DST_NHI(dst);
      bool ok = (dst >> 13) == 0u;
      if (s.dst == 3) ok = ok && dw != MW_W_RESERVED && dl == MW_N_RESERVED && dh == MW_N_RESERVED;
      else if (s.dst == 4) ok = ok && dw == MW_W_RESERVED && ((dl == MW_N_RESERVED) != (dh == MW_N_RESERVED));
      else ok = ok && dst == MW_DST_SCRATCH;
      if (!ok) return fail(MG_E_PROG, "bad write targets at instruction " + std::to_string(i));
    }
    if (!check_operand(s.a, a, d->nconst_words) ||
        !check_operand(s.b, b, d->nconst_words) || !check_operand(s.c, c, d->nconst_words))
      return fail(MG_E_PROG, "operand out of range at instruction " + std::to_string(i));
    if (s.dst == 3 || s.dst == 4 || s.a || s.b) {
      const u32 maxw = (s.wide || s.dst == 3) ? 256u : 32u;
      if (op != MW_CHECK && op != MW_CHECK_IMP && op != MW_CHECK_IMPEQ && op != MW_CHECK_IMPEQW &&
          op != MW_CHECK_IMPEQK && op != MW_CHECK_GRID && op != MW_STORE_W && op != MW_STORE_N && op != MW_SPILL_W &&
          op != MW_SPILL_N && op != MW_FILL_W && op != MW_FILL_N && op != MW_MOV_W && op != MW_MOV_N &&
          op != MW_LEAF_W && op != MW_LEAF_N && (w < 1 || w > maxw))
        return fail(MG_E_PROG, "bad width " + std::to_string(w) + " at instruction " + std::to_string(i));
    }
    switch (op) {
      case MW_LEAF_W: case MW_LEAF_N:
        if (I[3] >= d->nleaves) return fail(MG_E_PROG, "leaf index out of range");
        break;
      case MW_STORE_W:
        if ((u64)I[3] + 8 > d->n_trace_rows) return fail(MG_E_PROG, "trace row out of range");
        break;
      case MW_STORE_N:
        if ((u64)I[3] + 1 > d->n_trace_rows) return fail(MG_E_PROG, "trace row out of range");
        break;
      case MW_SPILL_W: case MW_FILL_W:   // imm = word offset of an 8-word slot in the spill area
        if ((u64)I[3] + 8 > d->n_spill) return fail(MG_E_PROG, "spill slot out of range");
        break;
      case MW_SPILL_N: case MW_FILL_N:
        if (I[3] >= d->n_spill) return fail(MG_E_PROG, "spill slot out of range");
        break;
      case MW_W_SHLI: case MW_W_LSHRI: case MW_N_EXTRACTW: case MW_W_INSN:
        if (I[3] >= 256) return fail(MG_E_PROG, "immediate shift out of range");
        break;
      case MW_W_CDINS:   // leaf index | insert offset << 16; c must be a constant (the byte index)
        if ((I[3] & 0xffffu) >= d->nleaves) return fail(MG_E_PROG, "leaf index out of range");
        if ((I[3] >> 16) >= 256) return fail(MG_E_PROG, "immediate shift out of range");
        if (!(c & MW_KBIT)) return fail(MG_E_PROG, "W_CDINS index must be a constant");
        break;
      case MW_W_SEXT: case MW_W_SEXTN: case MW_N_SEXT:
        if (I[3] < 1 || I[3] > w) return fail(MG_E_PROG, "bad sign-extension source width");
        break;
      case MW_CHECK_GRID:   // the table's words lie in the spill area
        if (c >= 0x8000u || (u64)(c & 1023u) + ((c >> 10) & 31u) + 1 > d->n_spill)
          return fail(MG_E_PROG, "grid table out of range");
        break;
      default: break;
    }
  }
  for (size_t l = 0; l < d->nleaves; ++l) {
    const u32* L = d->leaves + l * MW_LEAF_WORDS;
    if (L[MW_LEAF_WIDTH] < 1 || L[MW_LEAF_WIDTH] > 256) return fail(MG_E_PROG, "bad leaf width");
    if (L[MW_LEAF_KIND] >= 1 && L[MW_LEAF_KIND] <= 3) {
      if (L[MW_LEAF_BITS] > 24 || L[MW_LEAF_SHIFT] > 63) return fail(MG_E_PROG, "bad pool digit field");
      if (L[MW_LEAF_KIND] == 3 && L[MW_LEAF_BITS] &&
          (u64)L[MW_LEAF_SHIFT] + (u64)(L[MW_LEAF_BITS] - 1) * L[MW_LEAF_STRIDE] > 63)
        return fail(MG_E_PROG, "interleaved digit beyond the 64-bit index");
      u64 need = (u64)L[MW_LEAF_POOL] + ((u64)1 << L[MW_LEAF_BITS]) * MW_POOL_ENTRY_WORDS_OF(L[MW_LEAF_WIDTH]);
      if (need > d->npool_words) return fail(MG_E_PROG, "pool out of range");
    } else if (L[MW_LEAF_KIND] != 0) {
      return fail(MG_E_PROG, "bad leaf kind");
    }
    if ((u64)L[MW_LEAF_INROW] + (L[MW_LEAF_WIDTH] + 31) / 32 > d->n_input_rows && d->n_input_rows)
      return fail(MG_E_PROG, "leaf input row out of range");
  }
  return 0;
}

// The asm interpreter's copy of a validated program (mw_asm_interp.inc reads
// operands without decoding them): word 1 becomes a [15:0] | dst [31:16] (a
// first: s_set_gpr_idx_on takes the index from bits [7:0] of the word), the
// dst field the written register's index in its file (N slot 0..63, or W
// slot x 8); a W register operand becomes its slot x 8 (the VGPR offset of
// its limb 0 in the W file), N register operands and W constants stay as they are, except a
// W_CDINS byte index (always a constant) below 0x4000, which becomes
// 0x4000 | index (the handler then compares it with one 32-bit summary of the
// size instead of a signed 256-bit subtraction).
// hoff: the asm interpreter's introspection table (MW_ASM_NHTAB words,
// reported by the kernel itself, mw_kernels.hip asm_handler_offsets): the
// handler word offsets from Lpc0 per opcode (128 entries, then the fused
// handlers') of bank A, the same for bank B, then Lpc0's address (low, high).
// Instruction i runs in bank i & 1 (mythril_amd/asmgen.py: the interpreter
// alternates two SGPR banks), so word 0 becomes the low word of its handler's
// absolute address in that bank: the dispatch moves it into the jump target
// and jumps (Gen.next).  The width moves to word 1 [31:24] (as width - 1) and
// W_CDINS's FLAG_CHAIN to bit 31 of its immediate.  Returns -3 when a handler
// address would carry into the high word (the kernel keeps one high word).
// Narrow constants: every N-class constant operand becomes a register operand
// naming one of MW_ASM_NK VGPRs above the N file (index MW_ASM_NK_INDEX + k
// from its base), which the kernel fills once per block from nk[0..MW_ASM_NK)
// (the distinct values, in first-use order): the operand fetch is then the
// same indexed move for registers and constants, with no constant test and
// no scalar load.  Returns -1 (nothing usable written) when the program has
// more distinct narrow constants than that (it then runs on the compiled
// interpreter; the corpora have at most 3).
// Width masks: N_ADD / N_SUB / N_MUL / N_NOT, which have no immediate, get
// their result mask (width < 32 ? 2^width - 1 : ~0) in word 3.
// Fused handlers: hoff has MW_ASM_NHANDLERS entries, the fused sequences'
// (MW_ASM_FUSED_SEQS, mythril_amd/isa.py ASM_FUSED) after the opcodes'.
// Scanning left to right, the first instruction of every match (longest
// sequence first, list order among equal lengths) gets its sequence's handler:
// one dispatch runs the whole sequence, which takes the instructions after
// the first itself (their own words are left as they are).
// Layouts (mythril_amd/asmgen.py, round 5): nk_index / nk_max place the narrow
// constants of the interpreter kernel the copy is for (the wide kernel:
// MW_ASM_NK_INDEX / MW_ASM_NK; the narrow-layout kernel: MW_ASM_NK_INDEX_N /
// MW_ASM_NK_N); nfile > 0 also requires every N register operand and N result
// to lie below nfile slots, wfile > 0 every W register operand and W result
// below wfile slots (-2 otherwise: the program needs a wider kernel).
int mw_asm_predecode_layout(const u32* code, size_t nwords, const u32* consts, size_t nconst, const u32* hoff,
                            u32* out, u32* nk, u32 nk_index, u32 nk_max, u32 nfile, u32 wfile) {
  u32 nnk = 0;
  for (u32 k = 0; k < MW_ASM_NK; ++k) nk[k] = 0;
  if (nk_max > MW_ASM_NK) return -1;
  const u32 nh = MW_ASM_NHANDLERS, lpc0 = hoff[2 * nh];
  for (u32 k = 0; k < 2 * nh; ++k)
    if (uint64_t(lpc0) + 4ull * hoff[k] > 0xffffffffull) return -3;
  auto target = [&](size_t insn, u32 h) { return lpc0 + 4u * hoff[(insn & 1u) * nh + h]; };
  auto narrow = [&](int kind, u32 f, u32* dst) -> bool {   // dst: the predecoded field
    if (kind != 2 || !(f & MW_KBIT)) return true;
    const u32 val = consts[f & 0x7fffu];
    u32 k = 0;
    while (k < nnk && nk[k] != val) ++k;
    if (k == nnk) {
      if (nnk == nk_max) return false;
      nk[nnk++] = val;
    }
    *dst = nk_index + k;
    return true;
  };
  auto in_file = [&](int kind, u32 f) {
    if (f & MW_KBIT) return true;
    if (kind == 2) return !nfile || f < nfile;
    if (kind == 1) return !wfile || f < wfile;
    return true;
  };
  for (size_t i = 0; i + 3 < nwords; i += 4) {
    const u32* I = code + i;
    u32* O = out + i;
    OpShape sh;
    (void)op_shape(I[0] & 0xffu, sh);   // validated: every opcode is known
    const u32 dst = I[1] & 0xffffu, a = I[1] >> 16, b = I[2] & 0xffffu, c = I[2] >> 16;
    u32 d2 = 0;   // the written register's index in its file: N slot, or W slot x 8
    if (sh.dst == 4) d2 = MW_DST_NLO(dst) != MW_N_RESERVED ? MW_DST_NLO(dst) : 32u + MW_DST_NHI(dst);
    else if (sh.dst == 3) d2 = MW_DST_W(dst) * 8u;
    auto opnd = [](int kind, u32 f) { return (kind == 1 && !(f & MW_KBIT)) ? f * 8u : f; };
    const u32 op = I[0] & 0xffu, w = I[0] >> 16;
    u32 a2 = opnd(sh.a, a), b2 = opnd(sh.b, b), c2 = opnd(sh.c, c);
    if (op == MW_W_CDINS && (c & MW_KBIT)) {
      const size_t o = c & 0x7fffu;   // validated: o + 8 <= nconst
      bool small = o + 8 <= nconst && consts[o] < 0x4000u;
      for (int k = 1; k < 8 && small; ++k) small = consts[o + k] == 0u;
      if (small) c2 = 0x4000u | consts[o];
    }
    if (!in_file(sh.a, a) || !in_file(sh.b, b) || !in_file(sh.c, c) || (nfile && sh.dst == 4 && d2 >= nfile) ||
        (wfile && sh.dst == 3 && MW_DST_W(dst) >= wfile))
      return -2;
    if (!narrow(sh.a, a, &a2) || !narrow(sh.b, b, &b2) || !narrow(sh.c, c, &c2)) return -1;
    const bool chain = op == MW_W_CDINS && ((I[0] >> 8) & MW_FLAG_CHAIN);
    if (chain && (I[3] & 0x80000000u)) return -1;   // validated: leaf index | offset < 256 << 16
    O[0] = target(i / 4, op & 0x7fu);
    // s_set_gpr_idx_on reads bits [7:0]: a indexes from the word as it is, dst
    // (< 64) from word 1 >> 16 with the width above it
    O[1] = a2 | (d2 << 16) | (((w - 1u) & 0xffu) << 24);
    O[2] = b2 | (c2 << 16);
    O[3] = I[3] | (chain ? 0x80000000u : 0u);
    // no immediate: the c operand goes to word 3 too (mythril_amd/asmgen.py
    // C_IN_IMM: the handler indexes with it as it is, no shift)
    if (op == MW_N_ITE || op == MW_W_ITE || op == MW_CHECK_IMPEQ || op == MW_CHECK_IMPEQW) O[3] = c2;
    // a CHECK_IMPEQ followed by another: the handler takes that one itself
    // (a chain, mythril_amd/asmgen.py), bit 31 above its c field
    if (op == MW_CHECK_IMPEQ && i + 7 < nwords && (code[i + 4] & 0xffu) == MW_CHECK_IMPEQ) O[3] |= 0x80000000u;
    // CHECK_IMPEQK: word 3 is the premise constant, so its chain flag is bit
    // 31 of word 1 (the width above a is not read by its handler)
    if (op == MW_CHECK_IMPEQK)
      O[1] = (O[1] & 0x7fffffffu) |
             (i + 7 < nwords && (code[i + 4] & 0xffu) == MW_CHECK_IMPEQK ? 0x80000000u : 0u);
    if (op == MW_N_ADD || op == MW_N_SUB || op == MW_N_MUL || op == MW_N_NOT)
      O[3] = w >= 32u ? 0xffffffffu : (1u << w) - 1u;
  }
  static const u32 seqs[MW_ASM_NFUSED][MW_ASM_FUSED_MAX] = {MW_ASM_FUSED_SEQS};
  const size_t n = nwords / 4;
  for (size_t i = 0; i < n;) {
    int best = -1;
    size_t blen = 0;
    for (int k = 0; k < MW_ASM_NFUSED; ++k) {
      size_t len = 0;
      while (len < MW_ASM_FUSED_MAX && seqs[k][len] != 0xffu) ++len;
      if (len <= blen || i + len > n) continue;
      bool ok = true;
      for (size_t j = 0; j < len && ok; ++j) ok = (code[(i + j) * 4] & 0xffu) == seqs[k][j];
      if (ok) {
        best = k;
        blen = len;
      }
    }
    if (best < 0) {
      ++i;
      continue;
    }
    out[i * 4] = target(i, 128u + u32(best));
    i += blen;
  }
  return 0;
}

int mw_asm_predecode(const u32* code, size_t nwords, const u32* consts, size_t nconst, const u32* hoff,
                     u32* out, u32* nk) {
  return mw_asm_predecode_layout(code, nwords, consts, nconst, hoff, out, nk, MW_ASM_NK_INDEX, MW_ASM_NK, 0, 0);
}

}  // extern "C"
