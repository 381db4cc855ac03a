// mw_isa.h — witness-engine bytecode ISA (shared by kernels, host emulator, and
// mirrored in mythril_amd/isa.py; tests/test_isa_sync.py checks they agree).
//
// A program evaluates the conjunction of a Mythril path-constraint set
// (mythril/laser/ethereum/state/constraints.py:10-108) for one candidate
// assignment per lane.  Values live in two per-lane register files:
//   W file: MW_NW slots x 8 u32 limbs (widths 33..256, limb 0 least significant)
//   N file: MW_NN slots x 1 u32       (widths 1..32; Bool = width 1, 0/1)
// (8 + 64: Mythril's queries are mostly narrow values - calldata bytes, Bools -
// and the two files together must leave the interpreter within 256 VGPRs)
// Every value is canonical: bits at and above its width are zero.
//
// Instruction = 4 u32 words:
//   w0: [7:0] opcode  [15:8] flags  [31:16] width
//   w1: [15:0] dst    [31:16] a
//   w2: [15:0] b      [31:16] c
//   w3: imm (32 bits)
// Operand fields (a, b, c): bit 15 set -> constant: bits[14:0] = word offset
// into the program's constant pool (8 words for a W operand, 1 for N);
// otherwise a slot index in the file the opcode names.
#pragma once
#include <stdint.h>

#define MW_NW 8
#define MW_NN 64
// scratch slots the interpreter's write-back targets when an op writes the
// other file or nothing (mw_interp.h); never allocated, rejected as operands
#define MW_W_RESERVED (MW_NW - 1)
#define MW_N_RESERVED 31   // in each 32-slot half: N slots 31 and 63
#define MW_KBIT 0x8000u
#define MW_LEAF_WORDS 8
#define MW_POOL_ENTRY_WORDS 9      // wide leaves (width >= 32): flags + 8 limbs
#define MW_POOL_NARROW_RANDOM 0x80000000u  // narrow leaves (width < 32): ONE word per entry,
                                           // bit 31 = RANDOM, bits 0..30 = the value
// words per pool entry of a width-w leaf
#define MW_POOL_ENTRY_WORDS_OF(w) ((w) < 32u ? 1u : (uint32_t)MW_POOL_ENTRY_WORDS)
#define MW_MAX_WIDTH 256

// leaf table entry (MW_LEAF_WORDS u32 per leaf)
#define MW_LEAF_WIDTH 0
#define MW_LEAF_KIND 1   // 0 random (Philox), 1 pool (index bit-field), 2 pool (hashed digit),
                         // 3 pool (bit-interleaved digit: bits SHIFT, SHIFT+STRIDE, ...)
#define MW_LEAF_ID 2     // Philox key salt
#define MW_LEAF_SHIFT 3  // candidate-index bit offset of the pool digit
#define MW_LEAF_BITS 4   // log2(pool entries)
#define MW_LEAF_POOL 5   // word offset of entry 0 in the pool buffer
#define MW_LEAF_INROW 6  // first SoA input row (mg_eval)
#define MW_LEAF_STRIDE 7 // kind 3: index-bit stride between consecutive digit bits
// pool entry, width >= 32: word 0 = flags (bit0: RANDOM), words 1..8 = limbs;
// width < 32: one word, MW_POOL_NARROW_RANDOM or the value (calldata bytes and
// Bools are most pool entries: 9x less LDS when pools are staged there)

enum mw_opcode {
  MW_END = 0,
  MW_CHECK = 1,    // alive &= N[a]
  MW_LEAF_W = 2,   // W[dst] = leaf imm
  MW_LEAF_N = 3,   // N[dst] = leaf imm
  MW_STORE_W = 4,  // trace rows imm..imm+7 = W/K a
  MW_STORE_N = 5,  // trace row imm = N/K a
  MW_SPILL_W = 6,  // spill W slot imm = W[a]
  MW_FILL_W = 7,   // W[dst] = spill W slot imm
  MW_MOV_W = 8,    // W[dst] = W/K a
  MW_MOV_N = 9,    // N[dst] = N/K a
  MW_SPILL_N = 10,
  MW_FILL_N = 11,
  MW_CHECK_IMP = 12,  // alive &= (N[a] == 0) | (N[b] != 0): a congruence conjunct a => b in one dispatch
  MW_CHECK_IMPEQ = 13,   // alive &= (N[a] == 0) | (N/K[b] == N/K[c])   (a => (b = c), narrow)
  MW_CHECK_IMPEQW = 14,  // alive &= (N[a] == 0) | (W/K[b] == W/K[c])   (a => (b = c), wide)
  MW_CHECK_IMPEQK = 15,  // alive &= (N[a] != imm) | (N/K[b] == N/K[c]) (a keyed congruence premise, lower._index_key)

  // wide: W[dst] = f(W/K a, W/K b) at `width`
  MW_W_ADD = 16, MW_W_SUB = 17, MW_W_MUL = 18, MW_W_AND = 19, MW_W_OR = 20,
  MW_W_XOR = 21, MW_W_NOT = 22,
  MW_W_SHL = 23, MW_W_LSHR = 24, MW_W_ASHR = 25,
  MW_W_UDIV = 26, MW_W_UREM = 27, MW_W_SDIV = 28, MW_W_SREM = 29, MW_W_SMOD = 30,
  MW_W_ITE = 31,   // W[dst] = N[c] ? a : b
  MW_W_SHLI = 32,  // W[dst] = a << imm  (imm < 256), masked to width
  MW_W_LSHRI = 33, // W[dst] = a >> imm, masked to width (extract)
  MW_W_ZEXTN = 34, // W[dst] = N/K a
  MW_W_SEXT = 35,  // W[dst] = sign-extend(a from imm bits) to width
  MW_W_SEXTN = 36, // W[dst] = sign-extend(N/K a from imm bits) to width
  MW_W_INSN = 37,  // W[dst] = a | (N/K b << imm)   (concat builder)
  MW_W_CDINS = 38, // W[dst] = W/K a | ((K[c] <s W[b] (256-bit) ? leaf(imm & 0xffff) : 0) << (imm >> 16)):
                   // one guarded calldata byte ite(i <s size, cd[i], 0) inserted into a word
                   // (state/calldata.py:218-231), four dispatches in one
  MW_CHECK_GRID = 39,  // j = imm - N[a]; alive &= j >= n | (spill word T0 + j == N/K[b]),
                       // c a raw field: T0 = c & 1023, n = (c >> 10 & 31) + 1 (a congruence grid's row,
                       // compiler.py _form_grids; the table's words are stored by SPILL_N)

  // wide -> narrow
  MW_N_EXTRACTW = 48, // N[dst] = (a >> imm) masked to width (<= 32)
  MW_N_ULT = 49, MW_N_ULE = 50, MW_N_SLT = 51, MW_N_SLE = 52, MW_N_EQ = 53, // width = operand width
  MW_N_UMULNO = 54,   // a*b < 2^width
  MW_N_ADDC = 55,     // carry out of a + b at width

  // narrow: N[dst] = f(N/K a, N/K b) at `width` (<= 32)
  MW_N_ADD = 64, MW_N_SUB = 65, MW_N_MUL = 66, MW_N_AND = 67, MW_N_OR = 68,
  MW_N_XOR = 69, MW_N_NOT = 70,
  MW_N_SHL = 71, MW_N_LSHR = 72, MW_N_ASHR = 73,
  MW_N_UDIV = 74, MW_N_UREM = 75, MW_N_SDIV = 76, MW_N_SREM = 77, MW_N_SMOD = 78,
  MW_N_ITE = 79,
  MW_N_SHLI = 80, MW_N_LSHRI = 81,
  MW_N_SEXT = 82,     // sign-extend a from imm bits to width
  MW_N_ULTN = 83, MW_N_ULEN = 84, MW_N_SLTN = 85, MW_N_SLEN = 86, MW_N_EQN = 87,
  MW_N_UMULNON = 88,
  MW_N_ADDCN = 89,
};

// mg_search flags
#define MW_FLAG_EARLY_EXIT 1u   // per-wave ballot exit after a failing CHECK
#define MW_FLAG_STOP_AFTER_HIT 2u  // blocks stop once a lower witness is known
// specialised kernels skip the launch counters (evals, division paths): a
// timed exhaustive launch writes nothing but its witness minimum; the host
// reports evals = count per program.  Ignored with STOP_AFTER_HIT.
#define MW_FLAG_NO_COUNT 4u
