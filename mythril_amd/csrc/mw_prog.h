// mw_prog.h — bytecode format details used by the interpreter and the
// validator only (the specialised kernels are generated from the compiler's
// SSA and never read them; keeping them out of mw_isa.h keeps the specialised
// kernels' cache keys stable).  Mirrored in mythril_amd/isa.py.
#pragma once

// instruction flags (w0 bits [15:8])
#define MW_FLAG_CHAIN 1u   // W_CDINS: the next instruction is a W_CDINS whose acc operand is this
                           // result, its only use (the interpreter keeps it in registers)

// dst field (w1 bits [15:0]): the write targets of the interpreter's single
// write-back, resolved by the compiler.  Every dispatch writes r into W slot
// [2:0], r[0] into N slot [7:3] of the low half and into N slot [12:8] of the
// high half; a file the op does not write gets its scratch slot (MW_W_RESERVED,
// MW_N_RESERVED), so the interpreter needs no per-op "what do I write" logic.
#define MW_DST_W(d) ((d) & 7u)
#define MW_DST_NLO(d) (((d) >> 3) & 31u)
#define MW_DST_NHI(d) (((d) >> 8) & 31u)
#define MW_DST_SCRATCH (MW_W_RESERVED | (MW_N_RESERVED << 3) | (MW_N_RESERVED << 8))

// asm interpreter: narrow constants live in MW_ASM_NK VGPRs starting
// MW_ASM_NK_INDEX registers above the N file's base (v64 + 176 = v240), filled
// once per block (mw_validate.cpp mw_asm_predecode, mythril_amd/asmgen.py NK0)
#define MW_ASM_NK 16u
#define MW_ASM_NK_INDEX 176u
