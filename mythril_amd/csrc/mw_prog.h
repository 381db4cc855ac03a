// mw_prog.h — bytecode format details used by the interpreter and the
// validator only (the specialised kernels are generated from the compiler's
// SSA and never read them; keeping them out of mw_isa.h keeps the specialised
// kernels' cache keys stable).  Mirrored in mythril_amd/isa.py.
#pragma once

// instruction flags (w0 bits [15:8])
#define MW_FLAG_CHAIN 1u   // W_CDINS: the next instruction is a W_CDINS whose acc operand is this
                           // result, its only use (the interpreter keeps it in registers)
