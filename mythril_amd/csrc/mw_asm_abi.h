// mw_asm_abi.h — launch records and kernel body shared by the two asm engines:
// the threaded-dispatch interpreter (mw_kernels.hip mw_search_asm_kernel) and
// the assembled kernels (mw_asmjit_shell.hip, instantiated per program by
// mythril_amd/asmjit.py).  The asm text reads both records at fixed offsets
// (mythril_amd/asmgen.py gen(): "AsmArgs: ..." and "ProgDev: ...").
#pragma once
#include "mw_alu.h"

namespace mw {

struct ProgDev {
  const u32* code;     // the asm interpreter reads its predecoded copy here
  const u32* consts;
  const u32* leaves;
  const u32* pool;
  u32 n_spill;
  u32 npool;   // pool words (staged in LDS)
  u32 n_insn;
  u32 first_block;   // a 1D launch over several programs (AsmArgs.nprog): this program's first block
};

struct AsmArgs {
  u64 seed, begin, end;
  u32 flags, nlds, gstride, nchunks, gdx;
  u32 nprog;      // 0: grid y is the program, grid x its blocks (gdx of them); else a 1D grid whose
                  // blocks the nprog programs share, ProgDev.first_block each (mw_kernels.hip)
  u32* spillbuf;
  u32* verdict;   // per-candidate verdicts at cand - begin (mg_eval_generated), or null
  u32* trace;     // trace rows, row r of candidate cand at r * ncand + cand - begin (STORE_W / STORE_N), or null
  u32 ncand, pad2;
};
static_assert(sizeof(AsmArgs) == 80, "AsmArgs layout (mythril_amd/asmgen.py)");
static_assert(sizeof(ProgDev) == 48, "ProgDev layout (mythril_amd/asmgen.py)");

}  // namespace mw

// Kernel body: stage the program's pool in LDS after the spill words (LDS: the
// dynamic shared array), run ASMTEXT over this block's chunks (grid x: chunk
// stride, grid y: program; or, with AsmArgs.nprog, a 1D grid split between
// the programs by ProgDev.first_block: blocks in proportion to each program's
// cost, so the launch ends with its slowest program's last chunk, not with a
// tail of expensive rows), add the evals to the launch counter (stripe 0).
#define MW_ASM_KERNEL_BODY(ASMTEXT, LDS) MW_ASM_KERNEL_BODY_C(ASMTEXT, LDS, MW_ASM_CLOBBERS)
// CLOB: the asm block's clobbers (the interpreter's wide or narrow register layout)
#define MW_ASM_KERNEL_BODY_C(ASMTEXT, LDS, CLOB)                                                     \
  mw::u32 prow = blockIdx.y, ch0 = blockIdx.x, gdxp = args->gdx;                                     \
  if (const mw::u32 np_ = args->nprog) {                                                             \
    mw::u32 lo = 0, hi = np_;                                                                        \
    while (hi - lo > 1u) {                                                                           \
      const mw::u32 mid = (lo + hi) >> 1;                                                            \
      if (progs[mid].first_block <= blockIdx.x) lo = mid; else hi = mid;                             \
    }                                                                                                \
    prow = lo;                                                                                       \
    ch0 = blockIdx.x - progs[lo].first_block;                                                        \
    gdxp = (lo + 1u < np_ ? progs[lo + 1u].first_block : gridDim.x) - progs[lo].first_block;         \
  }                                                                                                  \
  const mw::ProgDev* P = progs + prow;                                                               \
  {                                                                                                  \
    mw::u32* dst = LDS + nlds * 256u;                                                                \
    const mw::u32 np = P->npool;                                                                     \
    const mw::u32* src = P->pool;                                                                    \
    for (mw::u32 i = threadIdx.x; i < np; i += 256u) dst[i] = src[i];                                \
    __syncthreads();                                                                                 \
  }                                                                                                  \
  const mw::u64 gtid = ((mw::u64)blockIdx.y * gridDim.x + blockIdx.x) * 256u + threadIdx.x;         \
  const mw::u32 goff = (mw::u32)(gtid * 4u);                                                         \
  const mw::u32 tid = threadIdx.x;                                                                   \
  mw::u64* om = out_min + prow;                                                                      \
  mw::u64 evals;                                                                                     \
  asm volatile(ASMTEXT                                                                               \
               : [evals] "=s"(evals)                                                                 \
               : [args] "s"(args), [prog] "s"(P), [outmin] "s"(om), [ch0] "s"(ch0), [gdx] "s"(gdxp),  \
                 [tid] "v"(tid), [goff] "v"(goff)                                                    \
               : CLOB);                                                                              \
  if ((threadIdx.x & 63u) == 0 && evals) atomicAdd((unsigned long long*)counter, (unsigned long long)evals);
