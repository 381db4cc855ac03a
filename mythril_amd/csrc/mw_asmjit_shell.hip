// mw_asmjit_shell.hip — the template of the assembled kernels.  Compiled once to
// gfx950 assembly by mythril_amd/build.py (hipcc --cuda-device-only -S ->
// build/asmjit/template.s); mythril_amd/asmjit.py replaces the marker line of
// MW_ASMJIT_TEMPLATE_BODY with a program's straight-line body
// (mythril_amd/asmgen.py static_body), renames the kernel and its signature
// word, and assembles the result with llvm-mc + ld.lld.  Launched like the
// asm interpreter (same records, same grid), one program per launch.
#include <hip/hip_runtime.h>

#include "mw_asm_abi.h"
#include "mw_asm_interp.inc"

// the whole 80 KiB spill-and-pool area (mg_search's asm_lds_fit keeps within it):
// two blocks per CU, as the asm interpreter
__shared__ mw::u32 mwa_lds[80 * 256];

extern "C" __global__ __launch_bounds__(256, 2) void mwa_TEMPLATE(const mw::ProgDev* __restrict__ progs,
                                                                  const mw::AsmArgs* __restrict__ args,
                                                                  mw::u64* __restrict__ out_min,
                                                                  mw::u64* __restrict__ counter, mw::u32 nlds) {
  MW_ASM_KERNEL_BODY(MW_ASMJIT_TEMPLATE_BODY, mwa_lds)
}

// FNV-1a 64 of the program (mg_prog_attach_asm checks it): a placeholder here
extern "C" __device__ const mw::u64 mwa_TEMPLATE_sig = 0x0123456789ABCDEFull;
