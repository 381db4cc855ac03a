// Probe: what a bytecode dispatch of the asm interpreter costs on gfx950,
// piece by piece.  Each kernel runs one instruction sequence 8x per loop
// iteration, 256 iterations, and lane 0 of every wave reports its clock64()
// cycles per sequence.  Launched with 1 wave (latency) and with 8 waves per
// CU (two per SIMD, the interpreter's occupancy).
//
//   nop      s_nop 0 x 3                           (SALU issue floor)
//   vmov     v_mov x 3                             (VALU issue floor)
//   idx      set_gpr_idx_on / v_mov / off          (one indexed operand read)
//   nadd     N_ADD's body as generated (fetch a, fetch b, add, and, write)
//   nfold    the same with the add reading a through the index and the
//            and writing through it (two v_movs fewer)
//   jmpcalc  and / lshl2_add / addc                (handler address)
//   setpc    getpc / add / addc / setpc to the next instruction (a jump)
//   smem     s_load_dwordx4 + s_waitcnt            (code fetch latency)
//   disp     the full dispatch: wait, 2 movs, add, load, and, lshl2_add,
//            addc, setpc (one-ahead prefetch, as the interpreter)
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

#define KERNEL(NAME, BODY, CLOB)                                                          \
  __global__ void NAME(unsigned long long* out, const unsigned* code) {                   \
    unsigned long long t0 = clock64();                                                    \
    for (int it = 0; it < 256; ++it) {                                                    \
      asm volatile("s_mov_b64 s[32:33], %0\n s_mov_b32 s41, 3\n s_mov_b32 s42, 5\n"       \
                   "s_mov_b32 s43, 0xffff\n s_mov_b32 s48, 0\n" REP8(BODY)                  \
                   :                                                                      \
                   : "s"(code)                                                            \
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v30", "v31", \
                     "v32", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s32", \
                     "s33", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", \
                     "s92", "s94", "s95", "m0", "scc", "memory" CLOB);                   \
    }                                                                                     \
    unsigned long long t1 = clock64();                                                    \
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = (t1 - t0);    \
  }

KERNEL(k_nop, "s_nop 0\n s_nop 0\n s_nop 0\n", )
KERNEL(k_vmov, "v_mov_b32 v30, v10\n v_mov_b32 v31, v11\n v_mov_b32 v32, v12\n", )
KERNEL(k_idx, "s_set_gpr_idx_on s41, gpr_idx(SRC0)\n v_mov_b32 v30, v10\n s_set_gpr_idx_off\n", )
KERNEL(k_nadd,
       "s_set_gpr_idx_on s41, gpr_idx(SRC0)\n v_mov_b32 v30, v10\n s_set_gpr_idx_off\n"
       "s_set_gpr_idx_on s42, gpr_idx(SRC0)\n v_mov_b32 v31, v10\n s_set_gpr_idx_off\n"
       "v_add_u32 v32, v30, v31\n v_and_b32 v32, s43, v32\n s_lshr_b32 s19, s41, 16\n"
       "s_set_gpr_idx_on s19, gpr_idx(DST)\n v_mov_b32 v10, v32\n s_set_gpr_idx_off\n", )
KERNEL(k_nfold,
       "s_set_gpr_idx_on s42, gpr_idx(SRC0)\n v_mov_b32 v31, v10\n s_set_gpr_idx_off\n"
       "s_set_gpr_idx_on s41, gpr_idx(SRC0)\n v_add_u32 v32, v10, v31\n s_set_gpr_idx_off\n"
       "s_lshr_b32 s19, s41, 16\n"
       "s_set_gpr_idx_on s19, gpr_idx(DST)\n v_and_b32 v10, s43, v32\n s_set_gpr_idx_off\n", )
KERNEL(k_jmpcalc, "s_and_b32 s92, s40, 0x7fff\n s_lshl2_add_u32 s94, s92, s41\n s_addc_u32 s95, s42, 0\n", )
KERNEL(k_setpc, "s_getpc_b64 s[94:95]\n s_add_u32 s94, s94, 12\n s_addc_u32 s95, s95, 0\n s_setpc_b64 s[94:95]\n", )
KERNEL(k_smem, "s_load_dwordx4 s[44:47], s[32:33], s48\n s_waitcnt lgkmcnt(0)\n", )
KERNEL(k_disp,
       "s_waitcnt lgkmcnt(0)\n s_mov_b64 s[40:41], s[44:45]\n s_mov_b64 s[42:43], s[46:47]\n"
       "s_add_u32 s48, s48, 16\n s_load_dwordx4 s[44:47], s[32:33], s48\n"
       "s_getpc_b64 s[94:95]\n s_add_u32 s94, s94, 20\n s_addc_u32 s95, s95, 0\n"
       "s_and_b32 s92, s40, 0x7fff\n s_setpc_b64 s[94:95]\n", )

typedef void (*kfn)(unsigned long long*, const unsigned*);

int main() {
  struct {
    const char* name;
    kfn f;
  } ks[] = {{"nop x3", k_nop},   {"vmov x3", k_vmov},       {"idx", k_idx},     {"nadd", k_nadd},
            {"nfold", k_nfold},  {"jmpcalc", k_jmpcalc}, {"setpc", k_setpc}, {"smem", k_smem},
            {"disp", k_disp}};
  unsigned long long* d;
  unsigned* code;
  hipMalloc(&d, 1024 * 16 * sizeof(unsigned long long));
  hipMalloc(&code, 1 << 20);
  hipMemset(code, 0, 1 << 20);
  for (int waves : {1, 8}) {
    for (auto& k : ks) {
      hipMemset(d, 0, 1024 * 16 * sizeof(unsigned long long));
      // 1 wave: one block of 64; 8 waves per CU: 256 blocks of 512 threads
      const int blocks = waves == 1 ? 1 : 256, threads = waves == 1 ? 64 : 512;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, code);   // warm
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, code);
      hipDeviceSynchronize();
      unsigned long long h[16];
      hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      double s = 0;
      int n = waves == 1 ? 1 : threads / 64;
      for (int i = 0; i < n; ++i) s += (double)h[i];
      printf("%-8s waves/CU %d: %7.1f cycles per sequence\n", k.name, waves, s / n / (256.0 * 8));
    }
  }
  hipFree(d);
  hipFree(code);
  return 0;
}
