// Probe: which bits of the SGPR operand of s_set_gpr_idx_on index the VGPRs
// on gfx950?  The asm interpreter could skip a field extraction per operand
// if only bits [7:0] count (ISA: M0[7:0] = S0[7:0]).  The index register
// holds 3 plus junk above bit 7; v10..v20 hold 100..110, so the read value is
// 103 when only the low byte is used.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* out, unsigned junk) {
  unsigned r;
  asm volatile(
      "v_mov_b32 v10, 100\n v_mov_b32 v11, 101\n v_mov_b32 v12, 102\n v_mov_b32 v13, 103\n"
      "v_mov_b32 v14, 104\n v_mov_b32 v15, 105\n v_mov_b32 v16, 106\n v_mov_b32 v17, 107\n"
      "v_mov_b32 v18, 108\n v_mov_b32 v19, 109\n v_mov_b32 v20, 110\n"
      "s_or_b32 s20, %1, 3\n"
      "s_set_gpr_idx_on s20, gpr_idx(SRC0)\n"
      "v_mov_b32 %0, v10\n"
      "s_set_gpr_idx_off\n"
      : "=v"(r)
      : "s"(junk)
      : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "s20", "m0");
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}

int main() {
  const unsigned junks[] = {0x0u, 0x100u, 0x8000u, 0xff00u, 0x12340000u, 0xffffff00u};
  unsigned* d;
  hipMalloc(&d, 64 * sizeof(unsigned));
  int ok = 1;
  for (unsigned j : junks) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, j);
    unsigned h = 0;
    hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("index register 0x%08x -> read %u (%s)\n", j | 3u, h, h == 103u ? "low byte only" : "OTHER");
    ok &= h == 103u;
  }
  hipFree(d);
  printf("%s\n", ok ? "s_set_gpr_idx_on uses S0[7:0]" : "s_set_gpr_idx_on uses more than S0[7:0]");
  return 0;
}
