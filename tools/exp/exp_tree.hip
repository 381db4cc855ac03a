// Experiment: minimal-structure interpreter (register-only W operands) to bound
// what the C++ dispatch can reach.  Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../mythril_amd/csrc/mw_alu.h"
using namespace mw;
typedef const __attribute__((address_space(4))) u32* kptr;
typedef u32 u32x16 __attribute__((ext_vector_type(16)));
enum { E_END = 0, E_ADD = 1, E_XOR = 2, E_SUB = 3, E_AND = 4, E_INIT = 5 };
#define FW(o, x) do { u32 _o = (o) & 15u; x[0]=F0[_o];x[1]=F1[_o];x[2]=F2[_o];x[3]=F3[_o];x[4]=F4[_o];x[5]=F5[_o];x[6]=F6[_o];x[7]=F7[_o]; } while (0)
#define WW(o, x) do { u32 _o = (o) & 15u; F0[_o]=x[0];F1[_o]=x[1];F2[_o]=x[2];F3[_o]=x[3];F4[_o]=x[4];F5[_o]=x[5];F6[_o]=x[6];F7[_o]=x[7]; } while (0)
extern "C" __global__ __launch_bounds__(256, 2) void exp_kernel(const u32* code_, u64 n, u32* out) {
  kptr code = (kptr)code_;
  for (u64 cand = (u64)blockIdx.x * 256 + threadIdx.x; cand < n; cand += (u64)gridDim.x * 256) {
    u32x16 F0 = 0, F1 = 0, F2 = 0, F3 = 0, F4 = 0, F5 = 0, F6 = 0, F7 = 0;
    u32 w0 = code[0], w1 = code[1];
    for (u32 pc = 2;; pc += 2) {
      const u32 op = w0 & 0xff, d = (w0 >> 8) & 0xff, a = (w0 >> 16) & 0xff, b = w0 >> 24;
      if (op == E_END) break;
      asm volatile("" ::: "memory");
      const u32 n0 = code[pc], n1 = code[pc + 1];
      u32 x[8], y[8], r[8];
      FW(a, x);
      FW(b, y);
      if (op < 3) {
        if (op == E_ADD) { add8(x, y, r); }
        else { for (int k = 0; k < 8; ++k) r[k] = x[k] ^ y[k]; }
      } else {
        if (op == E_SUB) { sub8(x, y, r); }
        else if (op == E_AND) { for (int k = 0; k < 8; ++k) r[k] = x[k] & y[k]; }
        else { for (int k = 0; k < 8; ++k) r[k] = (u32)cand * (k + w1); }
      }
      WW(d, r);
      w0 = n0; w1 = n1;
    }
    u32 x[8];
    FW(0, x);
    out[cand] = x[0] ^ x[7];
  }
}
