// mw_kernels.hip — gfx950 kernels and the C-ABI (include/mythril_witness.h).
//
// Kernels
//   mw_search_kernel  grid (x: candidate chunks, y: programs), 256-thread blocks,
//                     one candidate per lane; per-wave ballot -> lowest satisfying
//                     lane -> atomicMin(u64) on the program's witness index.
//   mw_eval_kernel    same interpreter on explicit (SoA) or generated assignments,
//                     writing per-candidate verdicts and traced node values.
//   mw_keccak_kernel  one message per lane, Keccak-256.
// Host side: context (device, stream, events, spill/min/counter buffers),
// program upload with full validation, thread-local error strings.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mythril_witness.h"
#include "mw_asm_abi.h"
#include "mw_asm_interp.inc"
#include "mw_handles.h"
#include "mw_inflight.h"
#include "mw_interp.h"
#include "mw_keccak.h"
#include "mw_leaf.h"

extern "C" int mw_fail(int code, const char* msg);
extern "C" int mg_validate_desc(const mg_prog_desc* d);
extern "C" int mw_asm_predecode(const uint32_t* code, size_t nwords, const uint32_t* consts, size_t nconst,
                                const uint32_t* hoff, uint32_t* out, uint32_t* nk);
extern "C" int mw_asm_predecode_layout(const uint32_t* code, size_t nwords, const uint32_t* consts, size_t nconst,
                                       const uint32_t* hoff, uint32_t* out, uint32_t* nk, uint32_t nk_index,
                                       uint32_t nk_max, uint32_t nfile, uint32_t wfile);

using namespace mw;

namespace {

constexpr int kBlock = 256;
constexpr int kNCounters = 5;  // counter words: evals, then DivCount fields x lanes
// d_counter: stripe 0 (interpreters) + MW_CTR_STRIPES stripes (specialised kernels), summed on readback
constexpr size_t kCounterWords = (size_t)(1 + MW_CTR_STRIPES) * MW_CTR_STRIPE_WORDS;
// Spill area: n_spill words per lane (a W spill slot is 8 consecutive words, an
// N slot one; the compiler puts the most-used words first).  Words
// [0, kLdsSpillWords) live in LDS as [word][lane] (consecutive lanes ->
// consecutive banks): 80 words = 80 KiB per 256-lane block, so two blocks (8
// waves) still fit a CU's 160 KiB; the rest in the global spill buffer,
// [word][thread].
constexpr u32 kLdsSpillWords = 80;
extern __shared__ u32 lds_spill[];

typedef const __attribute__((address_space(3))) u32* lptr;

// leaf_value (mw_leaf.h) with the pool staged in LDS: the per-lane pool gather
// is a ds_read (~100 cycles) instead of a global load (~2 000): a leaf cost
// ~2 800 cycles per wave with the pool in HBM (tools/c3_ablate.py).
__device__ __forceinline__ void leaf_value_lds(const u32* __restrict__ leaf_, lptr pool, u64 seed, u64 cand,
                                               u32 out[8]) {
  const __attribute__((address_space(4))) u32* leaf = (const __attribute__((address_space(4))) u32*)leaf_;
  const u32 w = leaf[MW_LEAF_WIDTH], id = leaf[MW_LEAF_ID];
#if defined(MW_ABLATE_LEAF)
  out[0] = (u32)cand ^ id;
#pragma unroll
  for (int k = 1; k < 8; ++k) out[k] = 0u;
  canon(out, w);
  return;
#endif
#if defined(MW_ABLATE_DIGIT)
  const u32 kind = leaf[MW_LEAF_KIND] == 3u ? 1u : leaf[MW_LEAF_KIND];
#else
  const u32 kind = leaf[MW_LEAF_KIND];
#endif
  if (kind >= 1u && kind <= 3u) {
    const u32 bits = leaf[MW_LEAF_BITS];
    u32 digit;
    if (kind == 3u) {
      const u32 sh = leaf[MW_LEAF_SHIFT], st = leaf[MW_LEAF_STRIDE];
      digit = 0;
      for (u32 b = 0; b < bits; ++b) digit |= (u32)((cand >> (sh + b * st)) & 1u) << b;
    } else {
      const u64 src = kind == 1u ? (cand >> leaf[MW_LEAF_SHIFT]) : fmix64(cand ^ ((u64)id * 0x9E3779B97F4A7C15ull));
      digit = (u32)src & ((bits >= 32) ? 0xffffffffu : ((1u << bits) - 1u));
    }
    lptr e = pool + leaf[MW_LEAF_POOL] + digit * MW_POOL_ENTRY_WORDS_OF(w);
    if (w < 32u) {  // one-word narrow entry
      const u32 x = e[0];
      if (x & MW_POOL_NARROW_RANDOM) {
        random_leaf(id, w, seed, cand, out);
      } else {
        out[0] = x;
#pragma unroll
        for (int k = 1; k < 8; ++k) out[k] = 0u;
      }
    } else if (e[0] & 1u) {
      random_leaf(id, w, seed, cand, out);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = e[1 + k];
      canon(out, w);
    }
  } else {
    random_leaf(id, w, seed, cand, out);
  }
}

template <bool POOL_LDS>
struct SearchEnv {
  const u32* __restrict__ leaves;
  const u32* __restrict__ pool;
  u64 seed;
  u64 cand;
  u32* __restrict__ spillbuf;
  u64 nthreads;
  u64 gtid;
  __device__ void leaf(u32 idx, u32 out[8]) {
    if (POOL_LDS)
      leaf_value_lds(leaves + (u64)idx * MW_LEAF_WORDS, (lptr)(lds_spill + nlds * kBlock), seed, cand, out);
    else
      leaf_value(leaves + (u64)idx * MW_LEAF_WORDS, pool, seed, cand, out);
  }
  __device__ void store(u32, const u32*, int) {}
  u32 nlds;  // spill words [0, nlds) live in LDS, the rest in the global spill buffer
  __device__ void spill(u32 off, const u32* v, int n) {
    for (int k = 0; k < n; ++k) {
      const u32 wd = off + (u32)k;   // uniform
      if (wd < nlds) lds_spill[wd * kBlock + threadIdx.x] = v[k];
      else spillbuf[(u64)(wd - nlds) * nthreads + gtid] = v[k];
    }
  }
  __device__ void fill(u32 off, u32* v, int n) {
    for (int k = 0; k < 8; ++k) {
      const u32 wd = off + (u32)k;
      v[k] = k >= n ? 0u : wd < nlds ? lds_spill[wd * kBlock + threadIdx.x] : spillbuf[(u64)(wd - nlds) * nthreads + gtid];
    }
  }
  __device__ bool none(bool alive) { return __ballot(alive) == 0ull; }
  DivCount dsteps;  // division paths this wave took (wave-uniform)
};

struct EvalEnv {
  const u32* __restrict__ leaves;
  const u32* __restrict__ pool;
  const u32* __restrict__ in;  // SoA rows, or null -> generated
  u32* __restrict__ trace;
  u64 ncand;
  u64 idx;   // candidate position within this call
  u64 seed;
  u64 cand;  // generated candidate index
  u32* __restrict__ spillbuf;
  u64 nthreads;
  u64 gtid;
  __device__ void leaf(u32 li, u32 out[8]) {
    const u32* L = leaves + (u64)li * MW_LEAF_WORDS;
    if (in) {
      const u32 w = L[MW_LEAF_WIDTH];
      const u32 row = L[MW_LEAF_INROW];
      const int nl = (int)((w + 31) / 32);
      for (int k = 0; k < 8; ++k) out[k] = k < nl ? in[((u64)row + k) * ncand + idx] : 0u;
      canon(out, w);
    } else {
      leaf_value(L, pool, seed, cand, out);
    }
  }
  __device__ void store(u32 row, const u32* v, int n) {
    if (trace)
      for (int k = 0; k < n; ++k) trace[((u64)row + k) * ncand + idx] = v[k];
  }
  u32 nlds;  // spill words [0, nlds) live in LDS, the rest in the global spill buffer
  __device__ void spill(u32 off, const u32* v, int n) {
    for (int k = 0; k < n; ++k) {
      const u32 wd = off + (u32)k;   // uniform
      if (wd < nlds) lds_spill[wd * kBlock + threadIdx.x] = v[k];
      else spillbuf[(u64)(wd - nlds) * nthreads + gtid] = v[k];
    }
  }
  __device__ void fill(u32 off, u32* v, int n) {
    for (int k = 0; k < 8; ++k) {
      const u32 wd = off + (u32)k;
      v[k] = k >= n ? 0u : wd < nlds ? lds_spill[wd * kBlock + threadIdx.x] : spillbuf[(u64)(wd - nlds) * nthreads + gtid];
    }
  }
  __device__ bool none(bool) { return false; }  // eval: never exit early
  DivCount dsteps;
};

}  // namespace

// POOL_LDS: the program's pool is copied into LDS after the spill words once
// per block (the launch sizes LDS for the largest pool of the launch).
template <bool POOL_LDS>
__global__ __launch_bounds__(kBlock, 2) void mw_search_kernel(const ProgDev* __restrict__ progs, u64 seed,
                                                           u64 begin, u64 count, u32 flags,
                                                           u64* __restrict__ out_min,
                                                           u64* __restrict__ counter,
                                                           u32* __restrict__ spillbuf, u32 nlds) {
  const ProgDev P = progs[blockIdx.y];
  if (POOL_LDS) {
    u32* dst = lds_spill + nlds * kBlock;
    for (u32 i = threadIdx.x; i < P.npool; i += kBlock) dst[i] = P.pool[i];
    __syncthreads();
  }
  const u64 nchunks = (count + kBlock - 1) / kBlock;
  const u64 end = begin + count;
  const u64 nthreads = (u64)gridDim.x * gridDim.y * kBlock;
  const u64 gtid = ((u64)blockIdx.y * gridDim.x + blockIdx.x) * kBlock + threadIdx.x;
  const u32 lane = threadIdx.x & 63u;
  u64 evals = 0, lsteps = 0, lfull = 0, lshort = 0, lgen = 0;   // division paths x lanes
  bool reported = false;   // this wave's later chunks hold only larger indices
  u32 iter = 0;
  for (u64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const u64 base = begin + ch * kBlock;
    // every 16th chunk of the block, not its first: every block reading the
    // one witness word at every chunk queues them all at one memory channel
    // (the asm interpreter's poll, mythril_amd/asmgen.py POLL_EVERY)
    if ((flags & MW_FLAG_STOP_AFTER_HIT) && (++iter & 15u) == 0u) {
      u64 m = __hip_atomic_load(&out_min[blockIdx.y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (m <= base) break;
    }
    const u64 cand = base + threadIdx.x;
    const bool valid = cand < end;
    SearchEnv<POOL_LDS> env{P.leaves, P.pool, seed, cand, spillbuf, nthreads, gtid, nlds};
    const bool ok = mw_run(P.code, P.consts, env, valid, flags);
    const u64 hit = __ballot(ok);
    if (hit && !reported) {
      const u32 first = (u32)__ffsll((unsigned long long)hit) - 1u;
      if (lane == first && cand < __hip_atomic_load(&out_min[blockIdx.y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin((unsigned long long*)&out_min[blockIdx.y], (unsigned long long)cand);
      reported = true;
    }
    const u64 nvalid = (u64)__popcll(__ballot(valid));
    evals += nvalid;
    lsteps += nvalid * env.dsteps.steps;
    lfull += nvalid * env.dsteps.full;
    lshort += nvalid * env.dsteps.shrt;
    lgen += nvalid * env.dsteps.gen;
  }
  if (lane == 0 && evals) {
    atomicAdd((unsigned long long*)counter, (unsigned long long)evals);
    if (lsteps) atomicAdd((unsigned long long*)(counter + 1), (unsigned long long)lsteps);
    if (lfull) atomicAdd((unsigned long long*)(counter + 2), (unsigned long long)lfull);
    if (lshort) atomicAdd((unsigned long long*)(counter + 3), (unsigned long long)lshort);
    if (lgen) atomicAdd((unsigned long long*)(counter + 4), (unsigned long long)lgen);
  }
}

// Threaded-dispatch interpreter (mythril_amd/asmgen.py -> mw_asm_interp.inc):
// the same result protocol as mw_search_kernel, for programs whose opcodes and
// leaf kinds all have an asm handler and whose pools are staged in LDS
// (mg_prog.asm_ok, checked on load; the launch checks the LDS fit).  The asm
// block runs the whole chunk loop of the block (one copy of the code: a loop
// around it gets unswitched into several copies) and reads its launch
// arguments from an AsmArgs record in device memory (mw_asm_abi.h).
__global__ __launch_bounds__(kBlock, 2) void mw_search_asm_kernel(const ProgDev* __restrict__ progs,
                                                                const AsmArgs* __restrict__ args,
                                                                u64* __restrict__ out_min,
                                                                u64* __restrict__ counter, u32 nlds) {
  MW_ASM_KERNEL_BODY_C(MW_ASM_BODY, lds_spill, MW_ASM_CLOBBERS)
}

// The same interpreter in the narrow register layout (round 5, asmgen.py
// variant("narrow")): a 24-slot N file, 166 VGPRs in the asm block, three
// waves per SIMD where the wide kernel's 256 allow two.  Programs whose N
// registers all lie below MW_ASM_NFILE_N are predecoded for it at load
// (Prog::asm_narrow); its launches keep the block's LDS within
// kLdsSpillWordsN KiB so that three blocks share a CU.
__global__ __launch_bounds__(kBlock, 3) void mw_search_asm_kernel_n(const ProgDev* __restrict__ progs,
                                                                  const AsmArgs* __restrict__ args,
                                                                  u64* __restrict__ out_min,
                                                                  u64* __restrict__ counter, u32 nlds) {
  MW_ASM_KERNEL_BODY_C(MW_ASM_BODY_N, lds_spill, MW_ASM_CLOBBERS_N)
}

// The quarter layout (asmgen.py variant("quarter")): 4 W slots and 16 N
// slots, 126 VGPRs in the asm block, four waves per SIMD, for programs whose
// W and N registers all lie in those files; LDS within kLdsSpillWordsQ KiB
// per block so that four blocks share a CU.
__global__ __launch_bounds__(kBlock, 4) void mw_search_asm_kernel_q(const ProgDev* __restrict__ progs,
                                                                  const AsmArgs* __restrict__ args,
                                                                  u64* __restrict__ out_min,
                                                                  u64* __restrict__ counter, u32 nlds) {
  MW_ASM_KERNEL_BODY_C(MW_ASM_BODY_Q, lds_spill, MW_ASM_CLOBBERS_Q)
}

// the asm interpreter's kernels by register layout (Prog::asm_layout)
typedef uint8_t u8;
enum AsmLayout : u8 { kWide = 0, kNarrow = 1, kQuarter = 2, kAsmLayouts = 3 };
typedef void (*AsmKernel)(const ProgDev*, const AsmArgs*, u64*, u64*, u32);
const AsmKernel kAsmKernel[kAsmLayouts] = {mw_search_asm_kernel, mw_search_asm_kernel_n, mw_search_asm_kernel_q};

__global__ __launch_bounds__(kBlock, 2) void mw_eval_kernel(ProgDev P, const u32* __restrict__ in,
                                                         u64 ncand, u64 seed, u64 begin,
                                                         u32* __restrict__ verdict,
                                                         u32* __restrict__ trace,
                                                         u32* __restrict__ spillbuf, u32 nlds) {
  const u64 nthreads = (u64)gridDim.x * kBlock;
  const u64 gtid = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u64 nchunks = (ncand + kBlock - 1) / kBlock;
  for (u64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const u64 idx = ch * kBlock + threadIdx.x;
    const bool valid = idx < ncand;
    EvalEnv env{P.leaves, P.pool, in, valid ? trace : nullptr, ncand, valid ? idx : 0,
                seed, begin + idx, spillbuf, nthreads, gtid, nlds};
    const bool ok = mw_run(P.code, P.consts, env, valid, 0u);
    if (valid) verdict[idx] = ok ? 1u : 0u;
  }
}

// The leaf values of one candidate: one thread per leaf, the candidate
// generator of every search engine (mw_leaf.h leaf_value), for mg_witness_leaves.
// The witness evaluations of mg_search_end read the candidate index the
// search found, on the device: record k evaluates index dmin[slot[k]] (0 when
// that search found nothing; the host ignores that trace).
__global__ __launch_bounds__(kBlock) void mw_witness_index_kernel(const u64* __restrict__ dmin,
                                                                   const u32* __restrict__ slot, AsmArgs* args,
                                                                   u32 n) {
  const u32 k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  u64 m = dmin[slot[k]];
  if (m == MG_NONE) m = 0;
  args[k].begin = m;
  args[k].end = m + 1;
}

__global__ __launch_bounds__(kBlock) void mw_leaf_kernel(const u32* __restrict__ leaves, const u32* __restrict__ pool,
                                                         u32 nleaves, u64 seed, u64 cand, u32* __restrict__ out) {
  const u32 l = blockIdx.x * kBlock + threadIdx.x;
  if (l >= nleaves) return;
  u32 v[8];
  leaf_value(leaves + (u64)l * MW_LEAF_WORDS, pool, seed, cand, v);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[(u64)l * 8 + k] = v[k];
}

__global__ __launch_bounds__(kBlock) void mw_keccak_kernel(const uint8_t* __restrict__ data,
                                                           const u64* __restrict__ off,
                                                           const u32* __restrict__ len, u64 n,
                                                           uint8_t* __restrict__ out) {
  for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
    u64 h[4];
    keccak256_msg(data + off[i], len[i], h);
    u64* o = (u64*)(out + 32 * i);
    o[0] = h[0];
    o[1] = h[1];
    o[2] = h[2];
    o[3] = h[3];
  }
}

// INT32 VALU peak microbenchmark: 8 independent v_add_u32 chains per lane
// (or v_mul_lo_u32 when mul != 0), all CUs, 8 waves per SIMD.
__global__ __launch_bounds__(kBlock) void mw_valu_peak_kernel(u32* __restrict__ out, u32 iters, u32 mul) {
  u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
      a7 = a0 + 7;
  const u32 b = blockIdx.x | 1u;
  if (mul) {
    for (u32 i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a1) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a2) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a3) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a4) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a5) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a6) : "v"(b));
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a7) : "v"(b));
      }
    }
  } else {
    for (u32 i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(b));
      }
    }
  }
  out[(u64)blockIdx.x * kBlock + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// =============================================================== host side
namespace {

int fail(int code, const std::string& msg) { return mw_fail(code, msg.c_str()); }

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t _e = (x);                                                            \
    if (_e != hipSuccess) return fail(MG_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

struct Prog;

// A search between its enqueue and its completion: mg_search does both in
// one call; mg_search_begin returns after the enqueue so the caller can work
// on the host (compile the witness programs) while the device searches, and
// mg_search_end completes it.  Meanwhile the context's launch records stay
// untouched: every other call that uses them is refused (context_busy).
struct Pending {
  bool active = false;
  std::vector<std::shared_ptr<Prog>> ps;   // the programs, alive until the end
  std::vector<size_t> slot;                // program i's word in d_min
  std::vector<size_t> interp, special;     // d_min order (search_complete)
  size_t nia = 0;
  u64 count = 0, ops = 0, seed = 0;
  u32 flags = 0;
  size_t nlaunches = 0;
  double t0 = 0.0;
  bool gpu_steps = false;
};

struct Ctx {
  int dev = 0;
  int ncu = 256;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipEvent_t ea = nullptr, eb = nullptr;   // step-time accounting only (MYTHRIL_AMD_STEP_TIMES=1)
  hipEvent_t eu = nullptr;                 // ... recorded before a program upload's copy
  bool eu_live = false;
  u32* d_spill = nullptr;
  size_t spill_bytes = 0;
  // One call's launch records, in one device block mirrored by a pinned host
  // block (stage_upload / stage_readback): counters, d_min, ProgDev records,
  // AsmArgs records.  A call uploads them with one copy and reads counters and
  // d_min back with one copy.
  uint8_t* d_blk = nullptr;
  uint8_t* h_blk = nullptr;
  size_t off_min = 0, off_progs = 0, off_args = 0;
  u64* d_counter = nullptr;   // [0] evals, [1..4] division steps/full/short/general x lanes (mg_stats)
  u64* d_min = nullptr;
  size_t nmin = 0;
  ProgDev* d_progs = nullptr; // nmin records
  AsmArgs* d_asmargs = nullptr;  // AsmArgs records: [0] the asm interpreter's launch, [1..] assembled kernels'
  size_t nasmargs_cap = 0;
  u32* d_alive = nullptr;     // per-candidate alive bits between the parts of a split program
  size_t alive_cap = 0;
  // pinned staging of program uploads (mg_prog_load): the copy is queued on
  // the stream, ahead of every launch that reads the program; the next upload
  // waits for it before reusing the buffer (up_pending).  Two buffers, used
  // in turn: a second upload right after the first (the witness programs of
  // mg_search_end after the search's) needs no synchronisation
  uint8_t* h_up[2] = {nullptr, nullptr};
  size_t up_bytes[2] = {0, 0};
  bool up_pending[2] = {false, false};
  int up_next = 0;
  void uploads_landed() { up_pending[0] = up_pending[1] = false; }
  // pinned landing area of small readbacks (eval verdicts and traces)
  uint8_t* h_rb = nullptr;
  size_t rb_bytes = 0;
  std::mutex mu;                 // serialises the calls on this context (mw_handles.h)
  bool dead = false;             // freed by mg_free (guarded by mu)
  // device buffers returned by freed programs and finished calls, by size
  // class (pool_get / pool_put below; guarded by mu)
  std::map<size_t, std::vector<void*>> pool;
  size_t pool_cached = 0;
  Pending pending;               // a begun search (mg_search_begin), guarded by mu
  uint8_t* h_wit = nullptr;      // pinned staging of the witness records (mg_search_end)
  size_t wit_bytes = 0;
};

struct Prog {
  std::shared_ptr<Ctx> ctx;     // keeps the context's record alive while this program's is
  bool dead = false;            // resources released (guarded by ctx->mu)
  u32* d_buf = nullptr;
  size_t buf_cls = 0;           // d_buf's size class in the context's pool
  ProgDev dev{};
  mg_prog_desc desc{};
  u64 ops_per_eval = 0;
  u64 sig = 0;                  // FNV-1a 64 of the program words (mythril_amd/jit.py signature)
  bool sig_ready = false;       // computed on the first attach (program_signature), not at load
  bool asm_ok = false;          // every opcode and leaf kind has a handler in mw_search_asm_kernel
  u8 asm_layout = kWide;        // the asm kernel adev is predecoded for (kAsmKernel)
  bool trace_full = false;      // STOREs cover every trace row: an evaluation needs no zeroed trace block
  ProgDev adev{};               // dev with code = its predecoded copy (mw_asm_predecode) and leaves =
                                // the asm leaf table (asm_leaf_table), in d_buf
  // specialised kernels (mg_prog_attach_kernel): one per part, launched in order
  struct Part {
    hipModule_t mod = nullptr;
    hipFunction_t fx = nullptr;  // exhaustive
    hipFunction_t fe = nullptr;  // early exit (optional)
  };
  std::vector<Part> parts;
  // assembled kernel (mg_prog_attach_asm): the asm interpreter's launch
  // records and grid, the program as straight-line code
  hipModule_t amod = nullptr;
  hipFunction_t afn = nullptr;
  bool jit_ready() const {
    if (parts.empty()) return false;
    for (const Part& q : parts)
      if (!q.fx) return false;
    return true;
  }
  void unload() {
    for (Part& q : parts)
      if (q.mod) hipModuleUnload(q.mod);
    parts.clear();
    if (amod) hipModuleUnload(amod);
    amod = nullptr;
    afn = nullptr;
  }
};

namespace {

u64 fnv1a(u64 h, const u32* w, size_t n) {
  for (size_t i = 0; i < n; ++i)
    for (int b = 0; b < 4; ++b) {
      h ^= (w[i] >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ull;
    }
  return h;
}


// A loaded program's signature (the context's mu held), from its words read
// back from the device on the first attach: only the specialised and
// assembled kernels check it, so an upload does not hash every program
// (mg_prog_load's FNV pass was a fifth of a LASER load, tools/dropin_profile.py).
u64 program_signature(Ctx* c, Prog* p) {
  if (p->sig_ready) return p->sig;
  const mg_prog_desc& d = p->desc;
  const size_t nl = d.nleaves * MW_LEAF_WORDS;
  std::vector<u32> w(d.ncode_words + d.nconst_words + nl + d.npool_words);
  u32* o = w.data();
  hipStreamSynchronize(c->stream);   // the upload may still be queued
  bool ok = hipMemcpy(o, p->dev.code, d.ncode_words * 4, hipMemcpyDeviceToHost) == hipSuccess;
  o += d.ncode_words;
  if (ok && d.nconst_words) ok = hipMemcpy(o, p->dev.consts, d.nconst_words * 4, hipMemcpyDeviceToHost) == hipSuccess;
  o += d.nconst_words;
  if (ok && nl) ok = hipMemcpy(o, p->dev.leaves, nl * 4, hipMemcpyDeviceToHost) == hipSuccess;
  o += nl;
  if (ok && d.npool_words) ok = hipMemcpy(o, p->dev.pool, d.npool_words * 4, hipMemcpyDeviceToHost) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    return ~0ull;   // matches no code object: the attach is refused
  }
  u64 h = 0xcbf29ce484222325ull;
  h = fnv1a(h, w.data(), w.size());
  p->sig = h;
  p->sig_ready = true;
  return h;
}

// Launch a program's specialised kernels over [begin, begin+count): one block
// per 256-candidate chunk (mw_jit.h), at most 2^30 blocks per launch.  A split
// program runs its parts in order over slices of kAliveSlice candidates,
// passing alive bits through c->d_alive.
constexpr u64 kAliveSlice = 1ull << 24;

int launch_part(Ctx* c, const Prog* p, size_t k, u64 seed, u64 begin, u64 count, u32 flags, u64* d_min,
                u32* d_verdict, u32 stage) {
  const Prog::Part& q = p->parts[k];
  hipFunction_t f = ((flags & MW_FLAG_EARLY_EXIT) && q.fe) ? q.fe : q.fx;
  const u64 nchunks = (count + kBlock - 1) / kBlock;
  const u64 kMaxBlocks = 1ull << 30;
  for (u64 chunk0 = 0; chunk0 < nchunks; chunk0 += kMaxBlocks) {
    const u32 nb = (u32)std::min<u64>(kMaxBlocks, nchunks - chunk0);
    const u32* pool = p->dev.pool;
    u64 sd = seed, bg = begin, ct = count, c0 = chunk0;
    u32 fl = flags, st = stage;
    u64* mn = d_min;
    u64* ctr = c->d_counter;
    u32* vd = d_verdict;
    u32* al = c->d_alive;
    void* args[] = {&pool, &sd, &bg, &ct, &c0, &fl, &mn, &ctr, &vd, &al, &st};
    HIPCHK(hipModuleLaunchKernel(f, nb, 1, 1, kBlock, 1, 1, 0, c->stream, args, nullptr));
  }
  return 0;
}

int launch_jit(Ctx* c, const Prog* p, u64 seed, u64 begin, u64 count, u32 flags, u64* d_min,
               u32* d_verdict) {
  const size_t np = p->parts.size();
  if (np == 1) return launch_part(c, p, 0, seed, begin, count, flags, d_min, d_verdict, 3u);
  const size_t need = (size_t)std::min<u64>(count, kAliveSlice);
  if (need > c->alive_cap) {
    if (c->d_alive) HIPCHK(hipFree(c->d_alive));
    c->d_alive = nullptr;
    c->alive_cap = 0;
    HIPCHK(hipMalloc(&c->d_alive, need * sizeof(u32)));
    c->alive_cap = need;
  }
  for (u64 s0 = 0; s0 < count; s0 += kAliveSlice) {
    const u64 sc = std::min<u64>(kAliveSlice, count - s0);
    for (size_t k = 0; k < np; ++k) {
      const u32 stage = (k == 0 ? 1u : 0u) | (k + 1 == np ? 2u : 0u);
      int rc = launch_part(c, p, k, seed, begin + s0, sc, flags, d_min, d_verdict ? d_verdict + s0 : nullptr, stage);
      if (rc) return rc;
    }
  }
  return 0;
}

// Live handles (include/mythril_witness.h, "Lifetimes"; the protocol is
// mw_handles.h): handles are ids that are never reused, resolved to
// reference-counted records, and every call re-checks them under the
// context's lock, so freeing in the wrong order, twice, or while another
// thread uses the handle is an MG_E_ARG, never a use-after-free.
mw::Registry<Ctx, Prog> g_reg;
using CallG = mw::Call<Ctx, Prog>;

inline u64 hid(const void* h) { return (u64)(uintptr_t)h; }

// the device resources of a program (its context's mu held)
// Device memory of one context is reused across calls: program buffers and
// per-call scratch come from power-of-two size classes (from 4 KiB) and go
// back there, instead of a hipMalloc and a hipFree per call (hipFree waits for
// the whole device; on the get_model path a query loads, searches and frees a
// program, and a witness loads and frees another).  Idle buffers are capped
// for the whole process, over all contexts (MYTHRIL_AMD_POOL_CACHE_MB, default
// 256): another context on the same device (a second Device, the keccak
// service) never meets an allocation failure behind more than that much
// cached memory; mg_free releases a context's buffers.  Every call
// synchronises its stream before it returns a buffer, so a reused buffer has
// no work pending.
std::atomic<size_t> g_pool_cached{0};

size_t pool_cache_limit() {
  static const size_t lim = [] {
    const char* e = getenv("MYTHRIL_AMD_POOL_CACHE_MB");
    long mb = e ? atol(e) : 256;
    return size_t(mb < 0 ? 0 : mb) << 20;
  }();
  return lim;
}

size_t pool_class(size_t bytes) {
  size_t k = 4096;
  while (k < bytes) k <<= 1;
  return k;
}

void pool_drain(Ctx* c) {
  for (auto& kv : c->pool)
    for (void* q : kv.second) hipFree(q);
  c->pool.clear();
  g_pool_cached -= c->pool_cached;
  c->pool_cached = 0;
}

void* pool_get(Ctx* c, size_t bytes, size_t* cls) {
  const size_t k = pool_class(bytes);
  *cls = k;
  auto it = c->pool.find(k);
  if (it != c->pool.end() && !it->second.empty()) {
    void* q = it->second.back();
    it->second.pop_back();
    c->pool_cached -= k;
    g_pool_cached -= k;
    return q;
  }
  void* q = nullptr;
  mw::inflight_step("pool_get/hipMalloc", k);
  if (hipMalloc(&q, k) == hipSuccess) return q;
  (void)hipGetLastError();
  mw::inflight_step("pool_get/drain", c->pool_cached);
  pool_drain(c);   // memory pressure: give the cached buffers back and try once more
  if (hipMalloc(&q, k) == hipSuccess) return q;
  (void)hipGetLastError();
  return nullptr;
}

void pool_put(Ctx* c, void* q, size_t cls) {
  if (!q) return;
  if (g_pool_cached.fetch_add(cls) + cls > pool_cache_limit()) {
    g_pool_cached -= cls;
    mw::inflight_step("pool_put/hipFree", cls);
    hipFree(q);
    return;
  }
  c->pool[cls].push_back(q);
  c->pool_cached += cls;
}

// A scratch buffer for one call: back to the pool when the call returns (after
// a stream synchronisation if the call did not reach its own).
struct Scratch {
  Ctx* c;
  void* p = nullptr;
  size_t cls = 0;
  bool synced = false;
  Scratch(Ctx* ctx, size_t bytes) : c(ctx) { if (bytes) p = pool_get(c, bytes, &cls); }
  ~Scratch() {
    if (!p) return;
    if (!synced) hipStreamSynchronize(c->stream);
    pool_put(c, p, cls);
  }
  u32* u() const { return (u32*)p; }
};

void release_prog(Prog& p) {
  hipSetDevice(p.ctx->dev);
  mw::inflight_step("release_prog/unload");
  p.unload();
  // every call on the context synchronises before it returns (and this runs
  // under the context's mu): no kernel still reads the buffer.  Only
  // mg_prog_load returns with its upload queued; whatever reuses the buffer
  // next is queued after that copy on the same stream
  // ... except a begun search (mg_search_begin): let it finish first
  if (p.d_buf && p.ctx->pending.active) hipStreamSynchronize(p.ctx->stream);
  if (p.d_buf) pool_put(p.ctx.get(), p.d_buf, p.buf_cls);
  p.d_buf = nullptr;
}

void release_ctx(Ctx& c) {
  hipSetDevice(c.dev);
  mw::inflight_step("release_ctx/sync");
  if (c.stream) hipStreamSynchronize(c.stream);
  mw::inflight_step("release_ctx/drain", c.pool_cached);
  pool_drain(&c);
  mw::inflight_step("release_ctx/free");
  if (c.d_spill) hipFree(c.d_spill);
  if (c.d_blk) hipFree(c.d_blk);
  if (c.h_blk) hipHostFree(c.h_blk);
  for (int k = 0; k < 2; ++k)
    if (c.h_up[k]) hipHostFree(c.h_up[k]);
  if (c.h_rb) hipHostFree(c.h_rb);
  if (c.h_wit) hipHostFree(c.h_wit);
  c.h_wit = nullptr;
  c.wit_bytes = 0;
  c.pending = Pending();
  c.h_rb = nullptr;
  c.rb_bytes = 0;
  c.h_up[0] = c.h_up[1] = nullptr;
  c.up_bytes[0] = c.up_bytes[1] = 0;
  c.uploads_landed();
  if (c.d_alive) hipFree(c.d_alive);
  if (c.e0) hipEventDestroy(c.e0);
  if (c.e1) hipEventDestroy(c.e1);
  if (c.ea) hipEventDestroy(c.ea);
  if (c.eb) hipEventDestroy(c.eb);
  if (c.eu) hipEventDestroy(c.eu);
  c.ea = c.eb = c.eu = nullptr;
  if (c.stream) hipStreamDestroy(c.stream);
  c.d_spill = nullptr;
  c.d_blk = c.h_blk = nullptr;
  c.d_min = nullptr;
  c.d_progs = nullptr;
  c.d_asmargs = nullptr;
  c.d_counter = nullptr;
  c.nmin = c.nasmargs_cap = 0;
  c.d_alive = nullptr;
  c.e0 = c.e1 = nullptr;
  c.stream = nullptr;
}

// Room for nmin d_min words and ProgDev records and nargs AsmArgs records in
// the launch block.  Runs before a call enqueues anything (the previous call on
// the context synchronised before it returned).
int ensure_launch(Ctx* c, size_t nmin, size_t nargs) {
  if (c->d_blk && nmin <= c->nmin && nargs <= c->nasmargs_cap) return 0;
  nmin = std::max({nmin, c->nmin, (size_t)16});
  nargs = std::max({nargs, c->nasmargs_cap, (size_t)4});
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t off_min = up(kCounterWords * sizeof(u64));
  const size_t off_progs = up(off_min + nmin * sizeof(u64));
  const size_t off_args = up(off_progs + nmin * sizeof(ProgDev));
  const size_t bytes = up(off_args + nargs * sizeof(AsmArgs));
  mw::inflight_step("ensure_launch/realloc", bytes);
  if (c->d_blk) HIPCHK(hipFree(c->d_blk));
  if (c->h_blk) HIPCHK(hipHostFree(c->h_blk));
  c->d_blk = c->h_blk = nullptr;
  c->d_counter = c->d_min = nullptr;
  c->d_progs = nullptr;
  c->d_asmargs = nullptr;
  c->nmin = c->nasmargs_cap = 0;
  HIPCHK(hipMalloc(&c->d_blk, bytes));
  HIPCHK(hipHostMalloc(&c->h_blk, bytes, hipHostMallocDefault));
  c->off_min = off_min;
  c->off_progs = off_progs;
  c->off_args = off_args;
  c->d_counter = (u64*)c->d_blk;
  c->d_min = (u64*)(c->d_blk + off_min);
  c->d_progs = (ProgDev*)(c->d_blk + off_progs);
  c->d_asmargs = (AsmArgs*)(c->d_blk + off_args);
  c->nmin = nmin;
  c->nasmargs_cap = nargs;
  return 0;
}

// Stage a call's launch records in the pinned mirror and enqueue one upload:
// zeroed counters, nmin d_min words at MG_NONE, nprogs ProgDev records and
// nargs AsmArgs records (ensure_launch sized the block).
hipError_t stage_upload(Ctx* c, size_t nmin, const ProgDev* progs, size_t nprogs, const AsmArgs* args,
                        size_t nargs) {
  std::memset(c->h_blk, 0, kCounterWords * sizeof(u64));
  u64* hm = (u64*)(c->h_blk + c->off_min);
  for (size_t i = 0; i < nmin; ++i) hm[i] = MG_NONE;
  size_t end = c->off_min + nmin * sizeof(u64);
  if (nprogs) {
    std::memcpy(c->h_blk + c->off_progs, progs, nprogs * sizeof(ProgDev));
    end = c->off_progs + nprogs * sizeof(ProgDev);
  }
  if (nargs) {
    std::memcpy(c->h_blk + c->off_args, args, nargs * sizeof(AsmArgs));
    end = c->off_args + nargs * sizeof(AsmArgs);
  }
  return hipMemcpyAsync(c->d_blk, c->h_blk, end, hipMemcpyHostToDevice, c->stream);
}

// Enqueue one readback of the counters and the first nmin d_min words into the
// pinned mirror (read them there after the stream synchronises).
hipError_t stage_readback(Ctx* c, size_t nmin) {
  return hipMemcpyAsync(c->h_blk, c->d_blk, c->off_min + nmin * sizeof(u64), hipMemcpyDeviceToHost, c->stream);
}

// One launch of a program's assembled kernel: the asm interpreter's grid (x:
// chunk stride, one program) and records (mw_asm_abi.h); its LDS is a fixed
// 80 KiB array in the kernel (mw_asmjit_shell.hip).
int launch_assembled(Ctx* c, const Prog* p, u32 gx, const ProgDev* dprog, const AsmArgs* dargs, u64* dmin,
                     u32 nlds) {
  u64* ctr = c->d_counter;
  void* args[] = {&dprog, &dargs, &dmin, &ctr, &nlds};
  HIPCHK(hipModuleLaunchKernel(p->afn, gx, 1, 1, kBlock, 1, 1, 0, c->stream, args, nullptr));
  return 0;
}

int ensure_spill(Ctx* c, size_t bytes) {
  if (bytes <= c->spill_bytes) return 0;
  mw::inflight_step("ensure_spill/realloc", bytes);
  if (c->d_spill) HIPCHK(hipFree(c->d_spill));
  c->d_spill = nullptr;
  c->spill_bytes = 0;
  HIPCHK(hipMalloc(&c->d_spill, bytes));
  c->spill_bytes = bytes;
  return 0;
}

// mw_search_asm_kernel handles this program: every opcode in MW_ASM_OPCODES,
// every leaf kind in MW_ASM_LEAF_KINDS (validated programs only)
bool asm_eligible(const mg_prog_desc* d) {
  static const u32 ops[] = {MW_ASM_OPCODES};
  static const u32 kinds[] = {MW_ASM_LEAF_KINDS};
  bool ok_op[256] = {false};
  for (u32 o : ops) ok_op[o & 0xffu] = true;
  u32 ndiv = 0;   // bit-serial wide divisions (asmgen.py udivrem): a few at most (isa.ASM_MAX_DIV)
  for (size_t i = 0; i < d->ncode_words / 4; ++i) {
    const u32 op = d->code[4 * i] & 0xffu;
    if (!ok_op[op]) return false;
    ndiv += (op == MW_W_UDIV || op == MW_W_UREM) ? 1u : 0u;
  }
  if (ndiv > MW_ASM_MAX_DIV) return false;
  for (size_t l = 0; l < d->nleaves; ++l) {
    const u32 kind = d->leaves[l * MW_LEAF_WORDS + MW_LEAF_KIND];
    bool ok = false;
    for (u32 k : kinds) ok = ok || k == kind;
    if (!ok) return false;
  }
  return true;
}

// LDS words of spill area for an asm launch whose largest pool has max_pool
// words: the pool is staged whole in LDS, the hottest spill words take what is
// left of the block's 80 KiB and the rest spill to the global buffer.  False if
// the pool alone does not fit (the programs then run on the compiled interpreter).
// The narrow-layout kernel's budget: 52 KiB per block, so three blocks (three
// waves per SIMD) fit a CU's 160 KiB; the quarter layout's 40 KiB (four).
constexpr u32 kLdsSpillWordsByLayout[kAsmLayouts] = {kLdsSpillWords, 52, 40};

// MYTHRIL_AMD_ASM_WIDE_LDS=n (81..160): the wide kernel's budget in words (A/B
// runs: a program that spills past 80 words keeps them in LDS at one block,
// one wave per SIMD, instead of two with the rest in global memory)
u32 wide_lds_words() {
  static const u32 w = [] {
    const char* e = std::getenv("MYTHRIL_AMD_ASM_WIDE_LDS");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return v > (long)kLdsSpillWords && v <= 160 ? (u32)v : kLdsSpillWords;
  }();
  return w;
}

bool asm_lds_fit(u32 max_spill, u32 max_pool, u32* nlds, u8 layout = kWide, bool interp = false) {
  const u32 words = layout == kWide && interp ? wide_lds_words() : kLdsSpillWordsByLayout[layout];
  const size_t budget = (size_t)words * kBlock * 4, pool_bytes = (size_t)max_pool * 4;
  if (pool_bytes > budget) return false;
  const u32 pool_words_lds = (u32)((pool_bytes + kBlock * 4 - 1) / (kBlock * 4));  // in spill-word rows
  *nlds = std::min(max_spill, words - pool_words_lds);
  return true;
}

bool asm_lds_fit(const Prog* p, u32* nlds) {
  return asm_lds_fit(p->dev.n_spill, p->dev.npool, nlds, p->asm_layout, true);
}

// MYTHRIL_AMD_ASM=0 keeps every program on the compiled interpreter (A/B runs, tests)
bool asm_enabled() {
  const char* e = std::getenv("MYTHRIL_AMD_ASM");
  return !(e && e[0] == '0');
}

// MYTHRIL_AMD_ASM_NARROW=0 predecodes every asm program for the wide kernel,
// MYTHRIL_AMD_ASM_QUARTER=0 keeps programs off the quarter layout (A/B runs)
bool asm_narrow_enabled() {
  const char* e = std::getenv("MYTHRIL_AMD_ASM_NARROW");
  return !(e && e[0] == '0');
}

bool asm_quarter_enabled() {
  const char* e = std::getenv("MYTHRIL_AMD_ASM_QUARTER");
  return asm_narrow_enabled() && !(e && e[0] == '0');
}

// The asm interpreter's introspection table, as the kernel itself reports it
// (AsmArgs.flags bit 7, mythril_amd/asmgen.py gen "introspection"): handler
// word offsets per opcode and fused sequence for each of its two instruction
// banks, then its base address.  mw_asm_predecode turns them into absolute
// handler addresses in the instructions, so the dispatch is one move and one
// jump.  Read once per device (each device loads the code object at its own
// address); until then, or if it fails, no program is asm-eligible there (the
// compiled interpreter runs them: same results).
constexpr int kMaxDevices = 64;
std::mutex g_hoff_mu;
bool g_hoff_ready[kMaxDevices];
u32 g_hoff[kMaxDevices][MW_ASM_NHTAB];     // mw_search_asm_kernel (mw_asm_interp.inc)
u32 g_hoff_n[kMaxDevices][MW_ASM_NHTAB];   // the same for mw_search_asm_kernel_n
u32 g_hoff_q[kMaxDevices][MW_ASM_NHTAB];   // and mw_search_asm_kernel_q

template <typename K>
int introspect(K kernel, hipStream_t stream, u32* hout) {
  void* buf = nullptr;
  const size_t bytes = sizeof(ProgDev) + sizeof(AsmArgs) + MW_ASM_NHTAB * sizeof(u32) + 2 * sizeof(u64);
  HIPCHK(hipMalloc(&buf, bytes));
  char* b = (char*)buf;
  ProgDev* dp = (ProgDev*)b;
  AsmArgs* da = (AsmArgs*)(b + sizeof(ProgDev));
  u32* dout = (u32*)(b + sizeof(ProgDev) + sizeof(AsmArgs));
  u64* dmin = (u64*)(dout + MW_ASM_NHTAB + (MW_ASM_NHTAB & 1));
  ProgDev hp{};
  AsmArgs ha{};
  ha.flags = 1u << 7;
  ha.verdict = dout;
  hipError_t e = hipMemsetAsync(buf, 0, bytes, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dp, &hp, sizeof hp, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(da, &ha, sizeof ha, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(kernel, dim3(1u, 1u), dim3(kBlock), 0, stream, (const ProgDev*)dp,
                       (const AsmArgs*)da, dmin, dmin + 1, 0u);
    e = hipGetLastError();
  }
  u32 h[MW_ASM_NHTAB];
  if (e == hipSuccess) e = hipMemcpyAsync(h, dout, sizeof h, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  hipFree(buf);
  if (e != hipSuccess) return fail(MG_E_HIP, std::string("asm handler offsets: ") + hipGetErrorString(e));
  for (int k = 0; k < 2 * MW_ASM_NHANDLERS; ++k) {
    if (h[k] == 0 || h[k] > 0xfffffu) return fail(MG_E_HIP, "asm handler offsets out of range");
    hout[k] = h[k];
  }
  if (h[2 * MW_ASM_NHANDLERS] == 0 && h[2 * MW_ASM_NHANDLERS + 1] == 0)
    return fail(MG_E_HIP, "asm interpreter base address missing");
  hout[2 * MW_ASM_NHANDLERS] = h[2 * MW_ASM_NHANDLERS];
  hout[2 * MW_ASM_NHANDLERS + 1] = h[2 * MW_ASM_NHANDLERS + 1];
  return 0;
}

int asm_handler_offsets(int dev, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_hoff_mu);
  if (dev < 0 || dev >= kMaxDevices) return 0;   // no asm engine on that device
  if (g_hoff_ready[dev]) return 0;
  HIPCHK(hipSetDevice(dev));
  int rc = introspect(mw_search_asm_kernel, stream, g_hoff[dev]);
  if (rc == 0) rc = introspect(mw_search_asm_kernel_n, stream, g_hoff_n[dev]);
  if (rc == 0) rc = introspect(mw_search_asm_kernel_q, stream, g_hoff_q[dev]);
  if (rc == 0) g_hoff_ready[dev] = true;
  return rc;
}

bool asm_offsets_ready(int dev) {
  std::lock_guard<std::mutex> lk(g_hoff_mu);
  return dev >= 0 && dev < kMaxDevices && g_hoff_ready[dev];
}

// The asm engines' copy of the leaf table: word 6 (the input row, which only
// the compiled interpreter's mg_eval reads) becomes the leaf's digit group,
// the index of the first leaf whose pool digit is the same function of the
// candidate (kind, shift, bits, stride, and the hash key for hashed digits):
// the Lleaf subroutine (mythril_amd/asmgen.py leaf) reuses the digit of the
// last pooled leaf it drew when the group matches, as the bytes of one
// calldata word do (LeafSpec.tie).  Leaves without a pool digit: 0xfffffffe.
void asm_leaf_table(const u32* leaves, size_t n, u32* out) {
  std::map<std::array<u32, 5>, u32> first;
  for (size_t i = 0; i < n; ++i) {
    const u32* L = leaves + i * MW_LEAF_WORDS;
    u32* O = out + i * MW_LEAF_WORDS;
    std::memcpy(O, L, MW_LEAF_WORDS * sizeof(u32));
    const u32 kind = L[1];
    if (kind < 1 || kind > 3) {
      O[6] = 0xfffffffeu;
      continue;
    }
    const std::array<u32, 5> key = {kind, L[3], L[4], L[7], kind == 2 ? L[2] : 0u};
    O[6] = first.emplace(key, (u32)i).first->second;
  }
}

}  // namespace

extern "C" {

int mg_device_count(int* n) {
  if (!n) return fail(MG_E_ARG, "null out");
  int c = 0;
  HIPCHK(hipGetDeviceCount(&c));
  *n = c;
  return 0;
}

int mg_init(int device, mg_ctx** out) {
  mw::CallMark mark("mg_init");
  if (!out) return fail(MG_E_ARG, "null out");
  *out = nullptr;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(MG_E_ARG, "no such device");
  HIPCHK(hipSetDevice(device));
  // MYTHRIL_AMD_SPIN=1 (A/B runs, tools/dropin_profile.py): synchronising
  // threads spin instead of yielding (lower wake-up latency per call)
  if (const char* e = std::getenv("MYTHRIL_AMD_SPIN"); e && e[0] == '1') {
    if (hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess) (void)hipGetLastError();
  }
  auto c = std::make_shared<Ctx>();
  c->dev = device;
  mark.step("properties");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->ncu = prop.multiProcessorCount;
  mark.step("stream");
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess ||
      (mw::step_times_on() && (hipEventCreate(&c->ea) != hipSuccess || hipEventCreate(&c->eb) != hipSuccess ||
                               hipEventCreate(&c->eu) != hipSuccess)) ||
      ensure_launch(c.get(), 16, 4) != 0) {
    release_ctx(*c);
    return fail(MG_E_HIP, "context setup failed");
  }
  // allow the LDS spill area (up to kLdsSpillWords x 1 KiB) beyond the 64 KiB default
  const int lds_max = (int)(kLdsSpillWords * kBlock * sizeof(u32));
  mark.step("attributes");
  if (hipFuncSetAttribute((const void*)mw_search_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
          hipSuccess ||
      hipFuncSetAttribute((const void*)mw_search_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
          hipSuccess ||
      hipFuncSetAttribute((const void*)mw_eval_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
          hipSuccess ||
      hipFuncSetAttribute((const void*)mw_search_asm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)(wide_lds_words() * kBlock * sizeof(u32))) != hipSuccess ||
      hipFuncSetAttribute((const void*)mw_search_asm_kernel_n, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
          hipSuccess ||
      hipFuncSetAttribute((const void*)mw_search_asm_kernel_q, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
          hipSuccess) {
    (void)hipGetLastError();  // older runtimes: the default limit already covers it
  }
  mark.step("asm offsets");
  if (asm_enabled() && asm_handler_offsets(c->dev, c->stream) != 0) {
    (void)hipGetLastError();  // the asm interpreter stays off: the compiled interpreter runs every program
    std::fprintf(stderr, "[mythril_amd] asm interpreter disabled: %s\n", mg_last_error());
  }
  *out = (mg_ctx*)(uintptr_t)g_reg.add_ctx(std::move(c));
  return 0;
}

int mg_free(mg_ctx* h) {
  if (!h) return 0;
  mw::CallMark mark("mg_free");
  mark.step("lock");
  // programs still loaded in this context are freed with it; a call in flight
  // on another thread finishes first (mw_handles.h free_ctx)
  if (!mw::free_ctx(g_reg, hid(h), release_prog, release_ctx)) return fail(MG_E_ARG, "mg_free: not a live context");
  return 0;
}

// Every trace row is written by some STORE of the program (rows validated in
// range, mw_validate.cpp); evaluations never exit early, so each STORE runs for
// every candidate and the rows need no zeroing first.
static bool trace_rows_covered(const mg_prog_desc* d) {
  if (!d->n_trace_rows) return false;
  std::vector<char> cov(d->n_trace_rows, 0);
  size_t left = d->n_trace_rows;
  for (size_t i = 0; i + 3 < d->ncode_words && left; i += 4) {
    const u32 op = d->code[i] & 0xffu, r = d->code[i + 3];
    const u32 n = op == MW_STORE_W ? 8u : op == MW_STORE_N ? 1u : 0u;
    for (u32 k = 0; k < n; ++k)
      if ((u64)r + k < d->n_trace_rows && !cov[r + k]) cov[r + k] = 1, --left;
  }
  return left == 0;
}

// The upload of a validated program into context c (its mu held, the
// device set): device buffer from the pool, staged through the pinned
// buffer, predecoded for the smallest asm layout that holds it, copy queued.
static int load_locked(const std::shared_ptr<Ctx>& cref, const mg_prog_desc* d, std::shared_ptr<Prog>& out) {
  Ctx* c = cref.get();
  mw::CallMark mark("load_locked");   // nested: its steps are the caller's
  // constants padded to >= MW_KPAD words: the interpreter's branch-free narrow
  // operand fetch reads cpool[slot] (slot < 64) before selecting the register
  const size_t nc = d->ncode_words, nk = (d->nconst_words + 8 > MW_KPAD ? d->nconst_words + 8 : MW_KPAD), nl = d->nleaves * MW_LEAF_WORDS + 8,
               np = d->npool_words + 8;
  bool asm_ok = asm_offsets_ready(c->dev) && asm_eligible(d);
  // predecoded copy + the block after END the dispatch prefetches + the narrow
  // constants the kernel loads into VGPRs (MW_ASM_NK words) + the asm leaf table
  const size_t na = asm_ok ? nc + 8 + MW_ASM_NK + nl : 0;
  const size_t total = nc + nk + nl + np + na;
  auto p = std::make_shared<Prog>();
  p->ctx = cref;
  p->desc = *d;
  p->ops_per_eval = d->ops_per_eval;
  p->trace_full = trace_rows_covered(d);
  mark.step("pool_get", total * 4);
  p->d_buf = (u32*)pool_get(c, total * sizeof(u32), &p->buf_cls);
  if (!p->d_buf) return fail(MG_E_NOMEM, "program upload allocation failed");
  // stage in the context's pinned buffer (after the previous upload from it has landed)
  mark.step("sync previous upload");
  const int ub = c->up_next;
  c->up_next ^= 1;
  if (c->up_pending[ub] && hipStreamSynchronize(c->stream) != hipSuccess) {
    release_prog(*p);
    return fail(MG_E_HIP, "program upload: stream synchronize failed");
  }
  if (c->up_pending[ub]) c->uploads_landed();   // the stream drained
  if (total * 4 > c->up_bytes[ub]) {
    mark.step("staging regrow", total * 4);
    if (c->h_up[ub]) hipHostFree(c->h_up[ub]);
    c->h_up[ub] = nullptr;
    c->up_bytes[ub] = 0;
    const size_t want = std::max<size_t>(total * 4, (size_t)1 << 18);
    if (hipHostMalloc(&c->h_up[ub], want, hipHostMallocDefault) != hipSuccess) {
      release_prog(*p);
      return fail(MG_E_NOMEM, "program upload staging allocation failed");
    }
    c->up_bytes[ub] = want;
  }
  mark.step("stage + predecode", total * 4);
  u32* hbuf = (u32*)c->h_up[ub];
  std::memset(hbuf, 0, total * 4);
  std::memcpy(hbuf, d->code, nc * 4);
  if (d->nconst_words) std::memcpy(hbuf + nc, d->consts, d->nconst_words * 4);
  if (d->nleaves) std::memcpy(hbuf + nc + nk, d->leaves, d->nleaves * MW_LEAF_WORDS * 4);
  if (d->npool_words) std::memcpy(hbuf + nc + nk + nl, d->pool, d->npool_words * 4);
  u8 layout = kWide;
  if (asm_ok) {
    u32* pre = hbuf + nc + nk + nl + np;
    // the smallest register layout whose files hold every register of the
    // program, whose LDS budget holds its pool (the quarter layout: its spill
    // words too) and whose registers its narrow constants: the quarter kernel
    // (four waves per SIMD), else the narrow one (three), else the wide one.
    // More distinct narrow constants than MW_ASM_NK: the compiled interpreter runs it
    u32 nl0 = 0;
    if (asm_quarter_enabled() && asm_lds_fit(d->n_spill, (u32)d->npool_words, &nl0, kQuarter) &&
        nl0 == d->n_spill &&
        mw_asm_predecode_layout(d->code, nc, d->consts, d->nconst_words, g_hoff_q[c->dev], pre, pre + nc + 8,
                                MW_ASM_NK_INDEX_Q, MW_ASM_NK_Q, MW_ASM_NFILE_Q, MW_ASM_WFILE_Q) == 0) {
      layout = kQuarter;
    } else if (asm_narrow_enabled() && asm_lds_fit(d->n_spill, (u32)d->npool_words, &nl0, kNarrow) &&
               (std::memset(pre, 0, (nc + 8 + MW_ASM_NK) * 4),
                mw_asm_predecode_layout(d->code, nc, d->consts, d->nconst_words, g_hoff_n[c->dev], pre,
                                        pre + nc + 8, MW_ASM_NK_INDEX_N, MW_ASM_NK_N, MW_ASM_NFILE_N, 0) == 0)) {
      layout = kNarrow;
    } else {
      std::memset(pre, 0, (nc + 8 + MW_ASM_NK) * 4);
      asm_ok = mw_asm_predecode(d->code, nc, d->consts, d->nconst_words, g_hoff[c->dev], pre, pre + nc + 8) == 0;
    }
    if (asm_ok) asm_leaf_table(d->leaves, d->nleaves, pre + nc + 8 + MW_ASM_NK);
  }
  // queued on the context's stream: every launch that reads the program is
  // queued after it on the same stream
  mark.step("upload", total * 4);
  if (c->eu && !c->eu_live) c->eu_live = hipEventRecord(c->eu, c->stream) == hipSuccess;
  if (hipMemcpyAsync(p->d_buf, hbuf, total * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
    release_prog(*p);
    return fail(MG_E_HIP, "program upload copy failed");
  }
  c->up_pending[ub] = true;
  p->dev.code = p->d_buf;
  p->dev.consts = p->d_buf + nc;
  p->dev.leaves = p->d_buf + nc + nk;
  p->dev.pool = p->d_buf + nc + nk + nl;
  p->dev.n_spill = d->n_spill;
  p->dev.npool = (u32)d->npool_words;
  p->dev.n_insn = (u32)(nc / 4);
  p->asm_ok = asm_ok;
  p->asm_layout = asm_ok ? layout : (u8)kWide;
  p->adev = p->dev;
  if (asm_ok) {
    p->adev.code = p->d_buf + nc + nk + nl + np;
    p->adev.leaves = p->adev.code + nc + 8 + MW_ASM_NK;
  }
  // the desc's host pointers are not retained
  p->desc.code = nullptr;
  p->desc.consts = nullptr;
  p->desc.leaves = nullptr;
  p->desc.pool = nullptr;
  out = std::move(p);
  return 0;
}

int mg_prog_load(mg_ctx* h, const mg_prog_desc* d, mg_prog** out) {
  if (!h || !d || !out) return fail(MG_E_ARG, "null argument");
  *out = nullptr;
  mw::CallMark mark("mg_prog_load");
  std::shared_ptr<Ctx> cref = g_reg.ctx(hid(h));
  if (!cref) return fail(MG_E_ARG, "mg_prog_load: not a live context");
  mark.step("validate", d->ncode_words);
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  Ctx* c = cref.get();
  mark.step("lock");
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->dead) return fail(MG_E_ARG, "mg_prog_load: the context was freed during the call");
  HIPCHK(hipSetDevice(c->dev));
  std::shared_ptr<Prog> p;
  rc = load_locked(cref, d, p);
  if (rc) return rc;
  *out = (mg_prog*)(uintptr_t)g_reg.add_prog(std::move(p));   // published under c->mu (mw_handles.h)
  return 0;
}

int mg_prog_free(mg_prog* h) {
  if (!h) return 0;
  mw::CallMark mark("mg_prog_free");
  mark.step("lock");
  if (!mw::free_prog(g_reg, hid(h), release_prog))
    return fail(MG_E_ARG, "mg_prog_free: not a live program (already freed, or freed with its context)");
  return 0;
}

int mg_prog_attach_kernel(mg_prog* h, const void* image, size_t size, const char* name) {
  if (!h || !image || !size || !name) return fail(MG_E_ARG, "null argument");
  if (std::strlen(name) > 200) return fail(MG_E_ARG, "kernel name too long");
  mw::CallMark mark("mg_prog_attach_kernel");
  mark.step("lock");
  CallG call;
  if (const char* why = mw::enter_prog(g_reg, hid(h), call)) return fail(MG_E_ARG, std::string("mg_prog_attach_kernel: ") + why);
  mark.step("hipModuleLoadData", size);
  Ctx* c = call.c.get();
  Prog* p = call.ps[0].get();
  HIPCHK(hipSetDevice(c->dev));
  hipModule_t mod = nullptr;
  HIPCHK(hipModuleLoadData(&mod, image));
  const std::string base(name);
  auto get32 = [&](const std::string& sym, u32* out) -> bool {
    hipDeviceptr_t d = nullptr;
    size_t n = 0;
    if (hipModuleGetGlobal(&d, &n, mod, sym.c_str()) != hipSuccess || n != sizeof(u32)) {
      (void)hipGetLastError();
      return false;
    }
    return hipMemcpyDtoH(out, d, sizeof(u32)) == hipSuccess;
  };
  hipDeviceptr_t dsig = nullptr;
  size_t nsig = 0;
  u64 sig = 0;
  hipFunction_t fx = nullptr, fe = nullptr;
  if (hipModuleGetGlobal(&dsig, &nsig, mod, (base + "_sig").c_str()) != hipSuccess || nsig != sizeof(u64) ||
      hipMemcpyDtoH(&sig, dsig, sizeof(u64)) != hipSuccess) {
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object has no program signature " + base + "_sig");
  }
  if (sig != program_signature(c, p)) {
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object was generated for another program (signature mismatch)");
  }
  u32 part = 0, nparts = 1;
  if (!get32(base + "_part", &part) || !get32(base + "_nparts", &nparts)) {
    part = 0;
    nparts = 1;
  }
  if (nparts == 0 || nparts > 1024 || part >= nparts) {
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "bad part index in code object");
  }
  if (hipModuleGetFunction(&fx, mod, (base + "_x").c_str()) != hipSuccess) {
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object lacks kernel " + base + "_x");
  }
  if (hipModuleGetFunction(&fe, mod, (base + "_e").c_str()) != hipSuccess) {
    (void)hipGetLastError();
    fe = nullptr;  // early exit is an optimisation only: the exhaustive kernel gives the same results
  }
  if (p->parts.size() != nparts) {  // a new split of this program replaces the old one
    p->unload();
    p->parts.resize(nparts);
  }
  Prog::Part& q = p->parts[part];
  if (q.mod) hipModuleUnload(q.mod);
  q.mod = mod;
  q.fx = fx;
  q.fe = fe;
  return 0;
}

int mg_prog_has_kernel(const mg_prog* h) {
  CallG call;
  if (mw::enter_prog(g_reg, hid(h), call)) return 0;
  return call.ps[0]->jit_ready() ? 1 : 0;
}

int mg_prog_engine(const mg_prog* h) {
  CallG call;
  if (const char* why = mw::enter_prog(g_reg, hid(h), call)) return fail(MG_E_ARG, std::string("mg_prog_engine: ") + why);
  const Prog* p = call.ps[0].get();
  if (p->jit_ready()) return 2;
  u32 nlds = 0;   // the engine mg_search gives this program alone (a pool too big for LDS: compiled)
  if (!p->asm_ok || !asm_enabled() || !asm_lds_fit(p, &nlds)) return 0;
  return p->afn ? 3 : 1;
}

int mg_prog_attach_asm(mg_prog* h, const void* image, size_t size, const char* name) {
  if (!h || !image || !size || !name) return fail(MG_E_ARG, "null argument");
  if (std::strlen(name) > 200) return fail(MG_E_ARG, "kernel name too long");
  mw::CallMark mark("mg_prog_attach_asm");
  mark.step("lock");
  CallG call;
  if (const char* why = mw::enter_prog(g_reg, hid(h), call)) return fail(MG_E_ARG, std::string("mg_prog_attach_asm: ") + why);
  mark.step("hipModuleLoadData", size);
  Ctx* c = call.c.get();
  Prog* p = call.ps[0].get();
  if (!p->asm_ok) return fail(MG_E_PROG, "mg_prog_attach_asm: the program has opcodes the asm engines lack");
  HIPCHK(hipSetDevice(c->dev));
  hipModule_t mod = nullptr;
  HIPCHK(hipModuleLoadData(&mod, image));
  const std::string base(name);
  hipDeviceptr_t dsig = nullptr;
  size_t nsig = 0;
  u64 sig = 0;
  if (hipModuleGetGlobal(&dsig, &nsig, mod, (base + "_sig").c_str()) != hipSuccess || nsig != sizeof(u64) ||
      hipMemcpyDtoH(&sig, dsig, sizeof(u64)) != hipSuccess) {
    (void)hipGetLastError();
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object has no program signature " + base + "_sig");
  }
  if (sig != program_signature(c, p)) {
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object was assembled for another program (signature mismatch)");
  }
  hipFunction_t fn = nullptr;
  if (hipModuleGetFunction(&fn, mod, base.c_str()) != hipSuccess) {
    (void)hipGetLastError();
    hipModuleUnload(mod);
    return fail(MG_E_PROG, "code object lacks kernel " + base);
  }
  if (p->amod) hipModuleUnload(p->amod);
  p->amod = mod;
  p->afn = fn;
  return 0;
}

// The eval paths below run inside a call (the context's mu held, handles live).
// Readbacks up to this size land in the context's pinned buffer with one copy
// and are handed over with a host memcpy (a copy straight into pageable
// memory costs a staged transfer per buffer).
constexpr size_t kReadbackMax = (size_t)1 << 20;

static bool ensure_readback(Ctx* c, size_t bytes) {
  if (bytes <= c->rb_bytes) return true;
  mw::inflight_step("ensure_readback/realloc", bytes);
  if (c->h_rb) hipHostFree(c->h_rb);
  c->h_rb = nullptr;
  c->rb_bytes = 0;
  const size_t want = std::max<size_t>(bytes, (size_t)1 << 16);
  if (hipHostMalloc(&c->h_rb, want, hipHostMallocDefault) != hipSuccess) return false;
  c->rb_bytes = want;
  return true;
}

// Plan and enqueue a search of ps (the context's mu held): the launch
// records upload, the kernels, the readback of counters and d_min; P gets what
// search_complete needs.  Nothing here waits for the device.
static int search_enqueue(Ctx* c, const std::vector<std::shared_ptr<Prog>>& ps, uint64_t seed, uint64_t begin,
                          uint64_t count, uint32_t flags, mw::CallMark& mark, Pending& P) {
  const size_t nprog = ps.size();
  std::vector<const Prog*> progs(nprog);
  for (size_t i = 0; i < nprog; ++i) progs[i] = ps[i].get();
  mark.step("plan", nprog);
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->dev));
  (void)hipGetLastError();  // start from a clean error state: launch errors are read back below
  int rc = 0;
  // Programs with a specialised kernel (mg_prog_attach_kernel) get one launch
  // each; the rest share interpreter launches (grid row per program): one of
  // the threaded-dispatch asm interpreter for the programs it handles, one of
  // the compiled interpreter for the others.  d_min holds the asm group, then
  // the compiled group, then the specialised programs.
  // Programs with an assembled kernel (mg_prog_attach_asm) get one launch each
  // on the asm interpreter's records, after the interpreter groups.
  std::vector<size_t> gasm, gcpp, gasb, special;
  u64 ops = 0;
  const bool use_asm = asm_enabled();
  for (size_t i = 0; i < nprog; ++i) {
    u32 n1 = 0;
    if (progs[i]->jit_ready()) special.push_back(i);
    else if (use_asm && progs[i]->afn && count < (1ull << 40) &&
             asm_lds_fit(progs[i]->dev.n_spill, progs[i]->dev.npool, &n1))
      gasb.push_back(i);
    else (use_asm && progs[i]->asm_ok ? gasm : gcpp).push_back(i);
    ops += progs[i]->ops_per_eval;
  }
  // the asm groups need their pools staged in LDS (programs whose pool does not
  // fit run on the compiled interpreter); one group per register layout
  // (kAsmKernel: the wide, narrow and quarter kernels)
  std::vector<size_t> glay[kAsmLayouts];
  u32 lay_nlds[kAsmLayouts] = {0, 0, 0};
  {
    u32 ms[kAsmLayouts] = {0, 0, 0}, mp[kAsmLayouts] = {0, 0, 0};
    for (size_t i : gasm) {
      u32 n1 = 0;
      const u8 L = progs[i]->asm_layout;
      if (count < (1ull << 40) && asm_lds_fit(progs[i], &n1)) {
        glay[L].push_back(i);
        ms[L] = std::max(ms[L], progs[i]->dev.n_spill);
        mp[L] = std::max(mp[L], progs[i]->dev.npool);
      } else {
        gcpp.push_back(i);
      }
    }
    for (int L = 0; L < kAsmLayouts; ++L)
      if (!glay[L].empty()) (void)asm_lds_fit(ms[L], mp[L], &lay_nlds[L], (u8)L, true);
  }
  std::vector<size_t> interp;
  for (int L = 0; L < kAsmLayouts; ++L) interp.insert(interp.end(), glay[L].begin(), glay[L].end());
  const size_t nasm = interp.size();
  interp.insert(interp.end(), gcpp.begin(), gcpp.end());
  const size_t ni = interp.size();
  interp.insert(interp.end(), gasb.begin(), gasb.end());   // d_progs / d_min: then the assembled ones
  const size_t nia = interp.size();
  std::vector<ProgDev> hp;
  for (size_t j = 0; j < nia; ++j)   // the asm groups read the predecoded code
    hp.push_back(j < nasm ? progs[interp[j]]->adev : progs[interp[j]]->dev);
  const u64 nchunks = (count + kBlock - 1) / kBlock;
  struct Group {
    size_t first, n;
    u64 gx;
    u32 nlds, max_pool;
  } groups[kAsmLayouts + 1];   // the asm layouts' groups, then the compiled interpreter's
  {
    size_t first = 0;
    for (int L = 0; L < kAsmLayouts; ++L) {
      groups[L] = {first, glay[L].size(), 1, 0, 0};
      first += glay[L].size();
    }
    groups[kAsmLayouts] = {nasm, gcpp.size(), 1, 0, 0};
  }
  size_t spill_need = 4;
  for (int gi = 0; gi <= kAsmLayouts; ++gi) {
    Group& G = groups[gi];
    if (!G.n) continue;
    u32 max_spill = 0;
    for (size_t j = G.first; j < G.first + G.n; ++j) {
      max_spill = std::max(max_spill, hp[j].n_spill);
      G.max_pool = std::max(G.max_pool, hp[j].npool);
    }
    // enough blocks to fill the chip several times over, split across programs
    G.gx = std::max<u64>(1, (u64)c->ncu * 8 / G.n);
    G.gx = std::min<u64>(G.gx, nchunks);
    u64 nthreads = G.gx * G.n * kBlock;
    if (gi < kAsmLayouts) {
      // the asm groups: one 1D grid, blocks in proportion to each program's
      // instructions (its cost per candidate), at least one, at most its chunks
      double wsum = 0;
      for (size_t j = G.first; j < G.first + G.n; ++j) wsum += std::max<u32>(1, hp[j].n_insn);
      const double B = (double)std::max<u64>(G.n, (u64)c->ncu * 8);
      u64 at = 0;
      for (size_t j = G.first; j < G.first + G.n; ++j) {
        const u64 b = std::min<u64>(nchunks, std::max<u64>(1, (u64)(B * std::max<u32>(1, hp[j].n_insn) / wsum)));
        hp[j].first_block = (u32)at;
        at += b;
      }
      G.gx = at;   // the whole grid
      nthreads = G.gx * kBlock;
    }
    G.nlds = gi < kAsmLayouts ? lay_nlds[gi] : std::min(max_spill, kLdsSpillWords);
    spill_need = std::max(spill_need, (size_t)(max_spill - G.nlds) * nthreads * sizeof(u32));
  }
  // assembled kernels: records kAsmLayouts.. (one program, the whole chip each)
  const u64 agx = std::min<u64>((u64)c->ncu * 8, nchunks);
  std::vector<AsmArgs> ha(kAsmLayouts + gasb.size());   // the layouts' groups, then the assembled kernels
  for (size_t k = 0; k < gasb.size(); ++k) {
    const ProgDev& d = hp[ni + k];
    AsmArgs& r = ha[kAsmLayouts + k];
    (void)asm_lds_fit(d.n_spill, d.npool, &r.nlds);
    r.seed = seed;
    r.begin = begin;
    r.end = begin + count;
    r.flags = flags;
    r.gstride = (u32)(agx * kBlock * 4);
    r.nchunks = (u32)nchunks;
    r.gdx = (u32)agx;
    r.verdict = nullptr;
    spill_need = std::max(spill_need, (size_t)(d.n_spill - r.nlds) * agx * kBlock * sizeof(u32));
  }
  const bool need_args = nasm || !gasb.empty();
  mark.step("buffers", nprog);
  rc = ensure_launch(c, nprog, need_args ? ha.size() : 0);
  if (rc) return rc;
  if (nia) {
    rc = ensure_spill(c, spill_need);
    if (rc) return rc;
  }
  for (size_t k = 0; k < gasb.size(); ++k) ha[kAsmLayouts + k].spillbuf = c->d_spill;
  for (int gi = 0; gi < kAsmLayouts && need_args; ++gi) {
    AsmArgs& aa = ha[gi];
    aa.seed = seed;
    aa.begin = begin;
    aa.end = begin + count;
    aa.flags = flags;
    aa.nlds = groups[gi].nlds;
    aa.gstride = (u32)(groups[gi].gx * kBlock * 4);   // a 1D grid of gx blocks (above)
    aa.nchunks = (u32)nchunks;
    aa.gdx = (u32)groups[gi].gx;
    aa.nprog = (u32)groups[gi].n;
    aa.spillbuf = c->d_spill;   // the launches run one after the other on the stream
    aa.verdict = nullptr;
  }
  // one upload: zeroed counters, d_min at MG_NONE, the ProgDev and AsmArgs records
  mark.step("enqueue", count);
  // step-time accounting: the stream's own time before the records upload
  // (a queued program upload), the upload, the kernels and the readback
  const bool gpu_steps = mw::step_times_on() && c->ea && c->eb;
  if (gpu_steps) HIPCHK(hipEventRecord(c->ea, c->stream));
  HIPCHK(stage_upload(c, nprog, hp.data(), nia, ha.data(), need_args ? ha.size() : 0));
  HIPCHK(hipEventRecord(c->e0, c->stream));
  for (int gi = 0; gi < kAsmLayouts; ++gi) {
    const Group& G = groups[gi];
    if (!G.n) continue;
    const size_t lds = (size_t)G.nlds * kBlock * 4 + (size_t)G.max_pool * 4;
    hipLaunchKernelGGL(kAsmKernel[gi], dim3((u32)G.gx, 1u), dim3(kBlock), lds, c->stream,
                       c->d_progs + G.first, (const AsmArgs*)c->d_asmargs + gi, c->d_min + G.first, c->d_counter,
                       G.nlds);
    HIPCHK(hipGetLastError());
  }
  if (groups[kAsmLayouts].n) {
    const Group& G = groups[kAsmLayouts];
    // stage the pools in LDS when they fit beside the spill words (80 KiB per
    // block keeps two blocks per CU)
    const size_t spill_bytes = (size_t)G.nlds * kBlock * 4, pool_bytes = (size_t)G.max_pool * 4;
    const ProgDev* dp = c->d_progs + G.first;
    u64* dm = c->d_min + G.first;
#ifdef MW_NO_POOL_LDS   // A/B builds only
    if (false)
#else
    if (G.max_pool && spill_bytes + pool_bytes <= (size_t)kLdsSpillWords * kBlock * 4)
#endif
      hipLaunchKernelGGL(mw_search_kernel<true>, dim3((u32)G.gx, (u32)G.n), dim3(kBlock), spill_bytes + pool_bytes,
                         c->stream, dp, seed, begin, count, flags, dm, c->d_counter, c->d_spill, G.nlds);
    else
      hipLaunchKernelGGL(mw_search_kernel<false>, dim3((u32)G.gx, (u32)G.n), dim3(kBlock), spill_bytes,
                         c->stream, dp, seed, begin, count, flags, dm, c->d_counter, c->d_spill, G.nlds);
    HIPCHK(hipGetLastError());
  }
  for (size_t k = 0; k < gasb.size(); ++k) {
    rc = launch_assembled(c, progs[gasb[k]], (u32)agx, c->d_progs + ni + k, c->d_asmargs + kAsmLayouts + k,
                          c->d_min + ni + k, ha[kAsmLayouts + k].nlds);
    if (rc) return rc;
  }
  for (size_t j = 0; j < special.size(); ++j) {
    rc = launch_jit(c, progs[special[j]], seed, begin, count, flags, c->d_min + nia + j, nullptr);
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(c->e1, c->stream));
  HIPCHK(stage_readback(c, nprog));   // counters and d_min, one copy
  if (gpu_steps) HIPCHK(hipEventRecord(c->eb, c->stream));
  P.ps = ps;
  P.interp = interp;
  P.special = special;
  P.nia = nia;
  P.slot.assign(nprog, 0);
  for (size_t j = 0; j < nia; ++j) P.slot[interp[j]] = j;
  for (size_t j = 0; j < special.size(); ++j) P.slot[special[j]] = nia + j;
  P.count = count;
  P.seed = seed;
  P.ops = ops;
  P.flags = flags;
  P.nlaunches = gasb.size() + special.size();
  for (const Group& G : groups) P.nlaunches += G.n ? 1 : 0;
  P.t0 = t0;
  P.gpu_steps = gpu_steps;
  return 0;
}

// Wait for a search enqueued by search_enqueue (and anything queued after it)
// and read its results (the context's mu held).
static int search_complete(Ctx* c, Pending& P, uint64_t* out_min_idx, mg_stats* st, mw::CallMark& mark) {
  const u64 count = P.count;
  mark.step("sync", count);
  HIPCHK(hipStreamSynchronize(c->stream));
  c->uploads_landed();   // the stream drained: a queued program upload has landed
  if (P.gpu_steps) {
    float a = 0.f, k = 0.f, b = 0.f;
    if (hipEventElapsedTime(&a, c->ea, c->e0) == hipSuccess && hipEventElapsedTime(&k, c->e0, c->e1) == hipSuccess &&
        hipEventElapsedTime(&b, c->e1, c->eb) == hipSuccess) {
      mw::step_times_add("mg_search", "gpu: records upload", a);
      mw::step_times_add("mg_search", "gpu: kernels", k);
      mw::step_times_add("mg_search", "gpu: readback", b);
    }
    float u = 0.f;
    if (c->eu_live && hipEventElapsedTime(&u, c->eu, c->ea) == hipSuccess)
      mw::step_times_add("mg_search", "gpu: queued program uploads", u);
  }
  c->eu_live = false;
  const u64* stripes = (const u64*)c->h_blk;
  const u64* mins = (const u64*)(c->h_blk + c->off_min);
  u64 ctr[kNCounters] = {0, 0, 0, 0, 0};
  for (size_t sidx = 0; sidx <= MW_CTR_STRIPES; ++sidx)
    for (int k = 0; k < kNCounters; ++k) ctr[k] += stripes[sidx * MW_CTR_STRIPE_WORDS + k];
  // specialised launches under MW_FLAG_NO_COUNT counted nothing: every
  // candidate of the range was evaluated (no stop-after-hit)
  const u64 evals = ctr[0] + ((P.flags & MW_FLAG_NO_COUNT) ? P.count * P.special.size() : 0u);
  for (size_t j = 0; j < P.nia; ++j) out_min_idx[P.interp[j]] = mins[j];
  for (size_t j = 0; j < P.special.size(); ++j) out_min_idx[P.special[j]] = mins[P.nia + j];
  if (st) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
    st->kernel_ms = ms;
    st->wall_ms = now_ms() - P.t0;
    st->evals = evals;  // summed over every program's blocks
    st->launches = P.nlaunches;
    st->ops = (double)evals / (double)P.ps.size() * (double)P.ops;
    st->lane_div_steps = ctr[1];
    st->lane_div_full = ctr[2];
    st->lane_div_short = ctr[3];
    st->lane_div_general = ctr[4];
  }
  return 0;
}

int mg_search(mg_ctx* h, mg_prog* const* hprogs, size_t nprog, uint64_t seed, uint64_t begin,
              uint64_t count, uint32_t flags, uint64_t* out_min_idx, mg_stats* st) {
  if (!h || !hprogs || !out_min_idx || nprog == 0) return fail(MG_E_ARG, "null argument");
  if (nprog > 65535) return fail(MG_E_ARG, "too many programs per launch");
  if (count == 0 || begin + count < begin) return fail(MG_E_ARG, "bad candidate range");
  if (flags & MW_FLAG_STOP_AFTER_HIT) flags &= ~MW_FLAG_NO_COUNT;   // blocks may skip: only the counters know
  std::vector<u64> ids(nprog);
  for (size_t i = 0; i < nprog; ++i) ids[i] = hid(hprogs[i]);
  mw::CallMark mark("mg_search");
  mark.step("lock", nprog);
  CallG call;   // resolved, reference-held and locked for the whole call (mw_handles.h)
  if (const char* why = mw::enter(g_reg, hid(h), ids.data(), nprog, call)) return fail(MG_E_ARG, std::string("mg_search: ") + why);
  Ctx* c = call.c.get();
  if (c->pending.active) return fail(MG_E_ARG, "mg_search: a search begun with mg_search_begin is pending");
  Pending P;
  int rc = search_enqueue(c, call.ps, seed, begin, count, flags, mark, P);
  if (rc) return rc;
  return search_complete(c, P, out_min_idx, st, mark);
}

int mg_search_begin(mg_ctx* h, mg_prog* const* hprogs, size_t nprog, uint64_t seed, uint64_t begin,
                    uint64_t count, uint32_t flags) {
  if (!h || !hprogs || nprog == 0) return fail(MG_E_ARG, "null argument");
  if (nprog > 65535) return fail(MG_E_ARG, "too many programs per launch");
  if (count == 0 || begin + count < begin) return fail(MG_E_ARG, "bad candidate range");
  if (flags & MW_FLAG_STOP_AFTER_HIT) flags &= ~MW_FLAG_NO_COUNT;
  std::vector<u64> ids(nprog);
  for (size_t i = 0; i < nprog; ++i) ids[i] = hid(hprogs[i]);
  mw::CallMark mark("mg_search_begin");
  mark.step("lock", nprog);
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), ids.data(), nprog, call))
    return fail(MG_E_ARG, std::string("mg_search_begin: ") + why);
  Ctx* c = call.c.get();
  if (c->pending.active) return fail(MG_E_ARG, "mg_search_begin: a search begun earlier is pending");
  Pending P;
  int rc = search_enqueue(c, call.ps, seed, begin, count, flags, mark, P);
  if (rc) {
    hipStreamSynchronize(c->stream);
    return rc;
  }
  P.active = true;
  c->pending = std::move(P);
  return 0;
}

// The witness evaluations of mg_search_end: each witness program is uploaded,
// its index patched in on the device from the search's d_min word, and
// evaluated for that one candidate on the asm interpreter, queued after the
// search; traced[i] = 1 for the programs whose trace will be read back.
struct WitPlan {
  std::vector<std::shared_ptr<Prog>> wps;
  std::vector<size_t> prog_of, trace_off;   // per witness record: its search program, its trace rows' offset
  size_t rb_bytes = 0, verd_off = 0;
};

static int witness_enqueue(Ctx* c, const std::shared_ptr<Ctx>& cref, Pending& P, const mg_prog_desc* const* wd,
                           int32_t* traced, WitPlan& W, std::unique_ptr<Scratch>& blk, mw::CallMark& mark) {
  const size_t nprog = P.ps.size();
  mark.step("witness loads", nprog);
  for (size_t i = 0; i < nprog; ++i) {
    traced[i] = 0;
    if (!wd[i]) continue;
    int rc = mg_validate_desc(wd[i]);
    if (rc) return rc;
    if (!wd[i]->n_trace_rows) continue;
    std::shared_ptr<Prog> wp;
    rc = load_locked(cref, wd[i], wp);
    if (rc) return rc;
    u32 nlds = 0;
    if (!wp->asm_ok || !asm_enabled() || !asm_lds_fit(wp.get(), &nlds)) {   // the caller evaluates it later
      release_prog(*wp);
      continue;
    }
    W.wps.push_back(std::move(wp));
    W.prog_of.push_back(i);
  }
  const size_t nw = W.wps.size();
  if (!nw) return 0;
  // device block: slots | ProgDev records | AsmArgs records | counter sink |
  // verdicts | trace rows
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_prog = up(nw * 4), o_args = up(o_prog + nw * sizeof(ProgDev)),
               o_ctr = up(o_args + nw * sizeof(AsmArgs)), o_verd = up(o_ctr + 8 * sizeof(u64));
  size_t rows = 0;
  for (auto& wp : W.wps) {
    W.trace_off.push_back(rows);
    rows += wp->desc.n_trace_rows;
  }
  const size_t o_tr = o_verd + nw * 4, total = o_tr + rows * 4, head = o_ctr;
  W.verd_off = o_verd;
  W.rb_bytes = total - o_verd;
  if (W.rb_bytes > kReadbackMax || !ensure_readback(c, W.rb_bytes)) {   // too big to read back in one copy
    for (auto& wp : W.wps) release_prog(*wp);
    W.wps.clear();
    return 0;
  }
  size_t spill = 4;
  for (auto& wp : W.wps) {
    u32 nlds = 0;
    (void)asm_lds_fit(wp.get(), &nlds);
    spill = std::max(spill, (size_t)(wp->dev.n_spill - nlds) * kBlock * sizeof(u32));
  }
  int rc = ensure_spill(c, spill);   // (a regrow frees the old buffer: hipFree waits for the search)
  if (rc) return rc;
  blk.reset(new Scratch(c, total));
  if (!blk->p) return fail(MG_E_NOMEM, "witness evaluation buffer");
  uint8_t* d = (uint8_t*)blk->p;
  if (head > c->wit_bytes) {
    if (c->h_wit) hipHostFree(c->h_wit);
    c->h_wit = nullptr;
    c->wit_bytes = 0;
    if (hipHostMalloc(&c->h_wit, std::max<size_t>(head, 4096), hipHostMallocDefault) != hipSuccess)
      return fail(MG_E_NOMEM, "witness staging allocation failed");
    c->wit_bytes = std::max<size_t>(head, 4096);
  }
  uint8_t* hw = c->h_wit;
  std::memset(hw, 0, head);
  u32* hslot = (u32*)hw;
  ProgDev* hprog = (ProgDev*)(hw + o_prog);
  AsmArgs* hargs = (AsmArgs*)(hw + o_args);
  for (size_t k = 0; k < nw; ++k) {
    const Prog* wp = W.wps[k].get();
    hslot[k] = (u32)P.slot[W.prog_of[k]];
    hprog[k] = wp->adev;
    AsmArgs& a = hargs[k];
    a.seed = 0;   // set below: the search's seed
    a.begin = 0;
    a.end = 1;    // patched on the device (mw_witness_index_kernel)
    a.flags = 0;
    (void)asm_lds_fit(wp, &a.nlds);
    a.gstride = kBlock * 4;
    a.nchunks = 1;
    a.gdx = 1;
    a.nprog = 0;
    a.spillbuf = c->d_spill;
    a.verdict = (u32*)(d + o_verd) + k;
    a.trace = (u32*)(d + o_tr) + W.trace_off[k];
    a.ncand = 1;
  }
  for (size_t k = 0; k < nw; ++k) hargs[k].seed = P.seed;
  mark.step("witness enqueue", nw);
  HIPCHK(hipMemcpyAsync(d, hw, head, hipMemcpyHostToDevice, c->stream));
  for (size_t k = 0; k < nw; ++k)
    if (!W.wps[k]->trace_full)
      HIPCHK(hipMemsetAsync(d + o_tr + W.trace_off[k] * 4, 0, W.wps[k]->desc.n_trace_rows * 4, c->stream));
  hipLaunchKernelGGL(mw_witness_index_kernel, dim3((u32)((nw + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                     (const u64*)c->d_min, (const u32*)d, (AsmArgs*)(d + o_args), (u32)nw);
  HIPCHK(hipGetLastError());
  for (size_t k = 0; k < nw; ++k) {
    const Prog* wp = W.wps[k].get();
    const u32 nlds = hargs[k].nlds;
    const size_t lds = (size_t)nlds * kBlock * 4 + (size_t)wp->dev.npool * 4;
    hipLaunchKernelGGL(kAsmKernel[wp->asm_layout], dim3(1u, 1u), dim3(kBlock), lds, c->stream,
                       (const ProgDev*)(d + o_prog) + k, (const AsmArgs*)(d + o_args) + k,
                       (u64*)(d + o_ctr) + 1, (u64*)(d + o_ctr), nlds);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpyAsync(c->h_rb, d + o_verd, W.rb_bytes, hipMemcpyDeviceToHost, c->stream));
  for (size_t k = 0; k < nw; ++k) traced[W.prog_of[k]] = 1;
  return 0;
}

int mg_search_end(mg_ctx* h, uint64_t* out_min_idx, mg_stats* st, const mg_prog_desc* const* witness,
                  uint32_t* const* out_trace, int32_t* traced) {
  if (!h || !out_min_idx) return fail(MG_E_ARG, "null argument");
  if (witness && (!out_trace || !traced)) return fail(MG_E_ARG, "witness programs need out_trace and traced");
  mw::CallMark mark("mg_search_end");
  mark.step("lock");
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), nullptr, 0, call)) return fail(MG_E_ARG, std::string("mg_search_end: ") + why);
  Ctx* c = call.c.get();
  if (!c->pending.active) return fail(MG_E_ARG, "mg_search_end: no search begun on this context");
  Pending P = std::move(c->pending);
  c->pending = Pending();
  HIPCHK(hipSetDevice(c->dev));
  WitPlan W;
  std::unique_ptr<Scratch> blk;
  int rc = 0;
  if (witness) rc = witness_enqueue(c, call.c, P, witness, traced, W, blk, mark);
  if (rc) {
    hipStreamSynchronize(c->stream);
    for (auto& wp : W.wps) release_prog(*wp);
    return rc;
  }
  rc = search_complete(c, P, out_min_idx, st, mark);   // one synchronisation for the search and the witnesses
  if (blk) blk->synced = rc == 0;
  if (rc == 0) {
    for (size_t k = 0; k < W.wps.size(); ++k) {
      const size_t i = W.prog_of[k];
      if (out_min_idx[i] == MG_NONE) {
        traced[i] = 0;
        continue;
      }
      // h_rb: the verdicts (one word per witness), then the trace rows
      std::memcpy(out_trace[i], c->h_rb + W.wps.size() * 4 + W.trace_off[k] * 4, W.wps[k]->desc.n_trace_rows * 4);
    }
  }
  for (auto& wp : W.wps) release_prog(*wp);
  return rc;
}

static int eval_common(Ctx* c, const Prog* p, const uint32_t* leaves_soa, size_t ncand, uint64_t seed,
                       uint64_t begin, uint32_t* verdict, uint32_t* trace) {
  if (!verdict || ncand == 0) return fail(MG_E_ARG, "null argument");
  HIPCHK(hipSetDevice(c->dev));
  (void)hipGetLastError();  // clean error state before the launch below
  const u64 nchunks = (ncand + kBlock - 1) / kBlock;
  const u64 gx = std::min<u64>(nchunks, (u64)c->ncu * 8);
  const u64 nthreads = gx * kBlock;
  const u32 nlds = std::min(p->dev.n_spill, kLdsSpillWords);
  int rc = ensure_spill(c, std::max<size_t>(4, (size_t)(p->dev.n_spill - nlds) * nthreads * sizeof(u32)));
  if (rc) return rc;
  const size_t nin = leaves_soa ? (size_t)p->desc.n_input_rows * ncand : 0;
  const size_t ntr = trace ? (size_t)p->desc.n_trace_rows * ncand : 0;
  // verdicts and trace rows in one device block: one readback
  const size_t vb = ncand * 4, tb = ntr * 4;
  Scratch s_in(c, nin * 4), s_vt(c, vb + tb);
  if ((nin && !s_in.p) || !s_vt.p) return fail(MG_E_NOMEM, "eval buffers");
  u32 *d_in = s_in.u(), *d_v = s_vt.u(), *d_t = ntr ? d_v + ncand : nullptr;
  if (nin && hipMemcpyAsync(d_in, leaves_soa, nin * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return fail(MG_E_HIP, "eval input copy");
  if (ntr && !p->trace_full) hipMemsetAsync(d_t, 0, tb, c->stream);
  hipLaunchKernelGGL(mw_eval_kernel, dim3((u32)gx), dim3(kBlock), (size_t)nlds * kBlock * 4, c->stream,
                     p->dev, (const u32*)d_in, (u64)ncand, seed, begin, d_v, d_t, c->d_spill, nlds);
  hipError_t e = hipGetLastError();
  const bool pinned = vb + tb <= kReadbackMax && ensure_readback(c, vb + tb);
  if (e == hipSuccess && pinned) {
    e = hipMemcpyAsync(c->h_rb, d_v, vb + tb, hipMemcpyDeviceToHost, c->stream);
  } else {
    if (e == hipSuccess) e = hipMemcpyAsync(verdict, d_v, vb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && ntr) e = hipMemcpyAsync(trace, d_t, tb, hipMemcpyDeviceToHost, c->stream);
  }
  mw::inflight_step("eval/sync", ncand);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  s_in.synced = s_vt.synced = e == hipSuccess;
  if (e != hipSuccess) return fail(MG_E_HIP, std::string("eval: ") + hipGetErrorString(e));
  c->uploads_landed();   // the stream drained: a queued program upload has landed
  if (pinned) {
    std::memcpy(verdict, c->h_rb, vb);
    if (ntr) std::memcpy(trace, c->h_rb + vb, tb);
  }
  return 0;
}

int mg_eval(mg_ctx* h, const mg_prog* hp, const uint32_t* leaves_soa, size_t ncand, uint32_t* verdict,
            uint32_t* trace) {
  if (!h || !hp) return fail(MG_E_ARG, "null argument");
  const u64 id = hid(hp);
  mw::CallMark mark("mg_eval");
  mark.step("lock", ncand);
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), &id, 1, call)) return fail(MG_E_ARG, std::string("mg_eval: ") + why);
  if (call.c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  mark.step("eval", ncand);
  const Prog* p = call.ps[0].get();
  if (p->desc.nleaves && p->desc.n_input_rows && !leaves_soa) return fail(MG_E_ARG, "leaves_soa required");
  if (p->desc.nleaves && !p->desc.n_input_rows) return fail(MG_E_ARG, "program has no input rows");
  static const u32 dummy = 0;
  return eval_common(call.c.get(), p, leaves_soa ? leaves_soa : (p->desc.nleaves ? nullptr : &dummy), ncand, 0, 0,
                     verdict, trace);
}

// Verdicts (and trace rows) of generated candidates on the asm interpreter
// (mw_search_asm_kernel with a verdict array; STORE_W / STORE_N write row r of
// candidate cand at trace[r * count + cand - begin], mw_eval_kernel's layout);
// 1 = not applicable (the caller uses mw_eval_kernel).
static int eval_asm(Ctx* c, const Prog* p, uint64_t seed, uint64_t begin, size_t count, uint32_t* verdict,
                    uint32_t* trace) {
  if (!asm_enabled() || !p->asm_ok || begin + count < begin || count >= (1ull << 40)) return 1;
  const size_t ntr = trace ? (size_t)p->desc.n_trace_rows * count : 0;
  // trace offsets are 32-bit byte offsets in the kernel (asmgen.py store_rows)
  if (trace && (count >= (1ull << 32) || ntr * 4 >= (1ull << 31))) return 1;
  const bool assembled = p->afn != nullptr && !trace;   // its assembled kernel, else the asm interpreter
  u32 nlds = 0;
  if (!(assembled ? asm_lds_fit(p->dev.n_spill, p->dev.npool, &nlds) : asm_lds_fit(p, &nlds))) return 1;
  const size_t lds = (size_t)nlds * kBlock * 4 + (size_t)p->dev.npool * 4;
  HIPCHK(hipSetDevice(c->dev));
  (void)hipGetLastError();
  int rc = ensure_launch(c, 1, 1);
  if (rc) return rc;
  const u64 nchunks = (count + kBlock - 1) / kBlock;
  const u64 gx = std::min<u64>(nchunks, (u64)c->ncu * 8);
  rc = ensure_spill(c, std::max<size_t>(4, (size_t)(p->dev.n_spill - nlds) * gx * kBlock * sizeof(u32)));
  if (rc) return rc;
  // verdicts and trace rows in one device block: one readback
  const size_t vb = count * 4, tb = ntr * 4;
  Scratch s_v(c, vb + tb);
  if (!s_v.p) return fail(MG_E_NOMEM, "eval verdict alloc");
  u32 *d_v = s_v.u(), *d_t = ntr ? d_v + count : nullptr;
  AsmArgs aa{};
  aa.seed = seed;
  aa.begin = begin;
  aa.end = begin + count;
  aa.flags = 0;
  aa.nlds = nlds;
  aa.gstride = (u32)(gx * kBlock * 4);
  aa.nchunks = (u32)nchunks;
  aa.gdx = (u32)gx;
  aa.spillbuf = c->d_spill;
  aa.verdict = d_v;
  aa.trace = d_t;
  aa.ncand = (u32)count;
  hipError_t e = ntr && !p->trace_full ? hipMemsetAsync(d_t, 0, tb, c->stream) : hipSuccess;
  if (e == hipSuccess) e = stage_upload(c, 1, assembled ? &p->dev : &p->adev, 1, &aa, 1);
  if (e == hipSuccess && assembled) {
    if (launch_assembled(c, p, (u32)gx, c->d_progs, c->d_asmargs, c->d_min, nlds)) return MG_E_HIP;
  } else if (e == hipSuccess) {
    hipLaunchKernelGGL(kAsmKernel[p->asm_layout], dim3((u32)gx, 1u), dim3(kBlock), lds, c->stream, c->d_progs,
                       (const AsmArgs*)c->d_asmargs, c->d_min, c->d_counter, nlds);
    e = hipGetLastError();
  }
  const bool pinned = vb + tb <= kReadbackMax && ensure_readback(c, vb + tb);
  if (e == hipSuccess && pinned) {
    e = hipMemcpyAsync(c->h_rb, d_v, vb + tb, hipMemcpyDeviceToHost, c->stream);
  } else {
    if (e == hipSuccess) e = hipMemcpyAsync(verdict, d_v, vb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && ntr) e = hipMemcpyAsync(trace, d_t, tb, hipMemcpyDeviceToHost, c->stream);
  }
  mw::inflight_step("eval_asm/sync", count);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  s_v.synced = e == hipSuccess;
  if (e != hipSuccess)
    return fail(MG_E_HIP, std::string(assembled ? "eval (assembled kernel): " : "eval (asm interpreter): ") +
                              hipGetErrorString(e));
  c->uploads_landed();   // the stream drained: a queued program upload has landed
  if (pinned) {
    std::memcpy(verdict, c->h_rb, vb);
    if (ntr) std::memcpy(trace, c->h_rb + vb, tb);
  }
  return 0;
}

int mg_eval_generated(mg_ctx* h, const mg_prog* hp, uint64_t seed, uint64_t begin, size_t count,
                      uint32_t* verdict, uint32_t* trace) {
  if (!h || !hp) return fail(MG_E_ARG, "null argument");
  const u64 id = hid(hp);
  mw::CallMark mark("mg_eval_generated");
  mark.step("lock", count);
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), &id, 1, call))
    return fail(MG_E_ARG, std::string("mg_eval_generated: ") + why);
  if (call.c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  mark.step("eval", count);
  Ctx* c = call.c.get();
  const Prog* p = call.ps[0].get();
  if (!p->jit_ready() && verdict && count) {
    const int rc = eval_asm(c, p, seed, begin, count, verdict, trace);
    if (rc != 1) return rc;
  }
  if (!p->jit_ready() || trace) return eval_common(c, p, nullptr, count, seed, begin, verdict, trace);
  // verdicts only, on the program's specialised kernel
  if (!verdict || count == 0 || begin + count < begin) return fail(MG_E_ARG, "bad argument");
  HIPCHK(hipSetDevice(c->dev));
  int rc = ensure_launch(c, 1, 0);
  if (rc) return rc;
  Scratch s_v(c, count * 4);
  if (!s_v.p) return fail(MG_E_NOMEM, "eval verdict alloc");
  u32* d_v = s_v.u();
  hipError_t e = stage_upload(c, 1, nullptr, 0, nullptr, 0);
  if (e == hipSuccess) {
    rc = launch_jit(c, p, seed, begin, count, 0u, c->d_min, d_v);
    if (rc) return rc;
    e = hipMemcpyAsync(verdict, d_v, count * 4, hipMemcpyDeviceToHost, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  s_v.synced = e == hipSuccess;
  if (e != hipSuccess) return fail(MG_E_HIP, std::string("eval (specialised): ") + hipGetErrorString(e));
  return 0;
}

// One-shot evaluation of a program that is not kept (a witness program:
// engine.WitnessEngine._materialize_traced): upload, evaluation and release
// in one call under one lock, the upload's buffer back to the pool after the
// evaluation's synchronisation.  Same results as mg_prog_load +
// mg_eval_generated + mg_prog_free.
int mg_eval_program(mg_ctx* h, const mg_prog_desc* d, uint64_t seed, uint64_t begin, size_t count, uint32_t* verdict,
                    uint32_t* trace) {
  if (!h || !d || !verdict || count == 0) return fail(MG_E_ARG, "null argument");
  mw::CallMark mark("mg_eval_program");
  std::shared_ptr<Ctx> cref = g_reg.ctx(hid(h));
  if (!cref) return fail(MG_E_ARG, "mg_eval_program: not a live context");
  mark.step("validate", d->ncode_words);
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  Ctx* c = cref.get();
  mark.step("lock");
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->dead) return fail(MG_E_ARG, "mg_eval_program: the context was freed during the call");
  if (c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  HIPCHK(hipSetDevice(c->dev));
  std::shared_ptr<Prog> p;
  rc = load_locked(cref, d, p);
  if (rc) return rc;
  mark.step("eval", count);
  rc = eval_asm(c, p.get(), seed, begin, count, verdict, trace);
  if (rc == 1) rc = eval_common(c, p.get(), nullptr, count, seed, begin, verdict, trace);
  if (rc != 0) hipStreamSynchronize(c->stream);   // a failed launch: nothing may still read the buffer
  mark.step("release");
  release_prog(*p);
  p->dead = true;
  return rc;
}

int mg_witness_leaves(mg_ctx* h, const mg_prog* hp, uint64_t seed, uint64_t index, uint32_t* out) {
  if (!h || !hp || !out) return fail(MG_E_ARG, "null argument");
  const u64 id = hid(hp);
  mw::CallMark mark("mg_witness_leaves");
  mark.step("lock");
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), &id, 1, call))
    return fail(MG_E_ARG, std::string("mg_witness_leaves: ") + why);
  if (call.c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  mark.step("launch + sync");
  Ctx* c = call.c.get();
  const Prog* p = call.ps[0].get();
  const u32 nl = (u32)p->desc.nleaves;
  if (nl == 0) return 0;
  HIPCHK(hipSetDevice(c->dev));
  (void)hipGetLastError();
  Scratch s_d(c, (size_t)nl * 8 * sizeof(u32));
  if (!s_d.p) return fail(MG_E_NOMEM, "witness leaf buffer");
  u32* d = s_d.u();
  hipLaunchKernelGGL(mw_leaf_kernel, dim3((nl + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, p->dev.leaves,
                     p->dev.pool, nl, seed, index, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, (size_t)nl * 8 * sizeof(u32), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  s_d.synced = e == hipSuccess;
  if (e != hipSuccess) return fail(MG_E_HIP, std::string("witness leaves: ") + hipGetErrorString(e));
  return 0;
}

int mg_valu_peak(mg_ctx* h, uint32_t mul, double* ops_per_s, double* kernel_ms) {
  if (!h || !ops_per_s) return fail(MG_E_ARG, "null argument");
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), nullptr, 0, call)) return fail(MG_E_ARG, std::string("mg_valu_peak: ") + why);
  if (call.c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  Ctx* c = call.c.get();
  HIPCHK(hipSetDevice(c->dev));
  const u32 blocks = (u32)c->ncu * 8, iters = 4096;
  u32* d = nullptr;
  HIPCHK(hipMalloc(&d, (size_t)blocks * kBlock * 4));
  hipLaunchKernelGGL(mw_valu_peak_kernel, dim3(blocks), dim3(kBlock), 0, c->stream, d, 16u, mul);  // warm
  HIPCHK(hipEventRecord(c->e0, c->stream));
  hipLaunchKernelGGL(mw_valu_peak_kernel, dim3(blocks), dim3(kBlock), 0, c->stream, d, iters, mul);
  HIPCHK(hipEventRecord(c->e1, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
  hipFree(d);
  *ops_per_s = (double)blocks * kBlock * iters * 32.0 / (ms * 1e-3);
  if (kernel_ms) *kernel_ms = ms;
  return 0;
}

int mg_keccak256_device(mg_ctx* h, const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                        uint8_t* d_out32, mg_stats* st) {
  if (!h || (!n)) return fail(MG_E_ARG, "bad argument");
  mw::CallMark mark("mg_keccak256_device");
  mark.step("lock", n);
  CallG call;
  if (const char* why = mw::enter(g_reg, hid(h), nullptr, 0, call)) return fail(MG_E_ARG, std::string("mg_keccak256: ") + why);
  if (call.c->pending.active) return fail(MG_E_ARG, "a search begun with mg_search_begin is pending on this context");
  Ctx* c = call.c.get();
  HIPCHK(hipSetDevice(c->dev));
  const double t0 = now_ms();
  const u64 gx = std::min<u64>((n + kBlock - 1) / kBlock, (u64)c->ncu * 16);
  HIPCHK(hipEventRecord(c->e0, c->stream));
  hipLaunchKernelGGL(mw_keccak_kernel, dim3((u32)gx), dim3(kBlock), 0, c->stream, d_data, (const u64*)d_off,
                     (const u32*)d_len, (u64)n, d_out32);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->e1, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (st) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
    st->kernel_ms = ms;
    st->wall_ms = now_ms() - t0;
    st->evals = n;
    st->launches = 1;
    st->ops = 0;
    st->lane_div_steps = 0;
    st->lane_div_full = st->lane_div_short = st->lane_div_general = 0;
  }
  return 0;
}

int mg_keccak256(mg_ctx* h, const uint8_t* data, size_t ndata, const uint64_t* off, const uint32_t* len, size_t n,
                 uint8_t* out32, mg_stats* st) {
  if (!h || !off || !len || !out32) return fail(MG_E_ARG, "null argument");
  mw::CallMark mark("mg_keccak256");
  mark.step("copy in", ndata);
  std::shared_ptr<Ctx> cref = g_reg.ctx(hid(h));   // its device, for the staging buffers
  if (!cref) return fail(MG_E_ARG, "mg_keccak256: not a live context");
  const Ctx* c = cref.get();
  if (n == 0) return 0;
  for (size_t i = 0; i < n; ++i)
    if (off[i] + len[i] > ndata) return fail(MG_E_ARG, "message out of range");
  HIPCHK(hipSetDevice(c->dev));
  uint8_t *dd = nullptr, *dout = nullptr;
  u64* doff = nullptr;
  u32* dlen = nullptr;
  auto cleanup = [&]() {
    if (dd) hipFree(dd);
    if (dout) hipFree(dout);
    if (doff) hipFree(doff);
    if (dlen) hipFree(dlen);
  };
  if (hipMalloc(&dd, std::max<size_t>(ndata, 1)) != hipSuccess || hipMalloc(&dout, 32 * n) != hipSuccess ||
      hipMalloc(&doff, 8 * n) != hipSuccess || hipMalloc(&dlen, 4 * n) != hipSuccess) {
    cleanup();
    return fail(MG_E_NOMEM, "keccak alloc");
  }
  hipError_t e = hipSuccess;
  if (ndata) e = hipMemcpy(dd, data, ndata, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(doff, off, 8 * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dlen, len, 4 * n, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    cleanup();
    return fail(MG_E_HIP, "keccak copy-in");
  }
  int rc = mg_keccak256_device(h, dd, doff, dlen, n, dout, st);   // the call proper (locked)
  if (rc == 0 && hipMemcpy(out32, dout, 32 * n, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(MG_E_HIP, "keccak copy-out");
  cleanup();
  return rc;
}

// The C-ABI calls in flight on every thread, one line each (mw_inflight.h):
// for a watchdog that finds a call that does not return.  Never blocks.
int mg_debug_inflight(char* buf, size_t n) { return mw::inflight_report(buf, n); }

// Wall time per call and step since the last read (MYTHRIL_AMD_STEP_TIMES=1;
// "call/step ms count" lines), then cleared; 0 lines when off.
int mg_debug_step_times(char* buf, size_t n) { return mw::step_times_report(buf, n); }

}  // extern "C"
