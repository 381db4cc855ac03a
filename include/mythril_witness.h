/* mythril_witness.h — C-ABI of the MI355X constraint-witness engine.
 *
 * Drop-in boundary.  The reference has no native FFI of its
 * own on this path: Mythril is pure Python and crosses into native code only
 * through z3-solver's and pysha3's ctypes/C-extension bindings.  Each entry
 * point below replaces one of those crossings and is bound from Python with
 * ctypes exactly the way z3's own bindings are:
 *
 *   mg_search     replaces z3 Optimize.check() for feasibility-only queries
 *                 (mythril/laser/smt/solver/solver.py:50-66, reached from
 *                  mythril/support/model.py:58 get_model)
 *   mg_eval       replaces z3 ModelRef.eval / substitute+simplify for a batch
 *                 of assignments (mythril/laser/smt/model.py:52-59)
 *   mg_keccak256  replaces _pysha3.keccak_256 (mythril/support/support_utils.py:50-59,
 *                 called by keccak_function_manager.py:57-69 find_concrete_keccak)
 *
 * Conventions: every call returns 0 on success or a negative MG_E* code; the
 * message for the calling thread is in mg_last_error().  The caller owns all
 * host buffers (copied in/out); program handles are library-owned until
 * mg_prog_free.  Nothing throws across the ABI.
 * Lifetimes and threads (mythril_amd/csrc/mw_handles.h): a handle is an opaque
 * id, never an address, and ids are never reused.  Calls on one context are
 * serialised; calls may come from any thread.  mg_free also frees every
 * program still loaded in that context, after the call in flight on it (from
 * another thread) has finished.  A handle that is not live (already freed,
 * freed with its context, never returned by the library) is refused with
 * MG_E_ARG by every entry point, also when it is freed by another thread
 * while the call waits for the context.  Programs are validated on load (slot ranges, constant offsets,
 * opcodes) so a malformed program can never be launched.
 */
#ifndef MYTHRIL_WITNESS_H
#define MYTHRIL_WITNESS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_OK 0
#define MG_E_ARG -1
#define MG_E_HIP -2
#define MG_E_PROG -3
#define MG_E_NOMEM -4

#define MG_NONE UINT64_MAX /* no witness in the searched range */

/* search flags (same values as MW_FLAG_* in mw_isa.h) */
#define MG_FLAG_EARLY_EXIT 1u
#define MG_FLAG_STOP_AFTER_HIT 2u
/* specialised kernels write no launch counters (division-path counts stay 0;
 * evals = count per program); ignored together with MG_FLAG_STOP_AFTER_HIT */
#define MG_FLAG_NO_COUNT 4u

typedef struct mg_ctx mg_ctx;
typedef struct mg_prog mg_prog;

/* A compiled constraint program (produced by mythril_amd.compiler). */
typedef struct {
  const uint32_t* code;   /* 4 words per instruction, ends with MW_END */
  size_t ncode_words;
  const uint32_t* consts; /* constant pool words */
  size_t nconst_words;
  const uint32_t* leaves; /* MW_LEAF_WORDS words per free variable */
  size_t nleaves;
  const uint32_t* pool;   /* candidate pools, MW_POOL_ENTRY_WORDS_OF(width) per entry */
  size_t npool_words;
  uint32_t n_spill;       /* spill-area words per lane (SPILL_W/FILL_W imm: 8-word slot offset, _N: 1 word) */
  uint32_t n_trace_rows;  /* rows written by MW_STORE_* (mg_eval trace) */
  uint32_t n_input_rows;  /* SoA leaf rows mg_eval reads */
  uint32_t reserved;
  uint64_t ops_per_eval;  /* algorithmic u32 ops per candidate */
} mg_prog_desc;

typedef struct {
  double kernel_ms;      /* device time of the search/eval kernels (HIP events) */
  double wall_ms;        /* host wall time of the call */
  uint64_t evals;        /* program x candidate verdicts determined */
  uint64_t launches;
  double ops;            /* algorithmic u32 ops executed (evals x ops_per_eval) */
  /* Wide divisions (mw_alu.h udivrem8) take one of three paths per wave; each
   * count is (events per wave) x (valid lanes of that wave), summed.  bench.py
   * and compiler.Program.executed_ops price the executed division work from
   * them (tests/test_gpu_fullsize.py and tests/test_divcount.py check them against oracle/c). */
  uint64_t lane_div_steps;    /* schoolbook digit positions run (some lane's digit nonzero) */
  uint64_t lane_div_full;     /* one-digit path: every lane's divisor full width */
  uint64_t lane_div_short;    /* short division: every lane's divisor one limb */
  uint64_t lane_div_general;  /* limb-aligned schoolbook entries */
} mg_stats;

int mg_device_count(int* n);
int mg_init(int device, mg_ctx** out);
int mg_free(mg_ctx* ctx);

/* Upload a program (replaces the per-query z3 model construction the
 * reference runs, mythril/support/model.py:15-63, with a device-resident
 * program).  The desc's arrays are copied before the call returns; the device
 * copy is queued on the context's stream, so every later call on the context
 * sees it, and a copy failure is reported by the next call that waits. */
int mg_prog_load(mg_ctx* ctx, const mg_prog_desc* desc, mg_prog** out);
int mg_prog_free(mg_prog* prog);

/* Search candidate indices [begin, begin+count) of every program; out_min_idx[i]
 * receives the lowest index whose assignment satisfies program i, or MG_NONE. */
int mg_search(mg_ctx* ctx, mg_prog* const* progs, size_t nprog, uint64_t seed,
              uint64_t begin, uint64_t count, uint32_t flags, uint64_t* out_min_idx,
              mg_stats* stats);

/* mg_search in two calls, so the caller can work on the host while the device
 * searches (engine.WitnessEngine compiles the witness programs meanwhile).
 * mg_search_begin validates, plans and enqueues the search and returns; until
 * mg_search_end every other call that launches work on this context is
 * refused (MG_E_ARG), and a program of the search freed meanwhile waits for it.
 * mg_search_end completes it: the same out_min_idx and stats as mg_search.
 * witness (nullable): per program, a witness program description (or NULL);
 * each is uploaded and evaluated at the index its program's search found,
 * queued after the search, read back with the same synchronisation into
 * out_trace[i] (its n_trace_rows words; traced[i] = 1), or left for the caller
 * (traced[i] = 0: no witness found, or a program the asm interpreter does not
 * run).  Replaces Optimize.check + model() of mythril/support/model.py:58-60. */
int mg_search_begin(mg_ctx* ctx, mg_prog* const* progs, size_t nprog, uint64_t seed, uint64_t begin,
                    uint64_t count, uint32_t flags);
int mg_search_end(mg_ctx* ctx, uint64_t* out_min_idx, mg_stats* stats, const mg_prog_desc* const* witness,
                  uint32_t* const* out_trace, int32_t* traced);

/* Evaluate one program on explicit assignments: leaves_soa has n_input_rows
 * rows of ncand u32 (row r, candidate i at [r*ncand + i]).  verdict[i] = 0/1;
 * trace (may be NULL) receives n_trace_rows rows of ncand u32. */
int mg_eval(mg_ctx* ctx, const mg_prog* prog, const uint32_t* leaves_soa, size_t ncand,
            uint32_t* verdict, uint32_t* trace);

/* Evaluate one program on generated candidates [begin, begin+count): the
 * verdict/trace of exactly what mg_search explores (parity tests), trace row
 * r of candidate begin+i at [r*count + i].  Programs the asm interpreter runs
 * are evaluated there, trace rows included (its STORE_W / STORE_N handlers);
 * the rest on the compiled interpreter.  The witness program's evaluation
 * behind WitnessEngine.materialize, in place of z3's model()
 * (mythril/laser/smt/solver/solver.py:68-77) for array cells and function
 * arguments. */
int mg_eval_generated(mg_ctx* ctx, const mg_prog* prog, uint64_t seed, uint64_t begin,
                      size_t count, uint32_t* verdict, uint32_t* trace);

/* The values of every leaf (free variable) of a loaded program at candidate
 * `index`: out receives nleaves x 8 u32 limbs, leaf by leaf in the program's
 * leaf-table order, as the search kernels generate them (the witness values
 * of an index mg_search returned).  Replaces z3's Optimize.model()
 * (mythril/laser/smt/solver/solver.py:68-77) for the free symbols. */
int mg_witness_leaves(mg_ctx* ctx, const mg_prog* prog, uint64_t seed, uint64_t index, uint32_t* out);

/* One-shot evaluation of a program description that is not kept: upload,
 * mg_eval_generated's evaluation of candidates [begin, begin+count) and the
 * release, in one call (a witness program read once at the found index).
 * Same validation, results and trace layout as mg_prog_load +
 * mg_eval_generated + mg_prog_free.  Replaces the reference's model
 * evaluation of the witness (z3 ModelRef.eval, mythril/support/model.py:58-60). */
int mg_eval_program(mg_ctx* ctx, const mg_prog_desc* desc, uint64_t seed, uint64_t begin, size_t count,
                    uint32_t* verdict, uint32_t* trace);

/* Attach a specialised kernel to a loaded program: `image` is a gfx950 code
 * object generated from this program's own IR by mythril_amd/jit.py (one
 * straight-line kernel per program, csrc/mw_jit.h).  It must export
 * `<name>_sig` (the program signature, checked against the loaded program:
 * a code object made for any other program is refused) and `<name>_x`
 * (exhaustive), optionally `<name>_e` (early exit).  mg_search and
 * mg_eval_generated (verdicts only) then launch it instead of the
 * interpreter; witness indices and verdicts are identical.  Same crossing as
 * mg_search (z3 Optimize.check, mythril/laser/smt/solver/solver.py:50-66). */
int mg_prog_attach_kernel(mg_prog* prog, const void* image, size_t size, const char* name);

/* Attach an assembled kernel to a loaded program: `image` is a gfx950 code
 * object that mythril_amd/asmjit.py assembled (llvm-mc + ld.lld, milliseconds)
 * from this program's own code, the asm interpreter's handlers instantiated
 * with literal operands in straight-line order (csrc/mw_asmjit_shell.hip).
 * It must export kernel `<name>` and `<name>_sig` (the program signature,
 * checked as for mg_prog_attach_kernel); the program must be one the asm
 * interpreter runs.  mg_search and mg_eval_generated (verdicts only) then
 * launch it on the asm interpreter's records; results are identical.  A
 * specialised kernel, when also attached, takes precedence.  Same crossing as
 * mg_search (z3 Optimize.check, mythril/laser/smt/solver/solver.py:50-66). */
int mg_prog_attach_asm(mg_prog* prog, const void* image, size_t size, const char* name);

/* 1 if a specialised kernel is attached to the program, else 0. */
int mg_prog_has_kernel(const mg_prog* prog);
/* The engine a search of this program runs on: 0 the compiled interpreter,
 * 1 the threaded-dispatch asm interpreter (every opcode and leaf kind has a
 * handler and the pool fits in LDS; MYTHRIL_AMD_ASM=0 disables it), 2 its
 * specialised kernel, 3 its assembled kernel.  Replaces
 * nothing in the reference: a diagnostic for tests and benchmarks. */
int mg_prog_engine(const mg_prog* prog);

/* Batched Keccak-256 (original 0x01 padding): message i is data[off[i] .. off[i]+len[i]). */
int mg_keccak256(mg_ctx* ctx, const uint8_t* data, size_t ndata, const uint64_t* off,
                 const uint32_t* len, size_t n, uint8_t* out32, mg_stats* stats);

/* Device-resident variant for benchmarking with inputs already in HBM. */
int mg_keccak256_device(mg_ctx* ctx, const uint8_t* d_data, const uint64_t* d_off,
                        const uint32_t* d_len, size_t n, uint8_t* d_out32, mg_stats* stats);

/* Diagnostic: measured INT32 VALU issue rate of the device (v_add_u32, or
 * v_mul_lo_u32 when mul != 0), u32 ops/s — the roofline peak bench.py reports. */
int mg_valu_peak(mg_ctx* ctx, uint32_t mul, double* ops_per_s, double* kernel_ms);

/* Validate a program without a device (the same check mg_prog_load runs). */
int mg_validate_desc(const mg_prog_desc* desc);

const char* mg_last_error(void);

/* Debugging (not a reference crossing): the C-ABI calls in flight on every
 * thread, one line each ("tid=... <call>/<step> arg=N call_ms=T step_ms=T"),
 * written NUL-terminated into buf (at most n bytes); returns how many calls
 * are in flight.  Lock-free: safe from a watchdog thread while another thread
 * is stuck inside a call.  A step slower than MYTHRIL_AMD_SLOW_STEP_MS
 * (default 2000) also prints one line on stderr when it ends. */
int mg_debug_inflight(char* buf, size_t n);

/* Debugging: with MYTHRIL_AMD_STEP_TIMES=1 in the environment, the wall time
 * (ms) and count of every call and step since the last read, one
 * "call/step ms count" line each (the whole call as "call/(call)"); the
 * table is then cleared.  Returns the number of lines (0 when off). */
int mg_debug_step_times(char* buf, size_t n);

#ifdef __cplusplus
}
#endif
#endif
