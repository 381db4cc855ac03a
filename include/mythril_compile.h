/* mythril_compile.h — the host compiler of the witness engine: constraint DAG
 * (after Ackermannisation and width legalisation, mythril_amd/lower.py) ->
 * interpreter bytecode, constant pool, leaf order, trace rows.
 *
 * Reference interface replaced: none directly.  This is the host half of the
 * get_model crossing (/root/reference/mythril/support/model.py:39-58): the
 * work between z3's constraint list and the device search, which the reference
 * hands to libz3's own bit-blaster.  mythril_amd/compiler.py
 * (compile_program) is the Python statement of the same passes and the parity
 * reference for this one: programs are byte-identical
 * (tests/test_native_compile.py, both corpora and random DAGs).
 *
 * The DAG arrives as one int32 record stream, nodes in operand-first order
 * (a node's operands precede it):
 *   op, width, flags, p0, p1, nargs, arg_0 .. arg_{nargs-1}
 *   op     index into MW_IR_OPS (mythril_amd/ccompile.py IR_OPS; -1: an op
 *          outside the vocabulary, compiled as Unsupported)
 *   width  bitvector width, 0 = Bool (array terms: the range width)
 *   flags  bit 0 array-sorted term, bit 1 traced (a STORE row is emitted)
 *   p0,p1  params (extract hi, lo; extension / repeat / rotate amount);
 *          const: index of its 256-bit value in `kvals` (32 little-endian
 *          bytes each); var: an id per distinct name (one leaf per name)
 *   arg_k  record index of operand k
 * roots: the conjuncts (top-level `and` already flattened, `true` dropped),
 * then the traced terms, as record indices.
 */
#ifndef MYTHRIL_COMPILE_H
#define MYTHRIL_COMPILE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mw_compiled mw_compiled;

typedef struct mw_compile_info {
  uint64_t ncode_words;     /* 4 per instruction */
  uint64_t nconst_words;
  uint64_t nleaves;         /* leaf records, in leaf-index order */
  uint64_t ntrace;          /* trace entries (3 words each: record, row, class 0=N/1=W) */
  uint64_t n_spill;         /* spill words per lane */
  uint64_t n_trace_rows;
  uint64_t ops_per_eval;    /* algorithmic u32 ops per candidate (compiler.py node_cost) */
  uint64_t div_nominal_ops;
  uint64_t n_nodes, n_div, n_spills, n_fills;
} mw_compile_info;

/* Compile one program.  Returns 0 and a result handle, or MG_E_ARG with
 * mg_last_error() = "unsupported: <reason>" when the formula is outside the
 * engine's vocabulary (the caller then answers with z3), or another MG_E_*
 * code for malformed input. */
int mw_compile(const int32_t* recs, size_t nrecs_words, size_t nnodes, const uint8_t* kvals, size_t nkvals,
               const int32_t* roots, size_t nconj, size_t ntrace, mw_compiled** out, mw_compile_info* info);

/* mw_compile with the register allocator limited to the W slots below
 * w_slots (4..8) and the N slots below n_slots (8..64): the programs of the
 * asm interpreter's smaller register layouts (mythril_amd/asmgen.py
 * variant("quarter"): 4 and 16).  MG_E_ARG for limits out of range. */
int mw_compile_slots(const int32_t* recs, size_t nrecs_words, size_t nnodes, const uint8_t* kvals, size_t nkvals,
                     const int32_t* roots, size_t nconj, size_t ntrace, uint32_t w_slots, uint32_t n_slots,
                     mw_compiled** out, mw_compile_info* info);

/* Copy the result out (buffers sized from mw_compile_info) and release it.
 * leaves: record index of each leaf's var node; trace: 3 words per entry. */
int mw_compiled_take(mw_compiled* r, uint32_t* code, uint32_t* consts, uint32_t* leaves, uint32_t* trace);

/* Release without copying (error paths). */
void mw_compiled_free(mw_compiled* r);

#ifdef __cplusplus
}
#endif
#endif
