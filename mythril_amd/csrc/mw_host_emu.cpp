// mw_host_emu.cpp — CPU build of the *same* interpreter/ALU/leaf code that runs
// on gfx950 (mw_interp.h, mw_alu.h, mw_leaf.h, mw_keccak.h), one candidate at a
// time.  TEST/DEVELOPMENT ONLY: lets tests/ check compiler + bytecode + ALU
// semantics against the oracle on a machine without a GPU, and is bench.py's
// fast CPU baseline (mwh_count_omp: the product's ALU on every host core,
// SURVEY §8(d) "build CPU restatement").  The product path (mythril_amd.runtime)
// never loads this library.
#include <omp.h>

#include <cstring>
#include <vector>

#include "../../include/mythril_witness.h"
#include "mw_interp.h"
#include "mw_keccak.h"
#include "mw_leaf.h"

using namespace mw;

namespace {
struct HostEnv {
  const u32* leaves;
  const u32* pool;
  const u32* in;  // SoA rows or null
  u32* trace;
  u64 ncand, idx, seed, cand;
  std::vector<u32>* spillv;
  DivCount dsteps;  // division paths (one candidate is one 'wave' here)
  void leaf(u32 li, u32 out[8]) {
    const u32* L = leaves + (u64)li * MW_LEAF_WORDS;
    if (in) {
      const u32 w = L[MW_LEAF_WIDTH], row = L[MW_LEAF_INROW];
      const int nl = (int)((w + 31) / 32);
      for (int k = 0; k < 8; ++k) out[k] = k < nl ? in[((u64)row + k) * ncand + idx] : 0u;
      canon(out, w);
    } else {
      leaf_value(L, pool, seed, cand, out);
    }
  }
  void store(u32 row, const u32* v, int n) {
    if (trace)
      for (int k = 0; k < n; ++k) trace[((u64)row + k) * ncand + idx] = v[k];
  }
  void spill(u32 off, const u32* v, int n) {   // spill area in words (mw_kernels.hip)
    if (spillv->size() < off + 8) spillv->resize(off + 8, 0u);
    for (int k = 0; k < n; ++k) (*spillv)[off + k] = v[k];
  }
  void fill(u32 off, u32* v, int n) {
    if (spillv->size() < off + 8) spillv->resize(off + 8, 0u);
    for (int k = 0; k < 8; ++k) v[k] = k < n ? (*spillv)[off + k] : 0u;
  }
  bool none(bool alive) { return !alive; }
};
}  // namespace

extern "C" {

int mg_validate_desc(const mg_prog_desc* d);

// Evaluate candidates [0, ncand) (explicit SoA inputs) or generated candidates
// [begin, begin+ncand) when leaves_soa == NULL.
int mwh_eval(const mg_prog_desc* d, const uint32_t* leaves_soa, uint64_t seed, uint64_t begin, size_t ncand,
             uint32_t flags, uint32_t* verdict, uint32_t* trace) {
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  std::vector<u32> consts(d->nconst_words + MW_KPAD, 0u);   // see mg_prog_load
  if (d->nconst_words) std::memcpy(consts.data(), d->consts, d->nconst_words * 4);
  std::vector<u32> code(d->ncode_words + 32, 0u);  // padded: the interpreter reads up to 20 words past END
  std::memcpy(code.data(), d->code, d->ncode_words * 4);
  std::vector<u32> spill;
  for (size_t i = 0; i < ncand; ++i) {
    HostEnv env{d->leaves, d->pool, leaves_soa, trace, (u64)ncand, (u64)i, seed, begin + i, &spill};
    verdict[i] = mw_run(code.data(), consts.data(), env, true, flags) ? 1u : 0u;
  }
  return 0;
}

// Division path counts (mw_alu.h DivCount) summed over generated candidates
// [begin, begin+ncand): out = {general digit steps, full, short, general}, the
// order of mg_stats.lane_div_*.  A host "wave" is one candidate.
int mwh_div_counts(const mg_prog_desc* d, uint64_t seed, uint64_t begin, size_t ncand, uint64_t* out) {
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  std::vector<u32> consts(d->nconst_words + MW_KPAD, 0u);
  if (d->nconst_words) std::memcpy(consts.data(), d->consts, d->nconst_words * 4);
  std::vector<u32> code(d->ncode_words + 32, 0u);
  std::memcpy(code.data(), d->code, d->ncode_words * 4);
  std::vector<u32> spill;
  for (int k = 0; k < 4; ++k) out[k] = 0;
  for (size_t i = 0; i < ncand; ++i) {
    HostEnv env{d->leaves, d->pool, nullptr, nullptr, (u64)ncand, (u64)i, seed, begin + i, &spill};
    (void)mw_run(code.data(), consts.data(), env, true, 0u);
    out[0] += env.dsteps.steps;
    out[1] += env.dsteps.full;
    out[2] += env.dsteps.shrt;
    out[3] += env.dsteps.gen;
  }
  return 0;
}

// Satisfied candidates among generated candidates [begin, begin+ncand) on
// nthreads OpenMP threads (0: the OpenMP default), each with its own spill
// area; verdict (optional) receives the per-candidate bits.
long long mwh_count_omp(const mg_prog_desc* d, uint64_t seed, uint64_t begin, size_t ncand, uint32_t flags,
                        uint8_t* verdict, int nthreads) {
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  std::vector<u32> consts(d->nconst_words + MW_KPAD, 0u);
  if (d->nconst_words) std::memcpy(consts.data(), d->consts, d->nconst_words * 4);
  std::vector<u32> code(d->ncode_words + 32, 0u);
  std::memcpy(code.data(), d->code, d->ncode_words * 4);
  if (nthreads <= 0) nthreads = omp_get_max_threads();
  long long sat = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : sat)
  {
    std::vector<u32> spill;
#pragma omp for schedule(dynamic, 256)
    for (long long i = 0; i < (long long)ncand; ++i) {
      HostEnv env{d->leaves, d->pool, nullptr, nullptr, (u64)ncand, (u64)i, seed, begin + (u64)i, &spill};
      const bool ok = mw_run(code.data(), consts.data(), env, true, flags);
      if (verdict) verdict[i] = ok ? 1 : 0;
      sat += ok ? 1 : 0;
    }
  }
  return sat;
}

int mwh_max_threads(void) { return omp_get_max_threads(); }

// Leaf values of candidate `cand` (the host twin of mg_witness_leaves).
int mwh_leaf_values(const mg_prog_desc* d, uint64_t seed, uint64_t cand, uint32_t* out) {
  int rc = mg_validate_desc(d);
  if (rc) return rc;
  for (size_t l = 0; l < d->nleaves; ++l) leaf_value(d->leaves + l * MW_LEAF_WORDS, d->pool, seed, cand, out + 8 * l);
  return 0;
}

int mwh_keccak256(const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n, uint8_t* out32) {
  for (size_t i = 0; i < n; ++i) {
    u64 h[4];
    keccak256_msg(data + off[i], len[i], h);
    std::memcpy(out32 + 32 * i, h, 32);
  }
  return 0;
}

}  // extern "C"
