// mw_compile.cpp — the host compiler (include/mythril_compile.h): constraint
// DAG -> interpreter bytecode.  The passes are those of
// mythril_amd/compiler.py (the parity reference; programs are byte-identical,
// tests/test_native_compile.py):
//   1. lower every term to machine ops on virtual registers, conjunct by
//      conjunct, operand-first, with the same rematerialisation rule for cheap
//      terms over leaves (compiler.py _Lowerer);
//   2. narrow results right after their operands (_schedule_narrow_early);
//   3. superinstructions CHECK_IMP / CHECK_IMPEQ(W) / W_CDINS (_fuse_checks);
//   4. Belady allocation of the W/N slot files with SPILL/FILL, spill slots
//      laid out hottest-first (_allocate, _layout_spills);
//   5. encode, constant pool in first-reference order.
// The Python prepare() spent most of its time here; this
// runs the same passes in a few microseconds per node.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mythril_compile.h"
#include "../../include/mythril_witness.h"
#include "mw_isa.h"

extern "C" int mw_fail(int code, const char* msg);

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

// MW_IR_OPS: the order of mythril_amd/ccompile.py IR_OPS (tests/test_native_compile.py checks it)
enum IrOp {
  IR_CONST, IR_VAR, IR_ARRAY, IR_APPLY, IR_SELECT, IR_STORE, IR_CONST_ARRAY,
  IR_AND, IR_OR, IR_NOT, IR_XOR, IR_IMPLIES, IR_EQ, IR_DISTINCT,
  IR_BVULT, IR_BVULE, IR_BVUGT, IR_BVUGE, IR_BVSLT, IR_BVSLE, IR_BVSGT, IR_BVSGE,
  IR_BVUMUL_NOOVFL, IR_BVSMUL_NOOVFL, IR_BVSMUL_NOUDFL, IR_BVADDC, IR_ITE,
  IR_BVADD, IR_BVMUL, IR_BVAND, IR_BVOR, IR_BVXOR, IR_CONCAT, IR_BVSUB,
  IR_BVUDIV, IR_BVUREM, IR_BVSDIV, IR_BVSREM, IR_BVSMOD, IR_BVSHL, IR_BVLSHR, IR_BVASHR,
  IR_BVNAND, IR_BVNOR, IR_BVXNOR, IR_BVCOMP, IR_BVNEG, IR_BVNOT,
  IR_EXTRACT, IR_ZERO_EXTEND, IR_SIGN_EXTEND, IR_REPEAT, IR_ROTATE_LEFT, IR_ROTATE_RIGHT,
  IR_NOPS
};

struct Unsupported {
  std::string msg;
};
struct BadInput {
  std::string msg;
};

const int NARROW_MAX = 32;
const int MAX_WIDTH = 256;
const int REMAT_MAX_COST = 16;
const int REMAT_DISTANCE = 32;
const size_t HOIST_CAP = 16;
const long long NEVER = 1LL << 60;

struct K256 {
  u32 l[8];
  bool operator<(const K256& o) const { return memcmp(l, o.l, sizeof l) < 0; }
  bool zero() const {
    for (int k = 0; k < 8; ++k)
      if (l[k]) return false;
    return true;
  }
};

K256 kmask(K256 v, int w) {
  for (int k = 0; k < 8; ++k) {
    int lo = 32 * k;
    if (lo >= w) v.l[k] = 0;
    else if (w - lo < 32) v.l[k] &= (1u << (w - lo)) - 1u;
  }
  return v;
}

K256 kshr(const K256& v, int s) {
  K256 r{};
  int q = s / 32, b = s % 32;
  for (int k = 0; k < 8; ++k) {
    int j = k + q;
    if (j >= 8) break;
    u64 x = v.l[j] >> b;
    if (b && j + 1 < 8) x |= (u64)v.l[j + 1] << (32 - b);
    r.l[k] = (u32)x;
  }
  return r;
}

K256 kshl(const K256& v, int s) {   // callers keep the result below 2^256 (compiler.py does not mask)
  K256 r{};
  int q = s / 32, b = s % 32;
  for (int k = 7; k >= 0; --k) {
    int j = k - q;
    if (j < 0) continue;
    u64 x = (u64)v.l[j] << b;
    if (b && j >= 1) x |= v.l[j - 1] >> (32 - b);
    r.l[k] = (u32)x;
  }
  return r;
}

// operands: a virtual register, a constant, or (after allocation) a physical slot
enum { O_NONE = 0, O_VREG = 1, O_CONST = 2, O_PHYS = 3, O_RAW = 4 };   // O_RAW: v is the field itself
struct Opnd {
  int kind = O_NONE;
  int v = 0;
};

struct Insn {
  int op = 0;
  int width = 0;
  int dst = -1;      // vreg id (before allocation) / physical slot (after), -1 none
  Opnd s[3];
  int ns = 0;
  long long imm = 0;  // STORE_*: the traced record until encode
  bool chain = false;
  bool grid = false;  // SPILL_N of a grid table entry (form_grids): a fixed word, not a spill slot
  bool cdleaf = false;  // a LEAF_N kept beside the W_CDINS that draws it again (fuse_checks)
};

// MYTHRIL_AMD_REMAT_LEAVES=0 turns leaf rematerialisation off (read once, as
// compiler.py reads it at import)
bool remat_leaves() {
  static const bool on = [] {
    const char* e = getenv("MYTHRIL_AMD_REMAT_LEAVES");
    return !(e && strcmp(e, "0") == 0);
  }();
  return on;
}

int dst_cls(int op) {   // 'W', 'N' or 0 (isa.SHAPES[op][0])
  if (op >= MW_W_ADD && op <= MW_W_CDINS) return 'W';
  if (op >= MW_N_EXTRACTW && op <= MW_N_ADDCN) return 'N';
  if (op == MW_LEAF_W || op == MW_FILL_W || op == MW_MOV_W) return 'W';
  if (op == MW_LEAF_N || op == MW_FILL_N || op == MW_MOV_N) return 'N';
  return 0;
}

int cls_of(int w) { return w <= NARROW_MAX ? 'N' : 'W'; }

int ceil_log2(int L) {
  int e = 0;
  while ((1 << e) < L) ++e;
  return e;
}

struct Node {
  int op, width, flags, p0, p1, nargs;
  const int32_t* args;
  int w() const { return width == 0 ? 1 : width; }
  bool is_array() const { return flags & 1; }
};

struct Compiler {
  // register slots the allocator may use (mw_compile_slots: fewer, for the
  // asm interpreter's smaller register layouts; W7 / N31 / N63 never)
  int w_slots = MW_NW, n_slots = MW_NN;
  std::vector<Node> nodes;
  const uint8_t* kvals = nullptr;
  size_t nkvals = 0;

  // constants created while lowering (compiler.py Const objects)
  std::vector<K256> kv;
  std::vector<char> kc;

  std::vector<Insn> insns;
  std::vector<char> vcls{0};   // vreg id -> class ('W'/'N'); ids start at 1
  std::vector<char> in_memo;
  std::vector<Opnd> memo;
  std::vector<int> memo_scope, memo_at;
  std::vector<int> cost;
  int scope = 0;
  std::map<int, int> leaf_index;   // var name id -> leaf index
  std::vector<int> leaf_nodes;
  std::vector<char> trace_req, trace_emitted;

  // ------------------------------------------------------------------ helpers
  const Node& N(int i) const { return nodes[i]; }
  int opcls(const Opnd& o) const { return o.kind == O_VREG ? vcls[o.v] : kc[o.v]; }

  Opnd mkconst(K256 v, int cls) {   // by value: callers pass elements of kv
    kv.push_back(v);
    kc.push_back((char)cls);
    return Opnd{O_CONST, (int)kv.size() - 1};
  }
  Opnd k(K256 v, int w) { return mkconst(kmask(v, w), cls_of(w)); }
  Opnd ksmall(u32 x, int w) {
    K256 v{};
    v.l[0] = x;
    return k(v, w);
  }
  K256 node_val(int i) const {
    K256 v{};
    size_t at = (size_t)nodes[i].p0;
    if (at >= nkvals) throw BadInput{"constant value index out of range"};
    memcpy(v.l, kvals + 32 * at, 32);   // little-endian limbs
    return v;
  }

  Opnd emit(int op, int width, std::initializer_list<Opnd> srcs, long long imm = 0) {
    Insn in;
    in.op = op;
    in.width = width;
    for (const Opnd& s : srcs) in.s[in.ns++] = s;
    in.imm = imm;
    int c = dst_cls(op);
    Opnd d;
    if (c) {
      vcls.push_back((char)c);
      in.dst = (int)vcls.size() - 1;
      d = Opnd{O_VREG, in.dst};
    }
    insns.push_back(in);
    return d;
  }
  void emit_void(int op, int width, std::initializer_list<Opnd> srcs) {
    Insn in;
    in.op = op;
    in.width = width;
    for (const Opnd& s : srcs) in.s[in.ns++] = s;
    insns.push_back(in);
  }

  Opnd as_cls(Opnd v, int width, int want) {
    if (opcls(v) == want) return v;
    if (want == 'W') {
      if (v.kind == O_CONST) return mkconst(kv[v.v], 'W');
      return emit(MW_W_ZEXTN, std::max(width, 33), {v});
    }
    throw Unsupported{"narrowing class change"};
  }

  // compiler.py node_cost
  int node_cost(int i) const {
    const Node& n = N(i);
    int op = n.op;
    if (op == IR_CONST || op == IR_VAR || op == IR_ARRAY || op == IR_APPLY) return 0;
    int kk = n.nargs;
    if (n.width == 0 && (op == IR_AND || op == IR_OR || op == IR_NOT || op == IR_XOR || op == IR_IMPLIES))
      return std::max(kk, 1);
    if (op == IR_ITE) return std::max(1, (n.w() + 31) / 32);
    if ((op == IR_EQ || op == IR_DISTINCT) && kk && N(n.args[0]).width == 0) return kk;
    int aw = kk ? N(n.args[0]).w() : n.w();
    int L = (aw + 31) / 32, Lo = (n.w() + 31) / 32;
    int m1 = std::max(kk - 1, 1);
    switch (op) {
      case IR_BVADD: case IR_BVSUB: case IR_BVAND: case IR_BVOR: case IR_BVXOR: return L * m1;
      case IR_BVADDC: case IR_BVNEG: case IR_BVNOT: return L;
      case IR_BVNAND: case IR_BVNOR: case IR_BVXNOR: return 2 * L;
      case IR_EQ: case IR_DISTINCT: return 2 * L * m1;
      case IR_BVULT: case IR_BVULE: case IR_BVUGT: case IR_BVUGE:
      case IR_BVSLT: case IR_BVSLE: case IR_BVSGT: case IR_BVSGE: return L + 1;
      case IR_EXTRACT: case IR_CONCAT: case IR_ZERO_EXTEND: case IR_SIGN_EXTEND: case IR_REPEAT:
      case IR_ROTATE_LEFT: case IR_ROTATE_RIGHT: return Lo;
      case IR_BVSHL: case IR_BVLSHR: case IR_BVASHR:
        return L > 1 ? 2 * L + L * std::max(1, ceil_log2(L)) : 2;
      case IR_BVMUL: return 2 * L * (L + 1) * m1;
      case IR_BVUMUL_NOOVFL: return 4 * L * L + L;
      case IR_BVUDIV: case IR_BVUREM: case IR_BVSDIV: case IR_BVSREM: case IR_BVSMOD: {
        int base;
        if (L == 1) {
          base = 20;
        } else {
          int lg = std::max(1, ceil_log2(L));
          base = L * (6 * L + 20) + 3 * (2 * L + L * lg);
        }
        return base + ((op == IR_BVSDIV || op == IR_BVSREM || op == IR_BVSMOD) ? 4 * L : 0);
      }
      case IR_BVCOMP: return 2 * L;
      default: return L;
    }
  }

  // ------------------------------------------------------------------ lowering
  bool fresh(int m) {
    if (!in_memo[m]) return false;
    const Node& n = N(m);
    if (n.op == IR_VAR || n.op == IR_CONST || n.nargs == 0 || cost[m] > REMAT_MAX_COST) return true;
    for (int j = 0; j < n.nargs; ++j) {
      int a = N(n.args[j]).op;
      if (a != IR_VAR && a != IR_CONST) return true;
    }
    int sc = memo_scope[m] < 0 ? scope : memo_scope[m];
    if (sc == scope && (long long)insns.size() - memo_at[m] <= REMAT_DISTANCE) return true;
    in_memo[m] = 0;   // recompute here
    return false;
  }

  bool lazy_concat(int m) const {
    const Node& n = N(m);
    return n.op == IR_CONCAT && cls_of(n.w()) == 'W' && n.w() <= MAX_WIDTH;
  }

  Opnd lower(int n) {
    if (fresh(n)) return memo[n];
    std::vector<std::pair<int, bool>> stack;
    stack.push_back({n, false});
    while (!stack.empty()) {
      std::pair<int, bool> top = stack.back();
      stack.pop_back();
      int m = top.first;
      if (top.second) {
        if (!in_memo[m]) lower_one(m);
        continue;
      }
      if (fresh(m)) continue;
      stack.push_back({m, true});
      if (lazy_concat(m)) continue;
      const Node& nm = N(m);
      for (int j = nm.nargs - 1; j >= 0; --j) {
        int a = nm.args[j];
        if (!fresh(a)) stack.push_back({a, false});
      }
    }
    return memo[n];
  }

  Opnd lower_one(int n) {
    if (in_memo[n]) return memo[n];
    Opnd v = lower_node(n);
    in_memo[n] = 1;
    memo[n] = v;
    memo_scope[n] = scope;
    memo_at[n] = (int)insns.size();
    if (trace_req[n] && !trace_emitted[n]) {
      trace_emitted[n] = 1;
      Insn st;
      st.op = opcls(v) == 'W' ? MW_STORE_W : MW_STORE_N;
      st.width = N(n).w();
      st.s[st.ns++] = v;
      st.imm = n;   // row patched at encode time
      insns.push_back(st);
    }
    return v;
  }

  Opnd bin(int op_w, int op_n, int width, Opnd a, Opnd b) {
    if (cls_of(width) == 'W') {
      Opnd x = as_cls(a, width, 'W');
      Opnd y = as_cls(b, width, 'W');
      return emit(op_w, width, {x, y});
    }
    return emit(op_n, width, {a, b});
  }

  Opnd fold(int op, int w, const std::vector<Opnd>& args) {
    if (args.size() == 1) return args[0];
    Opnd acc = args[0];
    bool wide = op >= MW_W_ADD && op <= MW_W_CDINS;
    for (size_t j = 1; j < args.size(); ++j) {
      if (wide) {
        Opnd x = as_cls(acc, w, 'W');
        Opnd y = as_cls(args[j], w, 'W');
        acc = emit(op, w, {x, y});
      } else {
        acc = emit(op, w, {acc, args[j]});
      }
    }
    return acc;
  }

  Opnd eq(int aw, Opnd a, Opnd b) {
    if (cls_of(aw) == 'W') {
      Opnd x = as_cls(a, aw, 'W');
      Opnd y = as_cls(b, aw, 'W');
      return emit(MW_N_EQ, aw, {x, y});
    }
    return emit(MW_N_EQN, aw, {a, b});
  }

  // one LSB-first part of a wide concat (compiler.py _concat / _concat_lazy, W class)
  void concat_w_step(Opnd& acc, bool& have, Opnd v, int w, int off) {
    if (!have) {
      have = true;
      if (v.kind == O_CONST) acc = mkconst(kv[v.v], 'W');
      else if (opcls(v) == 'W') acc = v;
      else acc = emit(MW_W_ZEXTN, w, {v});
    } else if (v.kind == O_CONST) {
      if (!kv[v.v].zero()) {
        Opnd x = as_cls(acc, w, 'W');
        Opnd c = mkconst(kshl(kv[v.v], off), 'W');
        acc = emit(MW_W_OR, w, {x, c});
      }
    } else if (opcls(v) == 'N') {
      Opnd x = as_cls(acc, w, 'W');
      acc = emit(MW_W_INSN, w, {x, v}, off);
    } else {
      Opnd sh = emit(MW_W_SHLI, w, {v}, off);
      Opnd x = as_cls(acc, w, 'W');
      acc = emit(MW_W_OR, w, {x, sh});
    }
  }

  Opnd concat_lazy(int n) {
    const Node& nn = N(n);
    int w = nn.w();
    Opnd acc;
    bool have = false;
    int off = 0;
    for (int j = nn.nargs - 1; j >= 0; --j) {
      int part = nn.args[j];
      int pw = N(part).w();
      Opnd v = lower(part);
      concat_w_step(acc, have, v, w, off);
      off += pw;
    }
    return acc;
  }

  Opnd concat(const std::vector<int>& widths, const std::vector<Opnd>& vals, int w) {
    int off = 0;
    Opnd acc;
    bool have = false;
    if (cls_of(w) == 'N') {
      for (int j = (int)vals.size() - 1; j >= 0; --j) {
        Opnd v = vals[j];
        if (!have) {
          acc = v;
          have = true;
        } else {
          Opnd sh = off ? emit(MW_N_SHLI, w, {v}, off) : v;
          acc = emit(MW_N_OR, w, {acc, sh});
        }
        off += widths[j];
      }
      return acc;
    }
    for (int j = (int)vals.size() - 1; j >= 0; --j) {
      concat_w_step(acc, have, vals[j], w, off);
      off += widths[j];
    }
    return acc;
  }

  Opnd lower_node(int i) {
    const Node& n = N(i);
    int op = n.op, w = n.w();
    if (n.is_array()) throw Unsupported{"array term outside select (Ackermannisation pending)"};
    if (op == IR_CONST) return k(node_val(i), w);
    if (op == IR_VAR) {
      if (w > MAX_WIDTH) throw Unsupported{"free variable wider than 256 bits"};
      auto it = leaf_index.find(n.p0);
      int li;
      if (it == leaf_index.end()) {
        li = (int)leaf_nodes.size();
        leaf_index[n.p0] = li;
        leaf_nodes.push_back(i);
      } else {
        li = it->second;
      }
      return emit(cls_of(w) == 'W' ? MW_LEAF_W : MW_LEAF_N, w, {}, li);
    }
    if (op < 0) throw Unsupported{"op outside the vocabulary"};
    bool too_wide = w > MAX_WIDTH;
    for (int j = 0; j < n.nargs && !too_wide; ++j) {
      const Node& a = N(n.args[j]);
      if (!a.is_array() && a.w() > MAX_WIDTH) too_wide = true;
    }
    if (too_wide) throw Unsupported{"term wider than 256 bits"};
    if (op == IR_SELECT || op == IR_STORE || op == IR_APPLY || op == IR_CONST_ARRAY)
      throw Unsupported{"array read / application (Ackermannisation pending)"};
    if (lazy_concat(i)) return concat_lazy(i);
    std::vector<Opnd> args;
    args.reserve(n.nargs);
    for (int j = 0; j < n.nargs; ++j) args.push_back(lower(n.args[j]));
    if (n.width == 0) {   // Bool connectives: width-1 N values
      switch (op) {
        case IR_AND: return fold(MW_N_AND, 1, args);
        case IR_OR: return fold(MW_N_OR, 1, args);
        case IR_XOR: return fold(MW_N_XOR, 1, args);
        case IR_NOT: { Opnd t = ksmall(1, 1); return emit(MW_N_XOR, 1, {args[0], t}); }
        case IR_IMPLIES: return emit(MW_N_ULEN, 1, {args[0], args[1]});
        case IR_EQ: case IR_DISTINCT: {
          int aw = N(n.args[0]).w();
          if (N(n.args[0]).is_array()) throw Unsupported{"array equality"};
          std::vector<Opnd> pairs;
          if (op == IR_EQ) {
            for (size_t j = 1; j < args.size(); ++j) pairs.push_back(eq(aw, args[0], args[j]));
            return fold(MW_N_AND, 1, pairs);
          }
          for (size_t a = 0; a < args.size(); ++a)
            for (size_t b = a + 1; b < args.size(); ++b) {
              Opnd e = eq(aw, args[a], args[b]);
              Opnd t = ksmall(1, 1);
              pairs.push_back(emit(MW_N_XOR, 1, {e, t}));
            }
          return fold(MW_N_AND, 1, pairs);
        }
        case IR_BVULT: case IR_BVULE: case IR_BVUGT: case IR_BVUGE:
        case IR_BVSLT: case IR_BVSLE: case IR_BVSGT: case IR_BVSGE: {
          int aw = N(n.args[0]).w();
          Opnd a = args[0], b = args[1];
          int wop, nop;
          bool swap = op == IR_BVUGT || op == IR_BVUGE || op == IR_BVSGT || op == IR_BVSGE;
          if (op == IR_BVULT || op == IR_BVUGT) { wop = MW_N_ULT; nop = MW_N_ULTN; }
          else if (op == IR_BVULE || op == IR_BVUGE) { wop = MW_N_ULE; nop = MW_N_ULEN; }
          else if (op == IR_BVSLT || op == IR_BVSGT) { wop = MW_N_SLT; nop = MW_N_SLTN; }
          else { wop = MW_N_SLE; nop = MW_N_SLEN; }
          if (swap) std::swap(a, b);
          if (cls_of(aw) == 'W') {
            Opnd x = as_cls(a, aw, 'W');
            Opnd y = as_cls(b, aw, 'W');
            return emit(wop, aw, {x, y});
          }
          return emit(nop, aw, {a, b});
        }
        case IR_BVADDC: {
          int aw = N(n.args[0]).w();
          if (cls_of(aw) == 'W') {
            Opnd x = as_cls(args[0], aw, 'W');
            Opnd y = as_cls(args[1], aw, 'W');
            return emit(MW_N_ADDC, aw, {x, y});
          }
          return emit(MW_N_ADDCN, aw, {args[0], args[1]});
        }
        case IR_BVUMUL_NOOVFL: {
          int aw = N(n.args[0]).w();
          if (cls_of(aw) == 'W') return bin(MW_N_UMULNO, MW_N_UMULNON, aw, args[0], args[1]);
          return emit(MW_N_UMULNON, aw, {args[0], args[1]});
        }
        case IR_ITE: return emit(MW_N_ITE, 1, {args[1], args[2], args[0]});
        default: throw Unsupported{"bool op outside the vocabulary"};
      }
    }
    int C = cls_of(w);
    bool W = C == 'W';
    switch (op) {
      case IR_BVADD: return fold(W ? MW_W_ADD : MW_N_ADD, w, args);
      case IR_BVMUL: return fold(W ? MW_W_MUL : MW_N_MUL, w, args);
      case IR_BVAND: return fold(W ? MW_W_AND : MW_N_AND, w, args);
      case IR_BVOR: return fold(W ? MW_W_OR : MW_N_OR, w, args);
      case IR_BVXOR: return fold(W ? MW_W_XOR : MW_N_XOR, w, args);
      case IR_BVSUB: return bin(MW_W_SUB, MW_N_SUB, w, args[0], args[1]);
      case IR_BVNEG: { Opnd z = ksmall(0, w); return bin(MW_W_SUB, MW_N_SUB, w, z, args[0]); }
      case IR_BVNOT: return emit(W ? MW_W_NOT : MW_N_NOT, w, {args[0]});
      case IR_BVNAND: case IR_BVNOR: case IR_BVXNOR: {
        Opnd t = op == IR_BVNAND ? bin(MW_W_AND, MW_N_AND, w, args[0], args[1])
                 : op == IR_BVNOR ? bin(MW_W_OR, MW_N_OR, w, args[0], args[1])
                                  : bin(MW_W_XOR, MW_N_XOR, w, args[0], args[1]);
        return emit(W ? MW_W_NOT : MW_N_NOT, w, {t});
      }
      case IR_BVUDIV: return bin(MW_W_UDIV, MW_N_UDIV, w, args[0], args[1]);
      case IR_BVUREM: return bin(MW_W_UREM, MW_N_UREM, w, args[0], args[1]);
      case IR_BVSDIV: return bin(MW_W_SDIV, MW_N_SDIV, w, args[0], args[1]);
      case IR_BVSREM: return bin(MW_W_SREM, MW_N_SREM, w, args[0], args[1]);
      case IR_BVSMOD: return bin(MW_W_SMOD, MW_N_SMOD, w, args[0], args[1]);
      case IR_BVSHL: case IR_BVLSHR: case IR_BVASHR: {
        Opnd a = args[0], b = args[1];
        if (b.kind == O_CONST && op != IR_BVASHR) {
          const K256& bv = kv[b.v];
          bool big = false;
          for (int q = 1; q < 8; ++q) big = big || bv.l[q];
          if (big || bv.l[0] >= (u32)w) return ksmall(0, w);
          if (bv.l[0] == 0) return a;
          int name = op == IR_BVSHL ? (W ? MW_W_SHLI : MW_N_SHLI) : (W ? MW_W_LSHRI : MW_N_LSHRI);
          return emit(name, w, {a}, bv.l[0]);
        }
        if (op == IR_BVSHL) return bin(MW_W_SHL, MW_N_SHL, w, a, b);
        if (op == IR_BVLSHR) return bin(MW_W_LSHR, MW_N_LSHR, w, a, b);
        return bin(MW_W_ASHR, MW_N_ASHR, w, a, b);
      }
      case IR_ITE: {
        Opnd c = args[0], a = args[1], b = args[2];
        if (W) {
          Opnd x = as_cls(a, w, 'W');
          Opnd y = as_cls(b, w, 'W');
          return emit(MW_W_ITE, w, {x, y, c});
        }
        return emit(MW_N_ITE, w, {a, b, c});
      }
      case IR_BVCOMP: return eq(N(n.args[0]).w(), args[0], args[1]);
      case IR_EXTRACT: {
        int hi = n.p0, lo = n.p1;
        (void)hi;
        Opnd a = args[0];
        int aw = N(n.args[0]).w();
        if (a.kind == O_CONST) return k(kshr(kv[a.v], lo), w);
        if (cls_of(aw) == 'W') {
          if (C == 'N') return emit(MW_N_EXTRACTW, w, {a}, lo);
          if (lo == 0 && w == aw) return a;
          return emit(MW_W_LSHRI, w, {a}, lo);
        }
        if (lo == 0 && w == aw) return a;
        return emit(MW_N_LSHRI, w, {a}, lo);
      }
      case IR_ZERO_EXTEND: {
        Opnd a = args[0];
        if (a.kind == O_CONST) return mkconst(kv[a.v], C);
        return as_cls(a, N(n.args[0]).w(), C);
      }
      case IR_SIGN_EXTEND: {
        Opnd a = args[0];
        int aw = N(n.args[0]).w();
        if (C == 'N') return emit(MW_N_SEXT, w, {a}, aw);
        if (opcls(a) == 'N') return emit(MW_W_SEXTN, w, {a}, aw);
        return emit(MW_W_SEXT, w, {a}, aw);
      }
      case IR_CONCAT: {
        std::vector<int> widths;
        for (int j = 0; j < n.nargs; ++j) widths.push_back(N(n.args[j]).w());
        return concat(widths, args, w);
      }
      case IR_REPEAT: {
        int aw = N(n.args[0]).w();
        std::vector<int> widths(n.p0, aw);
        std::vector<Opnd> vals(n.p0, args[0]);
        return concat(widths, vals, w);
      }
      case IR_ROTATE_LEFT: case IR_ROTATE_RIGHT: {
        int r = n.p0 % w;
        Opnd a = args[0];
        if (r == 0) return a;
        int left = op == IR_ROTATE_LEFT ? r : w - r;
        Opnd hi = emit(W ? MW_W_SHLI : MW_N_SHLI, w, {a}, left);
        Opnd lo = emit(W ? MW_W_LSHRI : MW_N_LSHRI, w, {a}, w - left);
        return emit(W ? MW_W_OR : MW_N_OR, w, {hi, lo});
      }
      default: throw Unsupported{"op outside the vocabulary"};
    }
  }

  // ------------------------------------------------------------------ scheduling
  static bool is_v(const Opnd& o) { return o.kind == O_VREG; }
  static bool is_def(const Opnd& o, const Insn& in) { return o.kind == O_VREG && in.dst >= 0 && o.v == in.dst; }

  std::vector<Insn> schedule_narrow_early(const std::vector<Insn>& in) {
    size_t nv = vcls.size();
    std::vector<int> anchor(nv, 0);
    std::vector<char> leafv(nv, 0);
    for (const Insn& x : in)
      if ((x.op == MW_LEAF_W || x.op == MW_LEAF_N) && x.dst >= 0) leafv[x.dst] = 1;
    std::vector<std::vector<int>> after(in.size());
    std::vector<char> keep(in.size(), 1);
    for (size_t i = 0; i < in.size(); ++i) {
      const Insn& x = in[i];
      bool nonleaf = false;
      int a = -1;
      for (int j = 0; j < x.ns; ++j)
        if (is_v(x.s[j])) {
          nonleaf = nonleaf || !leafv[x.s[j].v];
          a = std::max(a, anchor[x.s[j].v]);
        }
      bool lfm = x.op == MW_LEAF_W || x.op == MW_LEAF_N || x.op == MW_FILL_W || x.op == MW_FILL_N ||
                 x.op == MW_MOV_W || x.op == MW_MOV_N;
      bool movable = (x.dst >= 0 && vcls[x.dst] == 'N' && nonleaf && !lfm) || (x.op == MW_CHECK && nonleaf);
      if (movable && x.op != MW_CHECK) movable = after[a].size() < HOIST_CAP;
      if (movable) {
        after[a].push_back((int)i);
        if (x.dst >= 0) anchor[x.dst] = a;
        keep[i] = 0;
      } else {
        if (x.dst >= 0) anchor[x.dst] = (int)i;
      }
    }
    std::vector<Insn> out;
    out.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
      if (keep[i]) out.push_back(in[i]);
      for (int j : after[i]) out.push_back(in[j]);
    }
    return out;
  }

  std::vector<int> use_counts(const std::vector<Insn>& in) const {
    std::vector<int> u(vcls.size(), 0);
    for (const Insn& x : in)
      for (int j = 0; j < x.ns; ++j)
        if (is_v(x.s[j])) ++u[x.s[j].v];
    return u;
  }

  // p = (key = K); CHECK_IMPEQ p, x, y -> CHECK_IMPEQK key, x, y, imm = K for
  // K < 2^31 (compiler._fuse_keyed_premises): the premise flags of an index
  // key (lower._index_key) are dropped once nothing else reads them
  std::vector<Insn> fuse_keyed_premises(const std::vector<Insn>& in) {
    std::vector<int> def(vcls.size(), -1);
    for (size_t i = 0; i < in.size(); ++i)
      if (in[i].dst >= 0) def[in[i].dst] = (int)i;
    std::vector<char> fused(vcls.size(), 0);
    bool any = false;
    std::vector<Insn> out;
    out.reserve(in.size());
    for (const Insn& x : in) {
      if (x.op == MW_CHECK_IMPEQ && is_v(x.s[0]) && def[x.s[0].v] >= 0) {
        const Insn& d = in[def[x.s[0].v]];
        Opnd key = d.s[0], k = d.s[1];
        if (key.kind == O_CONST) std::swap(key, k);
        if (d.op == MW_N_EQN && d.width <= 32 && is_v(key) && k.kind == O_CONST && k_small31(kv[k.v])) {
          Insn c;
          c.op = MW_CHECK_IMPEQK;
          c.width = x.width;
          c.ns = 3;
          c.s[0] = key;
          c.s[1] = x.s[1];
          c.s[2] = x.s[2];
          c.imm = kv[k.v].l[0];
          out.push_back(c);
          fused[d.dst] = 1;
          any = true;
          continue;
        }
      }
      out.push_back(x);
    }
    if (!any) return out;
    std::vector<int> uses = use_counts(out);
    std::vector<Insn> kept;
    kept.reserve(out.size());
    for (const Insn& x : out)
      if (x.dst < 0 || !fused[x.dst] || uses[x.dst]) kept.push_back(x);
    return kept;
  }
  static bool k_small31(const K256& v) {
    for (int q = 1; q < 8; ++q)
      if (v.l[q]) return false;
    return v.l[0] < 0x80000000u;
  }

  // a run of W_CDINS links and the leaves kept beside them: the leaves first,
  // so the links stay adjacent and chain (compiler.py _hoist_cdins_leaves)
  static std::vector<Insn> hoist_cdins_leaves(const std::vector<Insn>& in) {
    std::vector<Insn> out;
    out.reserve(in.size());
    size_t i = 0;
    while (i < in.size()) {
      if (in[i].op == MW_W_CDINS || in[i].cdleaf) {
        size_t j = i;
        while (j < in.size() && (in[j].op == MW_W_CDINS || in[j].cdleaf)) ++j;
        for (size_t k = i; k < j; ++k)
          if (in[k].op != MW_W_CDINS) out.push_back(in[k]);
        for (size_t k = i; k < j; ++k)
          if (in[k].op == MW_W_CDINS) out.push_back(in[k]);
        i = j;
      } else {
        out.push_back(in[i++]);
      }
    }
    return out;
  }

  // ------------------------------------------------------------------ grids (compiler.py _form_grids)
  static constexpr size_t GRID_MIN = 64, GRID_MAX_N = 32;
  struct OKey {
    int kind, v;
    char cls;
    K256 val;
  };
  OKey okey(const Opnd& o) const {
    OKey k{o.kind, o.v, 0, K256{}};
    if (o.kind == O_CONST) {
      k.v = 0;
      k.cls = kc[o.v];
      k.val = kv[o.v];
    }
    return k;
  }
  static bool okey_eq(const OKey& a, const OKey& b) {
    if (a.kind != b.kind) return false;
    if (a.kind != O_CONST) return a.v == b.v;
    return a.cls == b.cls && memcmp(a.val.l, b.val.l, sizeof a.val.l) == 0;
  }
  struct GridPlan {
    std::vector<Opnd> table, rowop;
    std::vector<long long> rowE;
    std::vector<int> rowlast;
  };
  bool grid_plan(const std::vector<Insn>& in, const std::vector<int>& pos, GridPlan& gp) const {
    std::vector<OKey> keys;
    std::vector<Opnd> firsto;
    std::vector<std::vector<int>> adj;
    auto idx_of = [&](const Opnd& o) -> int {
      OKey k = okey(o);
      for (size_t q = 0; q < keys.size(); ++q)
        if (okey_eq(keys[q], k)) return (int)q;
      keys.push_back(k);
      firsto.push_back(o);
      adj.emplace_back();
      return (int)keys.size() - 1;
    };
    std::vector<std::pair<int, int>> pr(pos.size());
    for (size_t q = 0; q < pos.size(); ++q) {
      const Insn& x = in[pos[q]];
      if (okey_eq(okey(x.s[1]), okey(x.s[2]))) return false;
      int a = idx_of(x.s[1]), b = idx_of(x.s[2]);
      adj[a].push_back(b);
      adj[b].push_back(a);
      pr[q] = {a, b};
    }
    std::vector<int> col(keys.size(), -1);
    col[0] = 0;
    std::vector<int> st{0};
    while (!st.empty()) {
      int k = st.back();
      st.pop_back();
      for (int m : adj[k]) {
        if (col[m] < 0) {
          col[m] = 1 - col[k];
          st.push_back(m);
        } else if (col[m] == col[k]) {
          return false;
        }
      }
    }
    for (int c : col)
      if (c < 0) return false;
    size_t n0 = 0;
    for (int c : col) n0 += c == 0;
    const int first_side = n0 >= keys.size() - n0 ? 0 : 1;   // the larger side that fits is the table
    for (int ts = 0; ts < 2; ++ts) {
      const int tside = ts == 0 ? first_side : 1 - first_side;
      std::vector<int> tk, rk;
      for (size_t q = 0; q < keys.size(); ++q) (col[q] == tside ? tk : rk).push_back((int)q);
      size_t n = tk.size(), m = rk.size();
      if (n > GRID_MAX_N || n * m != pos.size()) continue;
      std::vector<int> tix(keys.size(), -1), rix(keys.size(), -1);
      for (size_t q = 0; q < n; ++q) tix[tk[q]] = (int)q;
      for (size_t q = 0; q < m; ++q) rix[rk[q]] = (int)q;
      std::vector<long long> e(n * m, -1);
      std::vector<int> last(m, -1);
      bool ok = true;
      for (size_t q = 0; q < pos.size() && ok; ++q) {
        int a = pr[q].first, b = pr[q].second;
        int t = col[a] == tside ? a : b, r = col[a] == tside ? b : a;
        long long& slot = e[(size_t)tix[t] * m + rix[r]];
        if (slot >= 0) ok = false;
        slot = in[pos[q]].imm;
        last[rix[r]] = pos[q];
      }
      if (!ok) continue;
      long long top = -1;
      for (size_t q = 0; q < n; ++q) top = std::max(top, e[q * m]);
      std::vector<long long> off(n);
      std::vector<char> seen(n, 0);
      for (size_t q = 0; q < n && ok; ++q) {
        off[q] = top - e[q * m];
        if (off[q] < 0 || off[q] >= (long long)n || seen[off[q]]) ok = false;
        else seen[off[q]] = 1;
      }
      if (!ok) continue;
      gp = GridPlan{};
      for (size_t r = 0; r < m && ok; ++r) {
        long long E = e[r] + off[0];
        for (size_t q = 1; q < n && ok; ++q) ok = e[q * m + r] + off[q] == E;
        gp.rowop.push_back(firsto[rk[r]]);
        gp.rowE.push_back(E);
        gp.rowlast.push_back(last[r]);
      }
      if (!ok) continue;
      gp.table.assign(n, Opnd{});
      for (size_t q = 0; q < n; ++q) gp.table[off[q]] = firsto[tk[q]];
      return true;
    }
    return false;
  }

  std::vector<Insn> form_grids(const std::vector<Insn>& in) {
    std::vector<int> gkey, gidx(vcls.size(), -1);
    std::vector<std::vector<int>> gpos;
    for (size_t i = 0; i < in.size(); ++i) {
      const Insn& x = in[i];
      if (x.op == MW_CHECK_IMPEQK && is_v(x.s[0])) {
        int k = x.s[0].v;
        if (gidx[k] < 0) {
          gidx[k] = (int)gkey.size();
          gkey.push_back(k);
          gpos.emplace_back();
        }
        gpos[gidx[k]].push_back((int)i);
      }
    }
    std::vector<int> defpos(vcls.size(), -1);
    for (size_t i = 0; i < in.size(); ++i)
      if (in[i].dst >= 0) defpos[in[i].dst] = (int)i;
    std::vector<char> drop(in.size(), 0);
    std::vector<std::vector<Insn>> after(in.size());
    std::vector<char> redrawn(vcls.size(), 0);
    bool any_redrawn = false;
    int t0 = 0;
    bool any = false;
    for (size_t g = 0; g < gkey.size(); ++g) {
      const std::vector<int>& pos = gpos[g];
      if (pos.size() < GRID_MIN) continue;
      GridPlan gp;
      if (!grid_plan(in, pos, gp)) continue;
      int n = (int)gp.table.size();
      if (t0 + n > 1024) break;
      Opnd key = in[pos[0]].s[0];
      int put = defpos[key.v];
      for (const Opnd& t : gp.table)
        if (is_v(t)) put = std::max(put, defpos[t.v]);
      for (int k = 0; k < n; ++k) {
        Insn p;
        p.op = MW_SPILL_N;
        p.grid = true;
        p.ns = 1;
        p.s[0] = gp.table[k];
        p.imm = t0 + k;
        after[put].push_back(p);
      }
      int width = in[pos[0]].width;
      for (size_t r = 0; r < gp.rowop.size(); ++r) {
        int at = gp.rowlast[r] > put ? gp.rowlast[r] : put;
        Opnd opnd = gp.rowop[r];
        if (is_v(opnd) && in[defpos[opnd.v]].op == MW_LEAF_N && defpos[opnd.v] < put) {
          // a leaf defined before the table: drawn again at its row rather than
          // kept live (a spill and a fill) across the program
          const Insn& d = in[defpos[opnd.v]];
          Insn l;
          l.op = MW_LEAF_N;
          l.width = d.width;
          l.dst = (int)vcls.size();
          vcls.push_back('N');
          l.ns = 0;
          l.imm = d.imm;
          after[at].push_back(l);
          redrawn[opnd.v] = 1;
          any_redrawn = true;
          opnd = Opnd{O_VREG, l.dst};
        }
        Insn c;
        c.op = MW_CHECK_GRID;
        c.width = width;
        c.ns = 3;
        c.s[0] = key;
        c.s[1] = opnd;
        c.s[2] = Opnd{O_RAW, t0 | (n - 1) << 10};
        c.imm = gp.rowE[r];
        after[at].push_back(c);
      }
      for (int p : pos) drop[p] = 1;
      t0 += n;
      any = true;
    }
    if (!any) return in;
    std::vector<Insn> out;
    out.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
      if (!drop[i]) out.push_back(in[i]);
      for (const Insn& a : after[i]) out.push_back(a);
    }
    if (any_redrawn) {   // the leaves drawn again that nothing else reads any more
      std::vector<int> u = use_counts(out);
      std::vector<Insn> kept;
      kept.reserve(out.size());
      for (const Insn& x : out)
        if (!(x.op == MW_LEAF_N && x.dst >= 0 && x.dst < (int)redrawn.size() && redrawn[x.dst] && u[x.dst] == 0))
          kept.push_back(x);
      out.swap(kept);
    }
    return out;
  }

  std::vector<Insn> fuse_checks(const std::vector<Insn>& in0) {
    std::vector<int> uses = use_counts(in0);
    std::vector<Insn> a1;
    a1.reserve(in0.size());
    for (size_t i = 0; i < in0.size();) {
      const Insn& x = in0[i];
      const Insn* nx = i + 1 < in0.size() ? &in0[i + 1] : nullptr;
      if (x.op == MW_N_ULEN && x.width == 1 && x.dst >= 0 && nx && nx->op == MW_CHECK && nx->ns == 1 &&
          is_def(nx->s[0], x) && uses[x.dst] == 1) {
        Insn c;
        c.op = MW_CHECK_IMP;
        c.width = 1;
        c.ns = x.ns;
        for (int j = 0; j < x.ns; ++j) c.s[j] = x.s[j];
        a1.push_back(c);
        i += 2;
        continue;
      }
      a1.push_back(x);
      i += 1;
    }
    uses = use_counts(a1);
    std::vector<Insn> out;
    out.reserve(a1.size());
    for (size_t i = 0; i < a1.size();) {
      const Insn& x = a1[i];
      const Insn* nx = i + 1 < a1.size() ? &a1[i + 1] : nullptr;
      if ((x.op == MW_N_EQN || x.op == MW_N_EQ) && x.dst >= 0 && nx && nx->op == MW_CHECK_IMP &&
          is_def(nx->s[1], x) && uses[x.dst] == 1) {
        Insn c;
        c.op = x.op == MW_N_EQN ? MW_CHECK_IMPEQ : MW_CHECK_IMPEQW;
        c.width = x.width;
        c.ns = 3;
        c.s[0] = nx->s[0];
        c.s[1] = x.s[0];
        c.s[2] = x.s[1];
        out.push_back(c);
        i += 2;
        continue;
      }
      if (i + 4 <= a1.size()) {
        const Insn &q0 = a1[i], &q1 = a1[i + 1], &q2 = a1[i + 2], &q3 = a1[i + 3];
        bool ok = q0.op == MW_N_SLT && q0.width == 256 && q0.s[0].kind == O_CONST && q0.s[1].kind == O_VREG &&
                  q1.op == MW_LEAF_N && q2.op == MW_N_ITE && is_def(q2.s[0], q1) && q2.s[1].kind == O_CONST &&
                  kv[q2.s[1].v].zero() && is_def(q2.s[2], q0) &&
                  ((q3.op == MW_W_INSN && is_def(q3.s[1], q2)) || (q3.op == MW_W_ZEXTN && is_def(q3.s[0], q2)));
        ok = ok && q0.dst >= 0 && q1.dst >= 0 && q2.dst >= 0 && uses[q0.dst] == 1 && uses[q2.dst] == 1 &&
             q1.imm < (1 << 16);
        if (ok) {
          if (uses[q1.dst] > 1) {   // the leaf has other uses: it stays, W_CDINS draws it again
            Insn l = q1;
            l.cdleaf = true;
            out.push_back(l);
          }
          Opnd acc = q3.op == MW_W_INSN ? q3.s[0] : mkconst(K256{}, 'W');
          long long off = q3.op == MW_W_INSN ? q3.imm : 0;
          Insn c;
          c.op = MW_W_CDINS;
          c.width = q3.width;
          c.dst = q3.dst;
          c.ns = 3;
          c.s[0] = acc;
          c.s[1] = q0.s[1];
          c.s[2] = mkconst(kv[q0.s[0].v], 'W');
          c.imm = q1.imm | (off << 16);
          out.push_back(c);
          i += 4;
          continue;
        }
      }
      out.push_back(x);
      i += 1;
    }
    out = form_grids(fuse_keyed_premises(hoist_cdins_leaves(out)));
    uses = use_counts(out);
    for (size_t i = 0; i + 1 < out.size(); ++i) {
      Insn& a = out[i];
      const Insn& b = out[i + 1];
      if (a.op == MW_W_CDINS && b.op == MW_W_CDINS && a.dst >= 0 && uses[a.dst] == 1 && is_def(b.s[0], a))
        a.chain = true;
    }
    return out;
  }

  // ------------------------------------------------------------------ allocation
  u64 n_spill_words = 0;

  std::vector<Insn> allocate(const std::vector<Insn>& in) {
    size_t nv = vcls.size();
    // uses as CSR lists
    std::vector<int> cnt(nv + 1, 0);
    for (const Insn& x : in)
      for (int j = 0; j < x.ns; ++j)
        if (is_v(x.s[j])) ++cnt[x.s[j].v + 1];
    for (size_t v = 0; v < nv; ++v) cnt[v + 1] += cnt[v];
    std::vector<int> ulist(cnt[nv]);
    std::vector<int> fillp(cnt.begin(), cnt.end() - 1);
    for (size_t i = 0; i < in.size(); ++i)
      for (int j = 0; j < in[i].ns; ++j)
        if (is_v(in[i].s[j])) ulist[fillp[in[i].s[j].v]++] = (int)i;
    std::vector<int> ptr(cnt.begin(), cnt.end() - 1);
    auto next_use = [&](int vid, long long i) -> long long {
      int p = ptr[vid], end = cnt[vid + 1];
      if (p >= end && cnt[vid] == end) return NEVER;
      while (p < end && ulist[p] < i) ++p;
      ptr[vid] = p;
      return p < end ? ulist[p] : NEVER;
    };
    std::vector<int> freeW, freeN;
    for (int s = w_slots - 1; s >= 0; --s)
      if (s != MW_W_RESERVED) freeW.push_back(s);
    for (int s = n_slots - 1; s >= 0; --s)
      if ((s & 31) != MW_N_RESERVED) freeN.push_back(s);
    std::vector<int> reg_of(nv, -1), spill_of(nv, -1);
    // wide leaves are drawn again where they are needed instead of spilled
    // and filled (compiler.py REMAT_LEAVES): remat_def = the defining LEAF_W
    std::vector<int> remat_def(nv, -1);
    std::vector<char> rematted(nv, 0);
    if (remat_leaves())
      for (size_t i = 0; i < in.size(); ++i)
        if (in[i].op == MW_LEAF_W && in[i].dst >= 0) remat_def[in[i].dst] = (int)i;
    std::vector<int> resW, resN;   // insertion-ordered resident vregs (compiler.py dict order)
    std::vector<int> spill_freeW, spill_freeN;
    std::vector<char> slot_cls;
    std::vector<Insn> out;
    out.reserve(in.size() + in.size() / 4);
    auto FREE = [&](int c) -> std::vector<int>& { return c == 'W' ? freeW : freeN; };
    auto RES = [&](int c) -> std::vector<int>& { return c == 'W' ? resW : resN; };
    auto SFREE = [&](int c) -> std::vector<int>& { return c == 'W' ? spill_freeW : spill_freeN; };
    auto erase = [](std::vector<int>& v, int x) {
      auto it = std::find(v.begin(), v.end(), x);
      if (it != v.end()) v.erase(it);
    };
    auto get_spill_slot = [&](int c) -> int {
      std::vector<int>& sf = SFREE(c);
      if (!sf.empty()) {
        int s = sf.back();
        sf.pop_back();
        return s;
      }
      slot_cls.push_back((char)c);
      return (int)slot_cls.size() - 1;
    };
    auto evict = [&](int c, long long i, const int* pinned, int npinned) {
      int best = -1;
      long long best_nu = -1;
      for (int vid : RES(c)) {
        bool pin = false;
        for (int j = 0; j < npinned; ++j) pin = pin || pinned[j] == vid;
        if (pin) continue;
        long long nu = next_use(vid, i);
        if (nu > best_nu) {
          best = vid;
          best_nu = nu;
        }
      }
      if (best < 0) throw Unsupported{"register pressure: too many simultaneous operands"};
      int slot = reg_of[best];
      reg_of[best] = -1;
      erase(RES(c), best);
      if (best_nu < NEVER && remat_def[best] >= 0) {
        rematted[best] = 1;
      } else if (best_nu < NEVER && spill_of[best] < 0) {
        int sp = get_spill_slot(c);
        spill_of[best] = sp;
        Insn m;
        m.op = c == 'W' ? MW_SPILL_W : MW_SPILL_N;
        m.ns = 1;
        m.s[0] = Opnd{O_PHYS, slot};
        m.imm = sp;
        out.push_back(m);
      }
      FREE(c).push_back(slot);
    };
    auto take = [&](int c, long long i, const int* pinned, int npinned) -> int {
      if (FREE(c).empty()) evict(c, i, pinned, npinned);
      std::vector<int>& f = FREE(c);
      int s = f.back();
      f.pop_back();
      return s;
    };
    for (size_t i = 0; i < in.size(); ++i) {
      const Insn& x = in[i];
      int pinned[3], np = 0;
      for (int j = 0; j < x.ns; ++j)
        if (is_v(x.s[j])) pinned[np++] = x.s[j].v;
      for (int j = 0; j < x.ns; ++j) {
        const Opnd& s = x.s[j];
        if (is_v(s) && reg_of[s.v] < 0 && rematted[s.v]) {
          int c = vcls[s.v];
          int slot = take(c, (long long)i, pinned, np);
          Insn r = in[remat_def[s.v]];
          r.dst = slot;
          out.push_back(r);
          reg_of[s.v] = slot;
          RES(c).push_back(s.v);
          continue;
        }
        if (is_v(s) && reg_of[s.v] < 0) {
          if (spill_of[s.v] < 0) throw BadInput{"use of undefined vreg"};
          int c = vcls[s.v];
          int slot = take(c, (long long)i, pinned, np);
          Insn f;
          f.op = c == 'W' ? MW_FILL_W : MW_FILL_N;
          f.dst = slot;
          f.imm = spill_of[s.v];
          out.push_back(f);
          reg_of[s.v] = slot;
          RES(c).push_back(s.v);
        }
      }
      Insn y = x;
      for (int j = 0; j < x.ns; ++j)
        if (is_v(x.s[j])) y.s[j] = Opnd{O_PHYS, reg_of[x.s[j].v]};
      for (int j = 0; j < x.ns; ++j) {
        const Opnd& s = x.s[j];
        if (is_v(s) && reg_of[s.v] >= 0 && next_use(s.v, (long long)i + 1) >= NEVER) {
          int c = vcls[s.v];
          int slot = reg_of[s.v];
          reg_of[s.v] = -1;
          erase(RES(c), s.v);
          FREE(c).push_back(slot);
          if (spill_of[s.v] >= 0) {
            SFREE(c).push_back(spill_of[s.v]);
            spill_of[s.v] = -1;
          }
        }
      }
      y.dst = -1;
      if (x.dst >= 0) {
        int c = vcls[x.dst];
        int slot = take(c, (long long)i, nullptr, 0);
        if (next_use(x.dst, (long long)i + 1) < NEVER) {
          reg_of[x.dst] = slot;
          RES(c).push_back(x.dst);
        } else {
          FREE(c).push_back(slot);   // dead result (e.g. traced only): slot reused
        }
        y.dst = slot;
      }
      out.push_back(y);
    }
    // spill slot layout: the grid tables first (form_grids' words), then the
    // slots, most accesses per word first (compiler.py _layout_spills)
    long long tables = 0;
    for (const Insn& x : out)
      if (x.grid) tables = std::max(tables, x.imm + 1);
    n_spill_words = (u64)tables;
    auto slot_op = [](const Insn& x) {
      return !x.grid && (x.op == MW_SPILL_W || x.op == MW_SPILL_N || x.op == MW_FILL_W || x.op == MW_FILL_N);
    };
    if (!slot_cls.empty()) {
      size_t ns = slot_cls.size();
      std::vector<long long> hits(ns, 0);
      for (const Insn& x : out)
        if (slot_op(x)) ++hits[x.imm];
      std::vector<int> order(ns);
      for (size_t q = 0; q < ns; ++q) order[q] = (int)q;
      auto size = [&](int q) -> long long { return slot_cls[q] == 'W' ? 8 : 1; };
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        long long l = hits[a] * size(b), r = hits[b] * size(a);   // -hits/size ascending
        if (l != r) return l > r;
        return a < b;
      });
      std::vector<long long> off(ns, 0);
      long long words = tables;
      for (int q : order) {
        off[q] = words;
        words += size(q);
      }
      for (Insn& x : out)
        if (slot_op(x)) x.imm = off[x.imm];
      n_spill_words = (u64)words;
    }
    return out;
  }

  // ------------------------------------------------------------------ driver
  std::vector<u32> code, consts, leaves_out, trace_out;
  u64 n_trace_rows = 0, ops = 0, div_nominal = 0, n_div = 0, n_spills = 0, n_fills = 0;

  static u32 encode_dst(int cls, int slot) {
    u32 w = MW_W_RESERVED, lo = MW_N_RESERVED, hi = MW_N_RESERVED;
    if (cls == 'W') w = (u32)slot;
    else if (cls == 'N') {
      if (slot < 32) lo = (u32)slot;
      else hi = (u32)(slot - 32);
    }
    return w | (lo << 3) | (hi << 8);
  }

  void run(const int32_t* roots, size_t nconj, size_t ntrace) {
    size_t nn = nodes.size();
    in_memo.assign(nn, 0);
    memo.assign(nn, Opnd{});
    memo_scope.assign(nn, -1);
    memo_at.assign(nn, 0);
    trace_req.assign(nn, 0);
    trace_emitted.assign(nn, 0);
    cost.resize(nn);
    for (size_t i = 0; i < nn; ++i) cost[i] = node_cost((int)i);
    for (size_t t = 0; t < ntrace; ++t) trace_req[roots[nconj + t]] = 1;
    for (size_t c = 0; c < nconj; ++c) {
      ++scope;
      int r = roots[c];
      if (N(r).op == IR_CONST && node_val(r).zero()) {
        Opnd z = ksmall(0, 1);
        emit_void(MW_CHECK, 1, {z});
        continue;
      }
      Opnd v = lower(r);
      emit_void(MW_CHECK, 1, {v});
    }
    for (size_t t = 0; t < ntrace; ++t) lower(roots[nconj + t]);
    emit_void(MW_END, 0, {});

    std::vector<Insn> fin = allocate(fuse_checks(schedule_narrow_early(insns)));

    // encode: constant pool in first-reference order
    std::map<std::pair<char, K256>, u32> kmap;
    auto kref = [&](int ki) -> u32 {
      std::pair<char, K256> key(kc[ki], kv[ki]);
      auto it = kmap.find(key);
      if (it != kmap.end()) return MW_KBIT | it->second;
      u32 at = (u32)consts.size();
      kmap.emplace(key, at);
      if (kc[ki] == 'W')
        for (int q = 0; q < 8; ++q) consts.push_back(kv[ki].l[q]);
      else
        consts.push_back(kv[ki].l[0]);
      return MW_KBIT | at;
    };
    u64 rows = 0;
    code.reserve(4 * fin.size());
    for (size_t q = 0; q < fin.size(); ++q) {
      const Insn& x = fin[q];
      u32 f[3] = {0, 0, 0};
      for (int j = 0; j < x.ns; ++j) f[j] = x.s[j].kind == O_CONST ? kref(x.s[j].v) : (u32)x.s[j].v;
      long long imm = x.imm;
      if (x.op == MW_STORE_W || x.op == MW_STORE_N) {
        bool wide = x.op == MW_STORE_W;
        trace_out.push_back((u32)imm);
        trace_out.push_back((u32)rows);
        trace_out.push_back(wide ? 1u : 0u);
        imm = (long long)rows;
        rows += wide ? 8 : 1;
      }
      int dc = x.dst >= 0 ? dst_cls(x.op) : 0;
      u32 dst = encode_dst(dc, x.dst >= 0 ? x.dst : 0);
      const Insn* nx = q + 1 < fin.size() ? &fin[q + 1] : nullptr;
      u32 flags = (x.chain && nx && nx->op == MW_W_CDINS && nx->ns && nx->s[0].kind == O_PHYS &&
                   x.dst >= 0 && nx->s[0].v == x.dst) ? 1u : 0u;
      code.push_back((u32)(x.op & 0xff) | ((flags & 0xff) << 8) | (((u32)x.width & 0xffff) << 16));
      code.push_back((dst & 0xffff) | ((f[0] & 0xffff) << 16));
      code.push_back((f[1] & 0xffff) | ((f[2] & 0xffff) << 16));
      code.push_back((u32)(imm & 0xffffffffLL));
      if ((x.op == MW_SPILL_W || x.op == MW_SPILL_N) && !x.grid) ++n_spills;
      if (x.op == MW_FILL_W || x.op == MW_FILL_N) ++n_fills;
    }
    if (consts.size() > 0x7fff) throw Unsupported{"constant pool overflow"};
    n_trace_rows = rows;
    for (int li : leaf_nodes) leaves_out.push_back((u32)li);
    for (size_t i = 0; i < nn; ++i) {
      ops += (u64)cost[i];
      const Node& n = N((int)i);
      if ((n.op == IR_BVUDIV || n.op == IR_BVUREM || n.op == IR_BVSDIV || n.op == IR_BVSREM || n.op == IR_BVSMOD) &&
          n.w() > NARROW_MAX) {
        int L = (n.w() + 31) / 32;
        bool sg = n.op == IR_BVSDIV || n.op == IR_BVSREM || n.op == IR_BVSMOD;
        div_nominal += (u64)(cost[i] - (sg ? 4 * L : 0));
        ++n_div;
      }
    }
  }
};

}  // namespace

struct mw_compiled {
  std::vector<u32> code, consts, leaves, trace;
};

extern "C" {

int mw_compile_slots(const int32_t* recs, size_t nrecs_words, size_t nnodes, const uint8_t* kvals, size_t nkvals,
                     const int32_t* roots, size_t nconj, size_t ntrace, uint32_t w_slots, uint32_t n_slots,
                     mw_compiled** out, mw_compile_info* info) {
  if (!out || !info || (nnodes && !recs) || ((nconj + ntrace) && !roots))
    return mw_fail(MG_E_ARG, "mw_compile: null argument");
  *out = nullptr;
  if (w_slots < 4 || w_slots > MW_NW || n_slots < 8 || n_slots > MW_NN)
    return mw_fail(MG_E_ARG, "mw_compile: register slots out of range");
  try {
    Compiler c;
    c.w_slots = (int)w_slots;
    c.n_slots = (int)n_slots;
    c.kvals = kvals;
    c.nkvals = nkvals;
    c.nodes.reserve(nnodes);
    size_t at = 0;
    for (size_t i = 0; i < nnodes; ++i) {
      if (at + 6 > nrecs_words) throw BadInput{"record stream truncated"};
      Node n;
      n.op = recs[at];
      n.width = recs[at + 1];
      n.flags = recs[at + 2];
      n.p0 = recs[at + 3];
      n.p1 = recs[at + 4];
      n.nargs = recs[at + 5];
      if (n.op < -1 || n.op >= IR_NOPS || n.width < 0 || n.nargs < 0 || at + 6 + (size_t)n.nargs > nrecs_words)
        throw BadInput{"bad node record " + std::to_string(i)};
      n.args = recs + at + 6;
      for (int j = 0; j < n.nargs; ++j)
        if (n.args[j] < 0 || (size_t)n.args[j] >= i) throw BadInput{"operand after its user at record " + std::to_string(i)};
      if (n.op == IR_CONST && (n.p0 < 0 || (size_t)n.p0 >= nkvals)) throw BadInput{"constant value index out of range"};
      if (n.op == IR_EXTRACT && (n.nargs != 1 || n.p1 < 0 || n.p0 < n.p1)) throw BadInput{"bad extract record"};
      if ((n.op == IR_REPEAT || n.op == IR_ROTATE_LEFT || n.op == IR_ROTATE_RIGHT) && (n.nargs != 1 || n.p0 < 0))
        throw BadInput{"bad parameter record"};
      c.nodes.push_back(n);
      at += 6 + (size_t)n.nargs;
    }
    for (size_t r = 0; r < nconj + ntrace; ++r)
      if (roots[r] < 0 || (size_t)roots[r] >= nnodes) throw BadInput{"root out of range"};
    c.run(roots, nconj, ntrace);
    mw_compiled* res = new mw_compiled;
    res->code.swap(c.code);
    res->consts.swap(c.consts);
    res->leaves.swap(c.leaves_out);
    res->trace.swap(c.trace_out);
    memset(info, 0, sizeof *info);
    info->ncode_words = res->code.size();
    info->nconst_words = res->consts.size();
    info->nleaves = res->leaves.size();
    info->ntrace = res->trace.size() / 3;
    info->n_spill = c.n_spill_words;
    info->n_trace_rows = c.n_trace_rows;
    info->ops_per_eval = c.ops;
    info->div_nominal_ops = c.div_nominal;
    info->n_nodes = nnodes;
    info->n_div = c.n_div;
    info->n_spills = c.n_spills;
    info->n_fills = c.n_fills;
    *out = res;
    return 0;
  } catch (const Unsupported& e) {
    return mw_fail(MG_E_ARG, ("unsupported: " + e.msg).c_str());
  } catch (const BadInput& e) {
    return mw_fail(MG_E_PROG, ("mw_compile: " + e.msg).c_str());
  } catch (const std::bad_alloc&) {
    return mw_fail(MG_E_NOMEM, "mw_compile: out of host memory");
  }
}

int mw_compile(const int32_t* recs, size_t nrecs_words, size_t nnodes, const uint8_t* kvals, size_t nkvals,
               const int32_t* roots, size_t nconj, size_t ntrace, mw_compiled** out, mw_compile_info* info) {
  return mw_compile_slots(recs, nrecs_words, nnodes, kvals, nkvals, roots, nconj, ntrace, MW_NW, MW_NN, out, info);
}

int mw_compiled_take(mw_compiled* r, uint32_t* code, uint32_t* consts, uint32_t* leaves, uint32_t* trace) {
  if (!r) return mw_fail(MG_E_ARG, "mw_compiled_take: null result");
  if (code && !r->code.empty()) memcpy(code, r->code.data(), 4 * r->code.size());
  if (consts && !r->consts.empty()) memcpy(consts, r->consts.data(), 4 * r->consts.size());
  if (leaves && !r->leaves.empty()) memcpy(leaves, r->leaves.data(), 4 * r->leaves.size());
  if (trace && !r->trace.empty()) memcpy(trace, r->trace.data(), 4 * r->trace.size());
  delete r;
  return 0;
}

void mw_compiled_free(mw_compiled* r) { delete r; }

}  // extern "C"
