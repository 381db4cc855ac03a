"""ORACLE (test infrastructure only): ctypes binding of oracle/c/dag_oracle.c.

Serialises an IR DAG into the C oracle's own node format (binary ops only:
n-ary terms are folded, comparisons normalised) and evaluates candidate
ranges on all host cores with OpenMP.  Leaves are Philox draws keyed by
crc32(name), the same candidate space the engine searches.
"""
from __future__ import annotations

import ctypes
import os
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None

OPS = ["CONST", "VAR", "ADD", "SUB", "MUL", "UDIV", "UREM", "SDIV", "SREM", "SMOD", "AND", "OR", "XOR",
       "NOT", "NEG", "SHL", "LSHR", "ASHR", "CONCAT", "EXTRACT", "ZEXT", "SEXT", "ITE", "EQ", "ULT", "ULE",
       "SLT", "SLE", "UMULNO", "ROTL", "ROTR", "ADDC"]
O = {n: i for i, n in enumerate(OPS)}


def available() -> bool:
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        if not available():
            subprocess_build()
        L = ctypes.CDLL(LIB)
        L.odag_eval.restype = ctypes.c_longlong
        L.odag_eval.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_uint64)]
        L.odag_eval_spec.restype = ctypes.c_longlong
        L.odag_eval_spec.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_uint64)]
        L.odag_div_paths.restype = ctypes.c_longlong
        L.odag_div_paths.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.odag_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def subprocess_build():
    import subprocess
    subprocess.run(["make", "-C", HERE], check=True, capture_output=True)


class Serialized:
    def __init__(self, specs=None):
        self.nodes = []     # [op, w, a, b, c, p0, p1, salt]
        self.consts = []    # 8-limb entries
        self.memo = {}
        self.kmemo = {}
        self.specs_in = specs or {}   # var name -> candidate spec (oracle/philox.py leaf_value fields)
        self.spec_rows = []           # [kind, shift, bits, stride, pool word offset]
        self.pool = []

    def _spec_index(self, name: str) -> int:
        """Spec row of a leaf: the candidate-space definition of oracle/philox.py
        (pool digits from index bit-fields, interleaved bits or a hash; RANDOM
        entries fall back to Philox), restated for the C oracle."""
        sp = self.specs_in.get(name)
        if not sp or not sp.get("pool"):
            return -1
        pool = list(sp["pool"])
        kind = 2 if sp.get("hashed") else (3 if sp.get("stride") else 1)
        off = len(self.pool)
        for e in pool:
            if e is None:
                self.pool.extend([1] + [0] * 8)
            else:
                self.pool.extend([0] + [(e >> (32 * k)) & 0xFFFFFFFF for k in range(8)])
        self.spec_rows.append([kind, sp.get("shift", 0), sp.get("bits", 0), sp.get("stride", 0), off])
        return len(self.spec_rows) - 1

    def _add(self, op, w, a=-1, b=-1, c=-1, p0=0, p1=0, salt=0):
        self.nodes.append([O[op], w, a, b, c, p0, p1, salt - (1 << 32) if salt >= (1 << 31) else salt])
        return len(self.nodes) - 1

    def const(self, v, w):
        key = (v, w)
        if key not in self.kmemo:
            idx = len(self.consts)
            self.consts.append([(v >> (32 * k)) & 0xFFFFFFFF for k in range(8)])
            self.kmemo[key] = self._add("CONST", w, p0=idx)
        return self.kmemo[key]

    def fold(self, op, w, xs):
        acc = xs[0]
        for x in xs[1:]:
            acc = self._add(op, w, acc, x)
        return acc

    def term(self, n) -> int:
        if n.id in self.memo:
            return self.memo[n.id]
        r = self._term(n)
        self.memo[n.id] = r
        return r

    def _term(self, n) -> int:
        op = n.op
        w = 1 if n.width == 0 else n.width
        if w > 256:
            raise ValueError("C oracle handles widths <= 256")
        if op == "const":
            return self.const(n.val, w)
        if op == "var":
            sp = self.specs_in.get(n.name)
            salt = sp["id"] if sp and "id" in sp else zlib.crc32(n.name.encode()) & 0xFFFFFFFF
            return self._add("VAR", w, p0=self._spec_index(n.name), salt=salt)
        a = [self.term(x) for x in n.args]
        aw = (1 if n.args[0].width == 0 else n.args[0].width) if n.args else w
        simple = {"bvsub": "SUB", "bvudiv": "UDIV", "bvurem": "UREM", "bvsdiv": "SDIV", "bvsrem": "SREM",
                  "bvsmod": "SMOD", "bvshl": "SHL", "bvlshr": "LSHR", "bvashr": "ASHR"}
        nary = {"bvadd": "ADD", "bvmul": "MUL", "bvand": "AND", "bvor": "OR", "bvxor": "XOR",
                "and": "AND", "or": "OR", "xor": "XOR"}
        if op in simple:
            return self._add(simple[op], w, a[0], a[1])
        if op in nary:
            return self.fold(nary[op], w, a)
        if op in ("bvnot", "not"):
            return self._add("NOT", w, a[0])
        if op == "bvneg":
            return self._add("NEG", w, a[0])
        if op in ("bvnand", "bvnor", "bvxnor"):
            inner = {"bvnand": "AND", "bvnor": "OR", "bvxnor": "XOR"}[op]
            return self._add("NOT", w, self._add(inner, w, a[0], a[1]))
        if op == "=>":
            return self._add("OR", 1, self._add("NOT", 1, a[0]), a[1])
        if op == "concat":
            acc, accw = a[0], (1 if n.args[0].width == 0 else n.args[0].width)
            for x, xn in zip(a[1:], n.args[1:]):
                accw += xn.width
                acc = self._add("CONCAT", accw, acc, x)
            return acc
        if op == "repeat":
            acc, accw = a[0], aw
            for _ in range(n.params[0] - 1):
                accw += aw
                acc = self._add("CONCAT", accw, acc, a[0])
            return acc
        if op == "extract":
            return self._add("EXTRACT", w, a[0], p0=n.params[0], p1=n.params[1])
        if op == "zero_extend":
            return self._add("ZEXT", w, a[0])
        if op == "sign_extend":
            return self._add("SEXT", w, a[0])
        if op in ("rotate_left", "rotate_right"):
            return self._add("ROTL" if op == "rotate_left" else "ROTR", w, a[0], p0=n.params[0])
        if op == "ite":
            return self._add("ITE", w, a[0], a[1], a[2])
        if op in ("=", "bvcomp"):
            eqs = [self._add("EQ", 1, a[0], x) for x in a[1:]]
            return self.fold("AND", 1, eqs)
        if op == "distinct":
            ne = [self._add("NOT", 1, self._add("EQ", 1, a[i], a[j]))
                  for i in range(len(a)) for j in range(i + 1, len(a))]
            return self.fold("AND", 1, ne)
        cmp = {"bvult": ("ULT", 0), "bvule": ("ULE", 0), "bvugt": ("ULT", 1), "bvuge": ("ULE", 1),
               "bvslt": ("SLT", 0), "bvsle": ("SLE", 0), "bvsgt": ("SLT", 1), "bvsge": ("SLE", 1)}
        if op in cmp:
            o, sw = cmp[op]
            x, y = (a[1], a[0]) if sw else (a[0], a[1])
            return self._add(o, 1, x, y)
        if op == "bvumul_noovfl":
            return self._add("UMULNO", 1, a[0], a[1])
        if op == "bvaddc":
            return self._add("ADDC", 1, a[0], a[1])
        raise ValueError(f"C oracle: unsupported op {op}")


def program_specs(prog) -> dict:
    """Candidate specs of a compiled program's leaves in oracle/philox.py's form
    (the fields the oracle restates; not the program's encoded leaf table)."""
    out = {}
    for node, sp in zip(prog.leaf_nodes, prog.leaf_specs):
        out[node.name] = {"id": sp.key_salt(), "width": sp.width, "shift": sp.shift, "bits": sp.bits,
                          "pool": sp.pool, "hashed": sp.hashed, "stride": sp.stride}
    return out


def evaluate(conjuncts, seed: int, begin: int, n: int, nthreads: int = 0, want_verdict: bool = False,
             specs=None):
    """Evaluate candidates [begin, begin+n) of the conjunction on all host cores.
    specs: {var name: oracle/philox.py spec} (e.g. program_specs(prog)) for
    pool-driven leaves; leaves without one are plain Philox draws."""
    s = Serialized(specs)
    roots = [s.term(c) for c in conjuncts]
    nodes = np.asarray(s.nodes, dtype=np.int32).reshape(-1)
    consts = np.asarray(s.consts or [[0] * 8], dtype=np.uint32).reshape(-1)
    r = np.asarray(roots or [0], dtype=np.int32)
    v = np.zeros(n, dtype=np.uint8) if want_verdict else None
    first = ctypes.c_uint64(0)
    if s.spec_rows:
        sp = np.asarray(s.spec_rows, dtype=np.int32).reshape(-1)
        pool = np.asarray(s.pool, dtype=np.uint32)
        total = lib().odag_eval_spec(nodes.ctypes.data, len(s.nodes), consts.ctypes.data, r.ctypes.data,
                                     len(roots), sp.ctypes.data, pool.ctypes.data, seed, begin, n,
                                     v.ctypes.data if v is not None else None, nthreads, ctypes.byref(first))
    else:
        total = lib().odag_eval(nodes.ctypes.data, len(s.nodes), consts.ctypes.data, r.ctypes.data, len(roots),
                                seed, begin, n, v.ctypes.data if v is not None else None, nthreads,
                                ctypes.byref(first))
    return total, (None if first.value == (1 << 64) - 1 else first.value), v


def div_paths(conjuncts, seed: int, begin: int, n: int, wave: int = 64, nthreads: int = 0, specs=None):
    """Division path counts of the product's kernels, restated from udivrem8's
    documented per-wave rules (dag_oracle.c odag_div_paths): a dict in
    mg_stats' names (lane_div_steps / _full / _short / _general, each x lanes)
    for candidates [begin, begin+n) in waves of `wave` consecutive indices."""
    s = Serialized(specs)
    for c in conjuncts:
        s.term(c)
    nodes = np.asarray(s.nodes, dtype=np.int32).reshape(-1)
    consts = np.asarray(s.consts or [[0] * 8], dtype=np.uint32).reshape(-1)
    sp = np.asarray(s.spec_rows or [[0] * 5], dtype=np.int32).reshape(-1)
    pool = np.asarray(s.pool or [0], dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint64)
    lib().odag_div_paths(nodes.ctypes.data, len(s.nodes), consts.ctypes.data,
                         sp.ctypes.data if s.spec_rows else None, pool.ctypes.data, seed, begin, n, wave, nthreads,
                         out.ctypes.data)
    return {"lane_div_steps": int(out[0]), "lane_div_full": int(out[1]), "lane_div_short": int(out[2]),
            "lane_div_general": int(out[3])}


def baseline(syn, prog, budget_s: float = 10.0, verdicts: bool = False):
    """bench.py cpu_baseline: all host cores, candidate indices 0.. in growing
    batches.  verdicts=True also returns the per-candidate verdict vector (the
    bench compares it with the GPU's on the same indices)."""
    cores = lib().odag_max_threads()
    n, t0, dt, sat = 0, time.perf_counter(), 0.0, 0
    batch = max(64, cores * 16)
    parts = []
    while dt < budget_s:
        tot, _, v = evaluate(syn.conjuncts, syn.seed, n, batch, want_verdict=verdicts)
        if verdicts:
            parts.append(v)
        sat += tot
        n += batch
        dt = time.perf_counter() - t0
        if dt < budget_s / 4:
            batch *= 2
    out = {"value": n / dt, "unit": "evals/s", "cores": cores, "kind": "port",
           "sample": f"candidate indices 0..{n - 1} of the same C5 program ({n} evals, {dt:.1f} s), "
                     f"C restatement oracle/c/dag_oracle.c, OpenMP x{cores}", "satisfied": int(sat)}
    if verdicts:
        return out, np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
    return out
