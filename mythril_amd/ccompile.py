"""The native host compiler (``csrc/mw_compile.cpp``, ``include/mythril_compile.h``).

``compile_native`` produces exactly the :class:`~mythril_amd.compiler.Program`
that :func:`~mythril_amd.compiler.compile_program` produces (same bytecode,
constant pool, leaf table, pools, trace rows and op counts;
tests/test_native_compile.py checks both corpora and random DAGs) with the
lowering, scheduling, fusion, register allocation and encoding done in C++.
The DAG crosses as one int32 record stream (operand-first order) plus the
256-bit constant values; the leaf table and pools are laid out here
(``layout_leaves``, shared with the Python compiler).

The Python compiler stays as the parity reference and as the source of the
SSA machine IR the specialised kernels are generated from (``jit.py``): a
natively compiled program builds it on first use (``Program.machine_ir``).

``prepare`` (engine.py) compiles every get_model query here (VERDICT r3
item 2: the Python passes were half of the host cost per query).
``MYTHRIL_AMD_PY_COMPILE=1`` selects the Python compiler instead.
"""
from __future__ import annotations

import ctypes
import os
import threading
from array import array
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .compiler import LeafSpec, Program, Unsupported, _flatten, compile_program, layout_leaves
from .ir import Node, topo

# record op codes: the order of csrc/mw_compile.cpp enum IrOp
IR_OPS = [
    "const", "var", "array", "apply", "select", "store", "const_array",
    "and", "or", "not", "xor", "=>", "=", "distinct",
    "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
    "bvumul_noovfl", "bvsmul_noovfl", "bvsmul_noudfl", "bvaddc", "ite",
    "bvadd", "bvmul", "bvand", "bvor", "bvxor", "concat", "bvsub",
    "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvshl", "bvlshr", "bvashr",
    "bvnand", "bvnor", "bvxnor", "bvcomp", "bvneg", "bvnot",
    "extract", "zero_extend", "sign_extend", "repeat", "rotate_left", "rotate_right",
]
_OPC = {op: i for i, op in enumerate(IR_OPS)}
_CONST, _VAR = _OPC["const"], _OPC["var"]
_M256 = (1 << 256) - 1
MG_E_ARG = -1


class MwCompileInfo(ctypes.Structure):
    """include/mythril_compile.h mw_compile_info"""
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "ncode_words", "nconst_words", "nleaves", "ntrace", "n_spill", "n_trace_rows", "ops_per_eval",
        "div_nominal_ops", "n_nodes", "n_div", "n_spills", "n_fills")]


_P = ctypes.c_void_p
_fns = None
_why: Optional[str] = None
_lock = threading.Lock()


def _bind():
    """The three entry points of the product library, bound once; None (with
    the reason in why_unavailable()) when the library is not built."""
    global _fns, _why
    if _fns is None and _why is None:
        with _lock:
            if _fns is None and _why is None:
                from .runtime import EngineUnavailable, load_library
                try:
                    lib = load_library()
                    c, t, f = lib.mw_compile_slots, lib.mw_compiled_take, lib.mw_compiled_free
                except (EngineUnavailable, AttributeError) as e:
                    _why = str(e)
                    return None
                c.restype, c.argtypes = ctypes.c_int, [_P, ctypes.c_size_t, ctypes.c_size_t, _P, ctypes.c_size_t,
                                                       _P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                                                       ctypes.c_uint32, ctypes.POINTER(_P),
                                                       ctypes.POINTER(MwCompileInfo)]
                t.restype, t.argtypes = ctypes.c_int, [_P, _P, _P, _P, _P]
                f.restype, f.argtypes = None, [_P]
                _fns = (lib, c, t, f)
    return _fns


def available() -> bool:
    return _bind() is not None


def why_unavailable() -> Optional[str]:
    _bind()
    return _why


def serialize(conj: Sequence[Node], trace: Sequence[Node], nodes: Optional[List[Node]] = None,
              memo: Optional[dict] = None):
    """(records, number of nodes, constant bytes, roots, nodes): the DAG below
    the (flattened) conjuncts and traced terms in the mythril_compile.h
    format, operand-first (``topo`` order, the node set compile_program
    counts ops over; `nodes` when the caller has that walk already).
    memo: an operation node's record head by node id, kept with a long-lived
    context (the head depends on the node alone; operand indices do not)."""
    if nodes is None:
        nodes = topo(list(conj) + list(trace))
    idx: Dict[int, int] = {}
    recs: List[int] = []
    kb = bytearray()
    names: Dict[str, int] = {}
    nk = 0
    ext, put, opc = recs.extend, recs.append, _OPC.get
    hget = memo.get if memo is not None else None
    for i, n in enumerate(nodes):
        idx[n.id] = i
        op = n.op
        if op == "const":
            kb += (n.val & _M256).to_bytes(32, "little")
            ext((_CONST, n.width, 0, nk, 0, 0))
            nk += 1
            continue
        if op == "var":
            nid = names.get(n.name)
            if nid is None:
                nid = names[n.name] = len(names)
            ext((_VAR, n.width, 0 if n.dom is None else 1, nid, 0, 0))
            continue
        args = n.args
        na = len(args)
        h = hget(n.id) if hget is not None else None
        if h is None:
            pr = n.params
            if pr:
                h = (opc(op, -1), n.width, 0 if n.dom is None else 1, pr[0], pr[1] if len(pr) > 1 else 0, na)
            else:
                h = (opc(op, -1), n.width, 0 if n.dom is None else 1, 0, 0, na)
            if memo is not None:
                memo[n.id] = h
        ext(h)
        if na == 2:   # the common arities without a comprehension
            a, b = args
            ext((idx[a.id], idx[b.id]))
        elif na == 1:
            put(idx[args[0].id])
        elif na:
            ext([idx[a.id] for a in args])
    roots = [idx[c.id] for c in conj] + [idx[t.id] for t in trace]
    return array("i", recs), len(nodes), bytes(kb), nk, array("i", roots), nodes, idx, names


def _addr(buf) -> int:
    return ctypes.addressof(ctypes.c_char.from_buffer(buf)) if len(buf) else 0


def compile_native(conjuncts: Sequence[Node], leaf_specs: Optional[Dict[str, LeafSpec]] = None,
                   trace: Sequence[Node] = (), pools: Optional[Dict[str, List[Optional[int]]]] = None,
                   reach=None, slots: Optional[Tuple[int, int]] = None, memo: Optional[dict] = None) -> Program:
    """compile_program(conjuncts, leaf_specs, trace, pools, slots), natively.
    reach: (flattened conjuncts, their topo) when the caller has them and
    nothing is traced (prepare: Lowered.flat, Lowered.nodes).  memo: a
    long-lived context's record heads (serialize)."""
    fns = _bind()
    if fns is None:
        raise RuntimeError(f"native compiler unavailable: {_why}")
    trace = list(trace)
    if reach is not None and not trace:
        conj, nodes = reach
        recs, nn, kb, nk, roots, nodes, idx, names = serialize(conj, trace, nodes, memo)
    else:
        conj = _flatten(conjuncts)
        recs, nn, kb, nk, roots, nodes, idx, names = serialize(conj, trace)
    info, code, consts, leaves, tr = _run(fns, recs, nn, kb, nk, roots, len(conj), len(trace), slots)
    leaf_nodes = [nodes[i] for i in leaves.tolist()]
    specs, leaf_words, pool_words, in_row = layout_leaves(leaf_nodes, leaf_specs, pools,
                                                          memo.setdefault("_pools", {}) if memo is not None else None)
    t = tr.tolist()
    trace_map = {nodes[t[k]].id: (t[k + 1], "W" if t[k + 2] else "N") for k in range(0, len(t), 3)}
    n_insn = int(info.ncode_words) // 4
    return Program(code=code, consts=consts if consts.size else np.zeros(1, dtype=np.uint32),
                   leaves=np.frombuffer(array("I", leaf_words), dtype=np.uint32),
                   pool=pool_words if pool_words.size else np.zeros(1, dtype=np.uint32),
                   n_spill=int(info.n_spill), n_trace_rows=int(info.n_trace_rows), n_input_rows=in_row,
                   ops_per_eval=int(info.ops_per_eval), leaf_specs=specs, leaf_nodes=leaf_nodes,
                   trace_map=trace_map, n_insn=n_insn, n_conjuncts=len(conj), stats=_stats(info, n_insn),
                   ssa_build=lambda: compile_program(conj, trace=trace, slots=slots).ssa,
                   native_dag=(recs, nn, kb, nk, nodes, idx, names))


def _stats(info, n_insn):
    return {"nodes": int(info.n_nodes), "insns": n_insn, "spills": int(info.n_spills), "fills": int(info.n_fills),
            "div_nominal_ops": int(info.div_nominal_ops), "wide_divisions": int(info.n_div)}


def _run(fns, recs, nn, kb, nk, roots, nconj, ntrace, slots=None):
    """One mw_compile_slots call: (info, code, consts, leaf record indices, trace triples)."""
    lib, c_compile, c_take, c_free = fns
    kbuf = ctypes.create_string_buffer(kb, len(kb)) if kb else None
    h = _P()
    info = MwCompileInfo()
    nw, nsl = slots or (isa.NW, isa.NN)
    rc = c_compile(_addr(recs), len(recs), nn, kbuf, nk, _addr(roots), nconj, ntrace, nw, nsl,
                   ctypes.byref(h), ctypes.byref(info))
    if rc != 0:
        msg = (lib.mg_last_error() or b"").decode()
        if rc == MG_E_ARG and msg.startswith("unsupported"):
            raise Unsupported(msg)
        raise RuntimeError(f"mw_compile failed ({rc}): {msg}")
    code = np.empty(info.ncode_words, dtype=np.uint32)
    consts = np.empty(info.nconst_words, dtype=np.uint32)
    leaves = np.empty(info.nleaves, dtype=np.uint32)
    tr = np.empty(3 * info.ntrace, dtype=np.uint32)
    ptr = lambda a: a.ctypes.data if a.size else None   # noqa: E731
    if c_take(h, ptr(code), ptr(consts), ptr(leaves), ptr(tr)) != 0:
        c_free(h)
        raise RuntimeError("mw_compiled_take failed")
    return info, code, consts, leaves, tr


def _outside(roots: Sequence[Node], idx: Dict[int, int]) -> List[Node]:
    """The nodes below roots that idx does not hold, operand-first."""
    out: List[Node] = []
    seen = set()
    for r in roots:
        if r.id in idx or r.id in seen:
            continue
        stack = [(r, False)]
        while stack:
            n, done = stack.pop()
            if done:
                out.append(n)
                continue
            if n.id in idx or n.id in seen:
                continue
            seen.add(n.id)
            stack.append((n, True))
            for a in reversed(n.args):
                if a.id not in idx and a.id not in seen:
                    stack.append((a, False))
    return out


def _serialize_more(extra: Sequence[Node], idx: Dict[int, int], names: Dict[str, int], start: int, nk: int):
    """serialize's records for `extra` (operand-first; operands in idx or
    earlier in extra), numbered from `start`: (records, constant bytes,
    constant count, {node id: record index})."""
    local: Dict[int, int] = {}
    recs: List[int] = []
    kb = bytearray()
    new_names: Dict[str, int] = {}
    ext = recs.extend

    def at(a):
        i = local.get(a.id)
        return idx[a.id] if i is None else i
    for j, n in enumerate(extra):
        local[n.id] = start + j
        op = n.op
        if op == "const":
            kb += (n.val & _M256).to_bytes(32, "little")
            ext((_CONST, n.width, 0, nk, 0, 0))
            nk += 1
            continue
        if op == "var":
            nid = names.get(n.name)
            if nid is None:
                nid = new_names.get(n.name)
                if nid is None:
                    nid = new_names[n.name] = len(names) + len(new_names)
            ext((_VAR, n.width, 0 if n.dom is None else 1, nid, 0, 0))
            continue
        pr = n.params
        ext((_OPC.get(op, -1), n.width, 0 if n.dom is None else 1, pr[0] if pr else 0,
             pr[1] if len(pr) > 1 else 0, len(n.args)))
        ext([at(a) for a in n.args])
    return recs, bytes(kb), nk, local


def compile_trace_native(prog: Program, trace: Sequence[Node]) -> Optional[Program]:
    """The witness program of a natively compiled `prog` (no conjuncts,
    `trace` traced, its leaves first in prog's order), compiled from prog's
    own record stream: no second serialisation, and prog's leaf table and
    pools as they are.  Code generation starts from the roots only, so the
    program is the one compile_native(trace=trace) makes; its ops_per_eval
    counts the whole stream (a witness launch is one candidate).  Traced
    terms outside the stream (cell indices no conjunct reads) get their
    records appended.  None when the leaves come out in another order: the
    caller compiles it afresh."""
    dag = prog.native_dag
    fns = _bind()
    if dag is None or fns is None:
        return None
    recs, nn, kb, nk, nodes, idx, names = dag
    extra = _outside(trace, idx)
    if extra:   # terms no conjunct reads (cell indices): their records appended
        more, kb2, nk, local = _serialize_more(extra, idx, names, nn, nk)
        recs = array("i", recs)
        recs.extend(more)
        kb += kb2
        nodes = nodes + extra
        nn += len(extra)
        pos = lambda i: local[i] if i in local else idx[i]   # noqa: E731
    else:
        pos = idx.__getitem__
    roots = array("i", [pos(t.id) for t in trace])
    info, code, consts, leaves, tr = _run(fns, recs, nn, kb, nk, roots, 0, len(roots))
    leaf_nodes = [nodes[i] for i in leaves.tolist()]
    if [n.id for n in leaf_nodes] != [n.id for n in prog.leaf_nodes]:
        return None
    t = tr.tolist()
    trace_map = {nodes[t[k]].id: (t[k + 1], "W" if t[k + 2] else "N") for k in range(0, len(t), 3)}
    n_insn = int(info.ncode_words) // 4
    return Program(code=code, consts=consts if consts.size else np.zeros(1, dtype=np.uint32),
                   leaves=prog.leaves, pool=prog.pool, n_spill=int(info.n_spill),
                   n_trace_rows=int(info.n_trace_rows), n_input_rows=prog.n_input_rows,
                   ops_per_eval=int(info.ops_per_eval), leaf_specs=prog.leaf_specs, leaf_nodes=leaf_nodes,
                   trace_map=trace_map, n_insn=n_insn, n_conjuncts=0, stats=_stats(info, n_insn))


USE_PYTHON = os.environ.get("MYTHRIL_AMD_PY_COMPILE", "0") == "1"


def compile_query(conjuncts: Sequence[Node], leaf_specs: Optional[Dict[str, LeafSpec]] = None,
                  trace: Sequence[Node] = (), pools=None, reach=None, slots=None, memo=None) -> Program:
    """The product's compiler: native when the library is built (always, on
    a GPU box: the device path needs the same library), else compiler.py.
    memo: a long-lived context's serialisation memo (compile_native)."""
    if not USE_PYTHON and available():
        return compile_native(conjuncts, leaf_specs, trace, pools, reach, slots, memo)
    return compile_program(conjuncts, leaf_specs=leaf_specs, trace=trace, pools=pools, slots=slots)
