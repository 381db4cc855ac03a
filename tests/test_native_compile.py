"""The native host compiler (csrc/mw_compile.cpp via mythril_amd/ccompile.py)
against compiler.py's compile_program, its parity reference: programs must be
byte-identical (code, constant pool, leaf table, pools, spill/trace layout, op
counts, leaf order) on both committed corpora (search and witness programs),
on random DAGs over every op the compiler lowers (with traced terms, pools,
register pressure) and on the shapes that exercise each superinstruction.
Runs on the CPU: the compiler is host code in the product library."""
import dataclasses
import os
import random
import re

import numpy as np
import pytest

from mythril_amd import ccompile, isa
from mythril_amd.compiler import Unsupported, compile_program
from mythril_amd.engine import prepare
from mythril_amd.ir import BOOL, Ctx
from mythril_amd.smt2 import parse_file
from tests.helpers import RandDag

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.skipif(not ccompile.available(), reason="product library not built")


def _same(a, b):
    for k in ("code", "consts", "leaves", "pool"):
        x, y = np.asarray(getattr(a, k)), np.asarray(getattr(b, k))
        assert x.dtype == y.dtype and np.array_equal(x, y), k
    for k in ("n_spill", "n_trace_rows", "n_input_rows", "ops_per_eval", "n_insn", "n_conjuncts", "stats",
              "trace_map"):
        assert getattr(a, k) == getattr(b, k), k
    assert [n.id for n in a.leaf_nodes] == [n.id for n in b.leaf_nodes]
    assert [dataclasses.asdict(s) for s in a.leaf_specs] == [dataclasses.asdict(s) for s in b.leaf_specs]


def _both(conj, trace=(), specs=None, pools=None):
    cp = lambda: None if specs is None else {k: dataclasses.replace(v) for k, v in specs.items()}  # noqa: E731
    a = compile_program(conj, leaf_specs=cp(), trace=trace, pools=pools)
    b = ccompile.compile_native(conj, leaf_specs=cp(), trace=trace, pools=pools)
    _same(a, b)
    return a, b


def test_ir_ops_match_the_native_enum():
    src = open(os.path.join(ROOT, "mythril_amd", "csrc", "mw_compile.cpp")).read()
    body = re.search(r"enum IrOp \{(.*?)\};", src, re.S).group(1)
    names = [t.strip() for t in body.replace("\n", " ").split(",") if t.strip()]
    assert names[-1] == "IR_NOPS"
    want = ["IR_" + op.upper().replace("=>", "IMPLIES").replace("=", "EQ") for op in ccompile.IR_OPS]
    assert names[:-1] == want


def _corpus(d):
    base = os.path.join(HERE, "golden", d)
    return [os.path.join(base, f) for f in sorted(os.listdir(base)) if f.endswith((".smt2", ".smt2.gz"))]


@pytest.mark.parametrize("corpus", ["solver_log", "laser"])
def test_corpus_programs_byte_identical(corpus):
    n = 0
    for f in _corpus(corpus):
        s = parse_file(f)
        q = prepare(s.asserts, s.ctx)
        specs = {x.name: x for x in q.program.leaf_specs}
        _both(q.lowered.conjuncts, specs=specs)
        # the witness program: no conjuncts, every leaf and cell index traced
        _both([], trace=list(q.program.leaf_nodes) + q.arg_terms, specs=specs)
        n += 1
    assert n >= (7 if corpus == "solver_log" else 500)


def test_prepare_uses_the_native_compiler():
    s = parse_file(_corpus("laser")[0])
    q = prepare(s.asserts, s.ctx)
    assert q.program.ssa == [] and q.program.ssa_build is not None   # native: machine IR on demand
    ir = q.program.machine_ir()
    assert ir and ir[-1].op == "END"
    ref = compile_program(q.lowered.conjuncts).ssa
    assert [(i.op, i.width, i.imm) for i in ir] == [(i.op, i.width, i.imm) for i in ref]


@pytest.mark.parametrize("seed", range(40))
def test_random_dags_byte_identical(seed):
    dag = RandDag(seed)
    conj = [dag.boolean(4) for _ in range(3)]
    traced = [dag.bv(w, 3) for w in (8, 64, 256)]
    pools = {v.name: [None, 0, 1, (1 << v.width) - 1] for v in dag.vars[:3]}
    for tr in ((), traced):
        try:
            _both(conj, trace=tr, pools=pools)
        except Unsupported:
            with pytest.raises(Unsupported):
                ccompile.compile_native(conj, trace=tr, pools=pools)


def test_register_pressure_spills_identical():
    """Forty wide products live at once (both folds read all of them): the W
    file (7 slots) spills and fills, the narrow file too; spill slots laid
    out hottest-first."""
    import functools
    c = Ctx()
    xs = [c.var(f"x{i}", 256) for i in range(40)]
    ws = [c.app("bvmul", x, xs[(i + 1) % 40]) for i, x in enumerate(xs)]
    f1 = functools.reduce(lambda a, b: c.app("bvadd", a, b), ws)
    f2 = functools.reduce(lambda a, b: c.app("bvxor", a, b), ws[::-1])
    conj = [c.app("bvult", f1, c.const(5, 256)), c.app("bvult", f2, c.const(7, 256))]
    ns = [c.app("extract", w, params=(7, 0)) for w in ws]
    conj += [c.app("=", c.app("bvxor", *ns), c.const(3, 8))]
    a, b = _both(conj)
    assert a.stats["spills"] > 0 and a.stats["fills"] > 0


def test_wide_leaves_redrawn_not_spilled():
    """Forty wide leaves live across two folds: with REMAT_LEAVES (the
    default) the allocators draw an evicted leaf again at its next use
    instead of spilling it (the same LEAF_W, same leaf), identically."""
    import functools
    from mythril_amd import compiler
    c = Ctx()
    xs = [c.var(f"x{i}", 256) for i in range(40)]
    f1 = functools.reduce(lambda a, b: c.app("bvadd", a, b), xs)
    f2 = functools.reduce(lambda a, b: c.app("bvxor", a, b), xs[::-1])
    conj = [c.app("bvult", f1, c.const(5, 256)), c.app("bvult", f2, c.const(7, 256))]
    a, b = _both(conj)
    inv = {v: k for k, v in isa.OPCODES.items()}
    ops = [inv[int(r[0]) & 0xFF] for r in a.code.reshape(-1, 4)]
    if compiler.REMAT_LEAVES:
        assert a.stats["spills"] == 0 and ops.count("LEAF_W") > 40
    else:
        assert a.stats["spills"] > 0


def test_superinstructions_identical():
    """CHECK_IMP, CHECK_IMPEQ(W) (congruence conjuncts) and W_CDINS chains
    (guarded calldata bytes of an ABI word) come out of both compilers."""
    c = Ctx()
    size = c.var("calldatasize", 256)
    off = c.var("off", 256)
    byte = lambda i: c.app("ite", c.app("bvslt", c.const(i, 256), size), c.var(f"cd{i}", 8), c.const(0, 8))  # noqa
    word = c.app("concat", *[byte(i) for i in range(4, 36)])
    i1, i2 = c.var("i1", 256), c.var("i2", 256)
    v1, v2 = c.var("v1", 256), c.var("v2", 256)
    n1, n2 = c.var("n1", 8), c.var("n2", 8)
    conj = [c.app("bvugt", word, c.const(5, 256)),
            c.app("=>", c.app("=", i1, i2), c.app("=", v1, v2)),
            c.app("=>", c.app("=", off, c.const(4, 256)), c.app("=", n1, n2)),
            c.app("=>", c.var("b", BOOL), c.app("bvult", n1, n2))]
    a, _ = _both(conj)
    ops = {int(w) & 0xFF for w in a.code[0::4]}
    for name in ("CHECK_IMPEQ", "CHECK_IMPEQW", "W_CDINS"):
        assert isa.OPCODES[name] in ops, name
    flags = [(int(w) >> 8) & 0xFF for w in a.code[0::4]]
    assert isa.FLAG_CHAIN in flags


def test_edge_shapes_identical():
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 32)
    conj = [c.false(), c.app("=", c.app("bvshl", x, c.const(300, 256)), c.const(0, 256)),
            c.app("=", c.app("bvlshr", x, c.const(0, 256)), x),
            c.app("distinct", y, c.const(1, 32), c.const(2, 32)),
            c.app("=", c.app("concat", c.const(0, 224), y), c.app("zero_extend", y, params=(224,))),
            c.app("bvsge", c.app("sign_extend", y, params=(224,)), c.const(7, 256)),
            c.app("=", c.app("repeat", c.app("extract", y, params=(7, 0)), params=(4,)), y),
            c.app("=", c.app("rotate_left", y, params=(32,)), y)]
    _both(conj, trace=[c.app("extract", c.const(0x1234, 256), params=(11, 4)), x, y])
    _both([c.true()], trace=[c.const(5, 256), c.const(1, 8)])
    _both([])


def test_unsupported_matches():
    c = Ctx()
    a = c.array("A", 256, 256)
    for conj in ([c.app("=", c.app("select", a, c.var("i", 256)), c.const(1, 256))],
                 [c.app("=", c.var("wide", 512), c.const(1, 512))]):
        with pytest.raises(Unsupported):
            compile_program(conj)
        with pytest.raises(Unsupported):
            ccompile.compile_native(conj)


def test_malformed_records_rejected():
    """The record stream is validated before any pass runs (operands after
    their users, out-of-range constants, truncation)."""
    import ctypes
    from array import array
    lib, comp, _, free = ccompile._bind()
    h = ctypes.c_void_p()
    info = ccompile.MwCompileInfo()
    for recs, nn, roots in ((array("i", [1, 8, 0, 0, 0, 1, 0]), 1, array("i", [0])),     # arg is itself
                            (array("i", [0, 8, 0, 5, 0, 0]), 1, array("i", [0])),        # const index 5 of 0
                            (array("i", [1, 8, 0]), 1, array("i", [0])),                 # truncated
                            (array("i", [1, 8, 0, 0, 0, 0]), 1, array("i", [3]))):       # root out of range
        rc = comp(ccompile._addr(recs), len(recs), nn, None, 0, ccompile._addr(roots), len(roots), 0,
                  isa.NW, isa.NN, ctypes.byref(h), ctypes.byref(info))
        assert rc == -3 and not h.value, lib.mg_last_error()


def test_random_dags_deep():
    """Deeper DAGs with shared subterms across conjuncts (rematerialisation of
    cheap terms over leaves in later conjuncts)."""
    for seed in range(8):
        dag = RandDag(1000 + seed, nvars=10)
        r = random.Random(seed)
        base = [dag.bv(r.choice([8, 64, 256]), 4) for _ in range(6)]
        conj = []
        for _ in range(12):
            a, b = r.sample(base, 2)
            if a.width == b.width:
                conj.append(c_cmp(dag.ctx, r, a, b))
            else:
                conj.append(dag.boolean(3))
        try:
            _both(conj, trace=base[:2])
        except Unsupported:
            pass


def c_cmp(c, r, a, b):
    return c.app(r.choice(["bvult", "=", "bvsle", "distinct"]), a, b)


def test_witness_program_from_the_search_stream_is_the_fresh_compile():
    """ccompile.compile_trace_native (the witness program compiled from the
    search program's own record stream, cell-index terms appended, the leaf
    table reused) gives the program a fresh compile of the trace gives."""
    import glob
    import dataclasses
    import numpy as np
    from mythril_amd import ccompile, engine
    from mythril_amd.smt2 import parse_file
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "laser", "*.smt2*")))[::9] + \
        sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "solver_log", "*.smt2*")))
    n = 0
    for f in files:
        s = parse_file(f)
        q = engine.prepare(s.asserts, s.ctx)
        traced = list(q.program.leaf_nodes) + list(q.arg_terms)
        b = ccompile.compile_trace_native(q.program, traced)
        assert b is not None, f
        fixed = {sp.name: dataclasses.replace(sp, pool=None if sp.pool is None else list(sp.pool))
                 for sp in q.program.leaf_specs}
        a = ccompile.compile_native([], leaf_specs=fixed, trace=traced)
        for k in ("code", "consts", "leaves", "pool"):
            assert np.array_equal(getattr(a, k), getattr(b, k)), (f, k)
        assert (a.trace_map, a.n_trace_rows, a.n_spill, a.n_input_rows) == \
            (b.trace_map, b.n_trace_rows, b.n_spill, b.n_input_rows), f
        assert [x.id for x in a.leaf_nodes] == [x.id for x in b.leaf_nodes]
        n += 1
    assert n >= 60


def _max_slots(p):
    mw = mn = -1
    for i in range(0, len(p.code), 4):
        w, n = isa.decode_dst(int(p.code[i + 1]) & 0xFFFF)
        mw = max(mw, -1 if w is None else w)
        mn = max(mn, -1 if n is None else n)
    return mw + 1, mn + 1


def test_slot_limited_programs_identical():
    """Round 5: compiled for the asm interpreter's quarter layout (4 W and 16
    N slots, mw_compile_slots), a program keeps its registers within those
    slots (spilling more) on both compilers, byte-identically; a program that
    fit already comes out unchanged."""
    files = _corpus("laser")[::9]
    grew = 0
    for f in files:
        s = parse_file(f)
        q = prepare(s.asserts, s.ctx)
        specs = {x.name: x for x in q.program.leaf_specs}
        cp = lambda: {k: dataclasses.replace(v) for k, v in specs.items()}  # noqa: E731
        a = compile_program(q.lowered.conjuncts, leaf_specs=cp(), slots=(4, 16))
        b = ccompile.compile_native(q.lowered.conjuncts, leaf_specs=cp(), slots=(4, 16))
        _same(a, b)
        w, n = _max_slots(b)
        assert w <= 4 and n <= 16, f
        w0, n0 = _max_slots(q.program)
        if w0 <= 4 and n0 <= 16:
            assert np.array_equal(b.code, q.program.code)
        else:
            grew += b.n_insn >= q.program.n_insn
    assert grew > 0
    c = Ctx()
    x = c.var("x", 8)
    with pytest.raises(RuntimeError):
        ccompile.compile_native([c.app("=", x, c.const(1, 8))], slots=(3, 16))
