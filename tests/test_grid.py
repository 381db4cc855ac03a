"""Congruence grids (compiler._form_grids, CHECK_GRID) on the host build of the
interpreter (mw_interp.h through mw_host_emu.cpp) against the C oracle over the
lowered conjuncts: an ABI word's bytes read at a symbolic calldata offset
against concrete cells (C3's shape, calldata.py:218-231), whose keyed
congruence checks become one table lookup per concrete cell."""
import random

import numpy as np
import pytest

from mythril_amd import ccompile, compiler, hostemu, isa, lower
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.ir import Ctx
from oracle import cdag


def _word_dag(seed, nsym=16, ncon=24, base_mask=31, shift=0):
    """bytes cd[off + k] (k < nsym, off = x & base_mask + shift) and cd[K] (K < ncon),
    with facts tying some of them: the grid's rows hold in some lanes and fail in others."""
    r = random.Random(seed)
    c = Ctx()
    cd = c.array("cd", 256, 8)
    off = c.app("bvadd", c.app("bvand", c.var("x", 256), c.const(base_mask, 256)), c.const(shift, 256))
    sym = [c.app("select", cd, c.app("bvadd", off, c.const(k, 256)) if k else off) for k in range(nsym)]
    con = [c.app("select", cd, c.const(k, 256)) for k in range(ncon)]
    conj = [c.app("not", c.app("=", x, c.const(0xF0 + i % 7, 8))) for i, x in enumerate(sym + con)]
    for _ in range(6):
        a, b = r.choice(sym), r.choice(con)
        conj.append(c.app("bvule", c.app("bvxor", a, b), c.const(r.choice((254, 255)), 8)))
    conj.append(c.app("bvule", c.var("x", 256), c.const(1 << 20, 256)))
    return c, conj


def _grid_rows(p):
    code = p.code.reshape(-1, 4)
    return [r for r in code if int(r[0]) & 0xFF == isa.OPCODES["CHECK_GRID"]]


@pytest.mark.parametrize("seed", range(6))
def test_grid_verdicts_equal_the_oracle(seed):
    shift = (0, 0, 7, 40, 3, 0)[seed]      # 40: the symbolic bytes lie past every concrete cell
    c, conj = _word_dag(9700 + seed, shift=shift)
    seen = set()
    for pools in (False, True):
        q = prepare(conj, c, use_pools=pools)
        p = q.program
        rows = _grid_rows(p)
        assert rows, "no grid"
        n = 1 << 12
        got, _ = hostemu.eval_generated(p, DEFAULT_SEED + seed, 0, n)
        _, _, want = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED + seed, 0, n, want_verdict=True,
                                   specs=cdag.program_specs(p) if pools else None)
        assert np.array_equal(got.astype(np.uint8), want), (seed, pools)
        seen |= set(want.tolist())
    assert seen == {0, 1}, seen     # rows that hold and rows that fail


def test_grid_matches_the_checks_it_replaces(monkeypatch):
    """The same set compiled with grids off (compiler.GRID_MIN out of reach,
    the Python compiler): identical verdicts on 2^14 candidates."""
    c, conj = _word_dag(9800, nsym=32, ncon=40)
    q = prepare(conj, c, use_pools=True)
    assert _grid_rows(q.program)
    n = 1 << 14
    grid, _ = hostemu.eval_generated(q.program, DEFAULT_SEED, 0, n)
    monkeypatch.setattr(ccompile, "USE_PYTHON", True)
    monkeypatch.setattr(compiler, "GRID_MIN", 1 << 30)
    q2 = prepare(conj, c, use_pools=True)
    ops = {int(w) & 0xFF for w in q2.program.code[0::4]}
    assert isa.OPCODES["CHECK_IMPEQK"] in ops and isa.OPCODES["CHECK_GRID"] not in ops
    checks, _ = hostemu.eval_generated(q2.program, DEFAULT_SEED, 0, n)
    assert np.array_equal(grid, checks)


def test_grid_tables_precede_the_spill_slots():
    """The tables take the first words of the spill area (each row's c field
    names its table's word and size), then the spill slots; the Python and
    native compilers agree byte for byte."""
    c, conj = _word_dag(9900, nsym=32, ncon=40)
    q = prepare(conj, c, use_pools=False)
    p = q.program
    rows = _grid_rows(p)
    tabs = sorted({(int(r[2]) >> 16) & 1023 for r in rows})
    sizes = {(int(r[2]) >> 16) & 1023: ((int(r[2]) >> 26) & 31) + 1 for r in rows}
    words = 0
    for t in tabs:
        assert t == words
        words += sizes[t]
    assert p.n_spill >= words
    code = p.code.reshape(-1, 4)
    puts = [int(r[3]) for r in code if int(r[0]) & 0xFF == isa.OPCODES["SPILL_N"] and int(r[3]) < words]
    assert sorted(puts) == list(range(words))
    py = ccompile.compile_program(q.lowered.conjuncts, leaf_specs={s.name: s for s in p.leaf_specs})
    assert np.array_equal(py.code, p.code) and np.array_equal(py.consts, p.consts)


def test_incomplete_grid_stays_checks():
    """A group of keyed checks that is not a complete grid (one pair's check
    missing) is left as it is."""
    ins = []
    key = compiler.VReg(0, "N")
    syms = [compiler.VReg(1 + k, "N") for k in range(8)]
    cons = [compiler.VReg(20 + k, "N") for k in range(9)]
    for v in [key] + syms + cons:
        ins.append(compiler.MInsn("LEAF_N", 8, v, [], imm=v.id))
    for K, b in enumerate(cons):
        for k, t in enumerate(syms):
            if (K, k) != (3, 5):
                ins.append(compiler.MInsn("CHECK_IMPEQK", 8, None, [key, b, t], imm=100 + K - k))
    ins.append(compiler.MInsn("END", 0, None, []))
    out = compiler._form_grids(ins)
    assert [i.op for i in out] == [i.op for i in ins]
    full = [i for i in ins if i.op != "CHECK_IMPEQK"][:-1]
    for K, b in enumerate(cons):
        for k, t in enumerate(syms):
            full.append(compiler.MInsn("CHECK_IMPEQK", 8, None, [key, b, t], imm=100 + K - k))
    full.append(compiler.MInsn("END", 0, None, []))
    out = compiler._form_grids(full)
    # the larger side (9 concrete cells) is the table, a row per symbolic byte
    assert sum(i.op == "GRID_PUT" for i in out) == len(cons)
    assert sum(i.op == "CHECK_GRID" for i in out) == len(syms)
    assert not any(i.op == "CHECK_IMPEQK" for i in out)
    puts = {id(i.srcs[0]): i.imm for i in out if i.op == "GRID_PUT"}
    # the rows' leaves are drawn again at the row (defined before the table):
    # the fresh register's LEAF_N names the original leaf (imm = its id here)
    drawn = {i.dst.id: i.imm for i in out if i.op == "LEAF_N"}
    assert sum(i.op == "LEAF_N" for i in out) == 1 + len(syms) + len(cons)   # key, cells, redrawn bytes
    # row of t_k: (key = 100 + K - k) <=> j = E - key = table offset of cell K
    for i in out:
        if i.op == "CHECK_GRID":
            k = [t.id for t in syms].index(drawn[i.srcs[1].id])
            for K, b in enumerate(cons):
                assert (i.imm - (100 + K - k)) & 0xFFFFFFFF == puts[id(b)], (k, K)


@pytest.mark.parametrize("nlds", [None, 0, 8, 80])
def test_grid_rows_assemble(nlds):
    """An assembled body's rows (asmgen._grid_static: no exec writes, the
    table wholly in LDS, wholly global, or split) assemble for gfx950, and the
    kernel reads the table the way the split puts it."""
    from mythril_amd import asmgen, asmjit
    c, conj = _word_dag(9701, nsym=32, ncon=40)
    q = prepare(conj, c, use_pools=True)
    p = q.program
    body = asmgen.static_body(p.code, p.consts, p.leaves, nlds=nlds, pool=p.pool)
    assert not any("exec" in ln for ln in body)
    sect, lds, glob = None, 0, 0
    for ln in body:
        if ln.startswith("; "):
            sect = ln.split(": ", 1)[-1]
        elif sect == "CHECK_GRID":
            lds += "ds_read_b32" in ln
            glob += "global_load_dword" in ln
    rows = len(_grid_rows(p))
    if nlds == 80:
        assert (lds, glob) == (rows, 0)
    if nlds == 0:
        assert (lds, glob) == (0, rows)
    if nlds in (None, 8):
        assert (lds, glob) == (rows, rows)
    co, name, _ = asmjit.assemble(p, cache=False)
    assert len(co) > 0 and name.startswith("mwa_")
