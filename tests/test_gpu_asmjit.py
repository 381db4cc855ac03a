"""Assembled kernels (mythril_amd/asmjit.py) on gfx950: the asm interpreter's
handlers instantiated per program as straight-line code.  Verdicts and search
results must equal the asm interpreter's (same program, no kernel attached)
and the oracle's:

* random DAGs over every opcode the asm engines handle, Philox and pooled
  leaves, widths 1..256;
* every corpus program (C2-C4 solver-log queries; the LASER corpus: W_CDINS
  chains, keccak UFs, congruence conjuncts; C3's global spill words);
* batched searches in every mode, witnesses in every wave.
"""
import os

import numpy as np
import pytest

from mythril_amd import asmjit, isa
from mythril_amd.compiler import compile_program
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.ir import Ctx
from mythril_amd.smt2 import parse_file
from oracle import cdag
from tests.test_gpu_asm import _corpus, _random_supported_dag

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.runtime import Device
    if not asmjit.available():
        pytest.fail(f"assembled kernels unavailable: {asmjit.why_unavailable()}")
    d = Device(0)
    yield d
    d.close()


def pair(dev, p):
    """(interpreter handle, assembled handle) of one program"""
    di = dev.load(p)
    da = dev.load(p)
    asmjit.attach(dev, da)
    assert dev.engine_of(di) == "asm" and dev.engine_of(da) == "asmjit"
    return di, da


def test_asmjit_00_smoke(dev):
    """One small program first (a hang here stops the run early)."""
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 8)
    conj = [c.app("bvult", x, c.const(1 << 255, 256)), c.app("bvugt", y, c.const(9, 8))]
    p = compile_program(conj)
    di, da = pair(dev, p)
    try:
        va, _ = dev.eval_generated(da, 7, 0, 1 << 12, trace=False)
        vi, _ = dev.eval_generated(di, 7, 0, 1 << 12, trace=False)
    finally:
        di.free()
        da.free()
    _, _, vo = cdag.evaluate(conj, 7, 0, 1 << 12, want_verdict=True)
    assert np.array_equal(va.astype(np.uint8), vo)
    assert np.array_equal(va, vi)
    assert 0 < int(va.sum()) < len(va)


@pytest.mark.parametrize("seed", range(16))
def test_asmjit_random_dags(dev, seed):
    c, conj = _random_supported_dag(9000 + seed)
    for pools in (False, True):
        q = prepare(conj, c, use_pools=pools)
        p = q.program
        if not isa.asm_eligible(p.code, p.leaves, p.consts):
            pytest.skip("lowered outside the asm opcode set")
        n = 1 << 12
        di, da = pair(dev, p)
        try:
            va, _ = dev.eval_generated(da, DEFAULT_SEED + seed, 1 << 20, n, trace=False)
            vi, _ = dev.eval_generated(di, DEFAULT_SEED + seed, 1 << 20, n, trace=False)
        finally:
            di.free()
            da.free()
        assert np.array_equal(va, vi), (seed, pools, int(np.count_nonzero(va != vi)))
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED + seed, 1 << 20, n, want_verdict=True,
                                 specs=cdag.program_specs(p) if pools else None)
        assert np.array_equal(va.astype(np.uint8), vo), (seed, pools)


@pytest.fixture(scope="module")
def corpus():
    from mythril_amd.smt2 import parse_file
    out = []
    for f in _corpus():
        s = parse_file(f)
        out.append((os.path.basename(f), prepare(s.asserts, s.ctx)))
    return out


def test_asmjit_corpus_verdicts(dev, corpus):
    n = 1 << 14
    for name, q in corpus:
        di, da = pair(dev, q.program)
        try:
            va, _ = dev.eval_generated(da, DEFAULT_SEED, 0, n, trace=False)
            vi, _ = dev.eval_generated(di, DEFAULT_SEED, 0, n, trace=False)
        finally:
            di.free()
            da.free()
        assert np.array_equal(va, vi), (name, int(np.count_nonzero(va != vi)))


def test_asmjit_corpus_search_modes(dev, corpus):
    """Batched: assembled programs launch one by one beside the interpreter
    group; the lowest witness per program matches the interpreter's in every
    search mode."""
    sub = corpus[:24]
    dis = [dev.load(q.program) for _, q in sub]
    das = [dev.load(q.program) for _, q in sub]
    for da in das:
        asmjit.attach(dev, da)
    try:
        for flags in (0, isa.FLAG_EARLY_EXIT, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            fi, sti = dev.search(dis, DEFAULT_SEED, 0, 1 << 16, flags)
            fa, sta = dev.search(das, DEFAULT_SEED, 0, 1 << 16, flags)
            assert fa == fi, flags
            if flags == 0:
                assert sta["evals"] == sti["evals"] == len(sub) << 16
            # mixed: half assembled, half interpreted, in one call
            fm, _ = dev.search(das[::2] + dis[1::2], DEFAULT_SEED, 0, 1 << 16, flags)
            assert fm == fi[::2] + fi[1::2], flags
    finally:
        for d in dis + das:
            d.free()


@pytest.mark.parametrize("k", range(4))
def test_asmjit_reports_the_satisfying_lane(dev, k):
    c = Ctx()
    x = c.var(f"x{k}", 8)
    p = compile_program([c.app("=", x, c.const(37 * k + 11, 8))])
    di, da = pair(dev, p)
    try:
        for flags in (0, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            (fa,), _ = dev.search([da], 3 + k, 1000 * k, 1 << 16, flags)
            (fi,), _ = dev.search([di], 3 + k, 1000 * k, 1 << 16, flags)
            assert fa == fi and fa is not None
    finally:
        di.free()
        da.free()


def test_engine_assembles_long_launches(dev, corpus):
    """WitnessEngine assembles a launch's programs once it is planned above
    asmjit_min_ops; the witnesses are the interpreter's."""
    from mythril_amd.engine import WitnessEngine
    qs = [q for _, q in corpus[:12]]
    with_asm = WitnessEngine(dev=dev, budget=1 << 20, op_budget=None, asmjit_min_ops=1)
    without = WitnessEngine(dev=dev, budget=1 << 20, op_budget=None, asmjit_min_ops=0)
    wa = with_asm.search(qs)
    wi = without.search(qs)
    assert [w.index if w else None for w in wa] == [w.index if w else None for w in wi]
    assert with_asm.stats["assembled"] == sum(asmjit.eligible(q.program) for q in qs) > 0
    assert without.stats["assembled"] == 0


def test_check_runs_with_true_premises(dev):
    """A run of CHECK_IMPEQ whose premises hold for some lanes: each check's
    consequence must be its own.  Round 4 found the assembled run reading the
    NEXT check's consequence through vcc: environments.sol.o's congruence
    conjuncts (calldata reads at symbolic offsets, runs of up to 8 checks
    between fills), found by tools/asmjit_bisect.py."""
    f = os.path.join(os.path.dirname(__file__), "golden", "laser",
                     "environments_t1_batch_transfer_q09_unknown.smt2.gz")
    s = parse_file(f)
    q = prepare(s.asserts, s.ctx)
    p = q.program
    ops = [int(w) & 0xFF for w in p.code[0::4]]
    # round 5: the congruence premises are keyed (lower._Rewriter.keyed) and
    # complete grids of them are table rows (compiler._form_grids): CHECK_GRID;
    # the unkeyed CHECK_IMPEQ runs are test_check_runs_unkeyed's
    assert isa.OPCODES["CHECK_GRID"] in ops
    n = 1 << 14
    di, da = pair(dev, p)
    try:
        va, _ = dev.eval_generated(da, DEFAULT_SEED, 0, n, trace=False)
        vi, _ = dev.eval_generated(di, DEFAULT_SEED, 0, n, trace=False)
    finally:
        di.free()
        da.free()
    _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, n, want_verdict=True,
                             specs=cdag.program_specs(p))
    assert np.array_equal(vi.astype(np.uint8), vo)
    assert np.array_equal(va.astype(np.uint8), vo), int(np.count_nonzero(va.astype(np.uint8) != vo))


@pytest.mark.parametrize("seed", range(6))
def test_grid_rows_on_every_engine(dev, seed, monkeypatch):
    """Congruence grids (tests/test_grid.py's sets: an ABI word's bytes at a
    symbolic offset against concrete cells, with the symbolic bytes partly or
    wholly past the concrete ones): the asm interpreter in each register
    layout the program fits (the quarter layout's 40-word LDS budget puts
    table words in the global buffer), the compiled interpreter, the
    assembled kernel and the oracle agree on every candidate."""
    from tests.test_gpu_asm import both
    from tests.test_grid import _grid_rows, _word_dag
    shift = (0, 0, 7, 40, 3, 0)[seed]
    c, conj = _word_dag(9700 + seed, nsym=16 + 16 * (seed & 1), ncon=24 + 16 * (seed & 1), shift=shift)
    n = 1 << 14
    for pools in (False, True):
        q = prepare(conj, c, use_pools=pools)
        p = q.program
        assert _grid_rows(p)
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED + seed, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(p) if pools else None)
        for env in ({}, {"MYTHRIL_AMD_ASM_QUARTER": "0"},
                    {"MYTHRIL_AMD_ASM_QUARTER": "0", "MYTHRIL_AMD_ASM_NARROW": "0"}):
            for k in ("MYTHRIL_AMD_ASM_QUARTER", "MYTHRIL_AMD_ASM_NARROW"):
                if k in env:
                    monkeypatch.setenv(k, env[k])
                else:
                    monkeypatch.delenv(k, raising=False)
            va, vi = both(dev, p, DEFAULT_SEED + seed, 0, n)
            assert np.array_equal(va, vo), (seed, pools, env, int(np.count_nonzero(va != vo)))
            assert np.array_equal(vi, vo), (seed, pools, env, int(np.count_nonzero(vi != vo)))
        monkeypatch.delenv("MYTHRIL_AMD_ASM_QUARTER", raising=False)
        monkeypatch.delenv("MYTHRIL_AMD_ASM_NARROW", raising=False)
        di, da = pair(dev, p)
        try:
            vj, _ = dev.eval_generated(da, DEFAULT_SEED + seed, 0, n, trace=False)
        finally:
            di.free()
            da.free()
        assert np.array_equal(vj.astype(np.uint8), vo), (seed, pools, int(np.count_nonzero(vj.astype(np.uint8) != vo)))


def test_check_runs_unkeyed(dev, monkeypatch):
    """The same query with keying off (lower.KEY_MIN out of reach): runs of
    CHECK_IMPEQ over premise flags, on both engines, against the oracle."""
    from mythril_amd import lower
    monkeypatch.setattr(lower, "KEY_MIN", 1 << 30)
    f = os.path.join(os.path.dirname(__file__), "golden", "laser",
                     "environments_t1_batch_transfer_q09_unknown.smt2.gz")
    s = parse_file(f)
    q = prepare(s.asserts, s.ctx)
    p = q.program
    ops = [int(w) & 0xFF for w in p.code[0::4]]
    imp = isa.OPCODES["CHECK_IMPEQ"]
    assert any(a == b == imp for a, b in zip(ops, ops[1:])), "no run of CHECK_IMPEQ"
    assert isa.OPCODES["CHECK_IMPEQK"] not in ops
    n = 1 << 14
    di, da = pair(dev, p)
    try:
        va, _ = dev.eval_generated(da, DEFAULT_SEED, 0, n, trace=False)
        vi, _ = dev.eval_generated(di, DEFAULT_SEED, 0, n, trace=False)
    finally:
        di.free()
        da.free()
    _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, n, want_verdict=True,
                             specs=cdag.program_specs(p))
    assert np.array_equal(vi.astype(np.uint8), vo)
    assert np.array_equal(va.astype(np.uint8), vo), int(np.count_nonzero(va.astype(np.uint8) != vo))


@pytest.mark.parametrize("seed", range(6))
def test_asmjit_variable_shifts(dev, seed):
    """W_SHL / W_LSHR / W_ASHR by per-lane amounts (round 5) instantiated in
    an assembled body: verdicts equal the asm interpreter's and the oracle's."""
    from tests.test_gpu_asm import _shift_dag
    c, conj, _ = _shift_dag(9300 + seed)
    for k in range(0, len(conj), 2):
        sub = conj[k:k + 2]
        p = compile_program(sub)
        assert asmjit.eligible(p)
        di, da = pair(dev, p)
        try:
            va, _ = dev.eval_generated(da, DEFAULT_SEED + seed, 1 << 20, 1 << 12, trace=False)
            vi, _ = dev.eval_generated(di, DEFAULT_SEED + seed, 1 << 20, 1 << 12, trace=False)
        finally:
            di.free()
            da.free()
        _, _, vo = cdag.evaluate(sub, DEFAULT_SEED + seed, 1 << 20, 1 << 12, want_verdict=True)
        assert np.array_equal(va, vi), (seed, k)
        assert np.array_equal(va.astype(np.uint8), vo), (seed, k)


def _check_run_dag(seed):
    """Long runs of CHECK / CHECK_IMP / CHECK_IMPEQ (the r4b
    miscompile class): 24-40 top-level conjuncts that mostly hold - bounds,
    disequalities, implications between equalities - plus calldata-like byte
    reads at symbolic offsets, whose Ackermann congruence pairs become runs of
    CHECK_IMPEQ with premises that hold in some lanes (pooled candidates make
    the offsets collide)."""
    import random
    r = random.Random(seed)
    c = Ctx()
    xs = [c.var(f"x{i}", w) for i, w in enumerate((8, 16, 32, 64, 160, 256))]
    cd = c.array("cd", 256, 8)
    off = c.app("bvand", c.var("off", 256), c.const(7, 256))
    reads = [c.app("select", cd, c.app("bvadd", off, c.const(k, 256)) if k else off) for k in range(4)]
    reads += [c.app("select", cd, c.const(k, 256)) for k in range(4)]
    conj = []
    for _ in range(r.randrange(24, 41)):
        k = r.random()
        x = r.choice(xs)
        if k < 0.3:
            conj.append(c.app("bvule", x, c.const((1 << x.width) - 1 - r.randrange(1 << max(1, x.width - 4)), x.width)))
        elif k < 0.5:
            conj.append(c.app("not", c.app("=", x, c.const(r.getrandbits(x.width), x.width))))
        elif k < 0.75:
            y = r.choice(xs)
            conj.append(c.app("=>", c.app("=", x, c.const(r.randrange(4), x.width)),
                              c.app("=", y, c.const(r.randrange(4), y.width))))
        else:
            a, b = r.sample(reads, 2)
            conj.append(c.app("=>", c.app("=", a, c.const(r.randrange(4), 8)), c.app("bvule", b, c.const(250, 8))))
    return c, conj


@pytest.mark.parametrize("seed", range(12))
def test_asmjit_long_check_runs(dev, seed):
    c, conj = _check_run_dag(9500 + seed)
    for pools in (False, True):
        q = prepare(conj, c, use_pools=pools)
        p = q.program
        ops = [int(w) & 0xFF for w in p.code[0::4]]
        checks = {isa.OPCODES[n] for n in ("CHECK", "CHECK_IMP", "CHECK_IMPEQ", "CHECK_IMPEQK")}
        run = best = 0
        for o in ops:
            run = run + 1 if o in checks else 0
            best = max(best, run)
        assert best >= 6, best
        if not asmjit.eligible(p):      # e.g. more distinct narrow constants than the asm engines hold
            continue
        n = 1 << 14
        di, da = pair(dev, p)
        try:
            va, _ = dev.eval_generated(da, DEFAULT_SEED + seed, 0, n, trace=False)
            vi, _ = dev.eval_generated(di, DEFAULT_SEED + seed, 0, n, trace=False)
        finally:
            di.free()
            da.free()
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED + seed, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(p) if pools else None)
        assert np.array_equal(vi.astype(np.uint8), vo), (seed, pools)
        assert np.array_equal(va.astype(np.uint8), vo), (seed, pools, int(np.count_nonzero(va.astype(np.uint8) != vo)))
        if not pools:   # pooled candidates lead with the values that break the facts: often none holds
            assert 0 < int(vo.sum()) < n, (seed, int(vo.sum()))
