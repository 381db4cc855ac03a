"""engine.search_phased: a stop-after-hit search tries the lowest
PROBE_CANDIDATES indices first and continues from there only for the programs
with no witness in them; the witness is the same lowest satisfying index as
one launch over the whole range (the host build standing in for the device)."""
from mythril_amd import engine, isa
from mythril_amd.compiler import compile_program
from mythril_amd.hostemu import term_values
from mythril_amd.synth import build_c5
from tests.fakedev import FakeDevice

WITNESS = 0x5EED0005 % (1 << 31)      # synth.build_c5's planted index
FLAGS = isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT


class _Counting(FakeDevice):
    def __init__(self, **kw):
        super().__init__(**kw)
        self.ranges = []

    def search(self, dps, seed, begin, count, flags=0):
        self.ranges.append((len(dps), begin, count))
        return super().search(dps, seed, begin, count, flags)


def _setup():
    syn = build_c5(term_values, n_nodes=200)
    dev = _Counting(chunk=1 << 12)
    return syn, dev, dev.load(compile_program(syn.conjuncts))


def test_hit_in_the_probe_is_one_launch():
    syn, dev, dp = _setup()
    begin = WITNESS - 1000
    found, st = engine.search_phased(dev, [dp], syn.seed, begin, 1 << 18, FLAGS)
    assert found == [WITNESS] and dev.ranges == [(1, begin, engine.PROBE_CANDIDATES)]


def test_miss_in_the_probe_continues_and_batches_keep_their_hits():
    syn, dev, dp = _setup()
    dp2 = dev.load(compile_program(syn.conjuncts))
    begin = WITNESS - engine.PROBE_CANDIDATES - 5000      # the witness lies past the probe
    count = 1 << 18
    (want,), _ = dev.search([dp], syn.seed, begin, count, FLAGS)
    dev.ranges.clear()
    found, st = engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS)
    assert found == [want] == [WITNESS]
    assert dev.ranges == [(1, begin, engine.PROBE_CANDIDATES),
                          (1, begin + engine.PROBE_CANDIDATES, count - engine.PROBE_CANDIDATES)]
    assert st["evals"] > 0
    # exhaustive searches and short ranges are one launch
    dev.ranges.clear()
    engine.search_phased(dev, [dp, dp2], syn.seed, begin, count, 0)
    engine.search_phased(dev, [dp], syn.seed, begin, 2 * engine.PROBE_CANDIDATES, FLAGS)
    assert [r[2] for r in dev.ranges] == [count, 2 * engine.PROBE_CANDIDATES]


def test_the_launch_after_the_probe_runs_the_long_program():
    """Round 5: the launch after the probe may run another compile of the same
    constraints (Query.long_program: the quarter register layout's); it is
    loaded for that launch alone and freed after it, and the witness is the
    same lowest satisfying index."""
    syn, dev, dp = _setup()
    begin = WITNESS - engine.PROBE_CANDIDATES - 5000
    count = 1 << 18
    (want,), _ = dev.search([dp], syn.seed, begin, count, FLAGS)
    long_prog = compile_program(syn.conjuncts, slots=(4, 16))
    loaded = []
    real_load = dev.load

    def load(p):
        loaded.append(real_load(p))
        return loaded[-1]
    dev.load = load
    dev.ranges.clear()
    found, _ = engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS, [lambda n: long_prog])
    assert found == [want] == [WITNESS]
    assert len(loaded) == 1 and loaded[0].prog is long_prog
    assert len(dev.ranges) == 2
    # a program that is its own long program is not loaded again
    loaded.clear()
    engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS, [lambda n: dp.prog])
    assert loaded == []


def test_search_program_repays_its_compile():
    """engine.search_program: the quarter layout's compile only for searches
    whose candidates x instructions reach LONG_PROGRAM_MIN_WORK (a default
    LASER search of 2^22 candidates does not repay it); it keeps the search
    program's leaf table and pools (the same candidates)."""
    import os

    import numpy as np

    from mythril_amd.smt2 import parse_file
    f = os.path.join(os.path.dirname(__file__), "golden", "laser",
                     "calls_t2_fixed_address_q14_EtherThief_unknown.smt2.gz")
    s = parse_file(f)
    q = engine.prepare(s.asserts, s.ctx)
    n = q.program.n_insn
    assert engine.search_program(q, 1 << 22) is q.program
    long_ = engine.search_program(q, engine.LONG_PROGRAM_MIN_WORK // n + 1)
    assert long_ is q.long_program and long_ is not q.program
    assert np.array_equal(long_.leaves, q.program.leaves) and np.array_equal(long_.pool, q.program.pool)
    w, nn = engine._slots_used(long_)
    assert w <= engine.QUARTER_SLOTS[0] and nn <= engine.QUARTER_SLOTS[1]


def test_an_assembled_program_keeps_its_kernel():
    """when WitnessEngine._assemble attached an assembled kernel,
    the launch after the probe keeps that program (the long program would run
    on the interpreter); a long program the loader puts on another engine
    than the asm interpreter is not used either."""
    syn, dev, dp = _setup()
    begin = WITNESS - engine.PROBE_CANDIDATES - 5000
    count = 1 << 18
    long_prog = compile_program(syn.conjuncts, slots=(4, 16))
    asked = []

    def lp(n):
        asked.append(n)
        return long_prog
    dp.assembled = "mw_asmjit_test"
    dev.ranges.clear()
    found, _ = engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS, [lp])
    assert found == [WITNESS] and asked == []
    dp.assembled = None
    searched = []
    real_search = dev.search

    def search(dps, *a, **k):
        searched.append([d.prog for d in dps])
        return real_search(dps, *a, **k)
    dev.search = search
    dev.engine_of = lambda d: "interp"
    found, _ = engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS, [lp])
    assert found == [WITNESS] and asked and searched[-1] == [dp.prog]
    dev.engine_of = lambda d: "asm"
    engine.search_phased(dev, [dp], syn.seed, begin, count, FLAGS, [lp])
    assert searched[-1] == [long_prog]


def test_long_program_respects_layout_switches(monkeypatch):
    """MYTHRIL_AMD_ASM=0 / _NARROW=0 keep the program as it is;
    _QUARTER=0 allows the narrow layout only; a recompiled program always
    fits the layout it was compiled for (narrow constants, LDS budget)."""
    import os

    from mythril_amd.smt2 import parse_file
    from mythril_amd import isa
    f = os.path.join(os.path.dirname(__file__), "golden", "laser",
                     "calls_t2_fixed_address_q14_EtherThief_unknown.smt2.gz")
    s = parse_file(f)
    for var in ("MYTHRIL_AMD_ASM", "MYTHRIL_AMD_ASM_NARROW"):
        monkeypatch.setenv(var, "0")
        q = engine.prepare(s.asserts, s.ctx)
        assert q.long_program is q.program, var
        monkeypatch.delenv(var)
    monkeypatch.setenv("MYTHRIL_AMD_ASM_QUARTER", "0")
    q = engine.prepare(s.asserts, s.ctx)
    lp = q.long_program
    w, n = engine._slots_used(lp)
    assert w <= engine.NARROW_SLOTS[0] and n <= engine.NARROW_SLOTS[1]
    if lp is not q.program:
        assert engine._lands_on(lp, "narrow") and not engine._lands_on(lp, "quarter") or \
            (w > engine.QUARTER_SLOTS[0] or n > engine.QUARTER_SLOTS[1])
    monkeypatch.delenv("MYTHRIL_AMD_ASM_QUARTER")
    q = engine.prepare(s.asserts, s.ctx)
    lp = q.long_program
    assert lp is not q.program and engine._lands_on(lp, "quarter")
    assert len(isa.asm_narrow_constants(lp.code, lp.consts)) <= isa.ASM_NK_BY_LAYOUT["quarter"]
