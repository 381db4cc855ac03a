"""The threaded-dispatch asm interpreter (csrc/mw_asm_interp.inc) on gfx950,
against the compiled interpreter (MYTHRIL_AMD_ASM=0: same library, same
programs) and the oracle:

* every opcode the asm interpreter handles, on random DAGs over Philox and
  pooled leaves (all four leaf kinds), at widths 1..256;
* every corpus program (C2-C4 solver-log queries, the LASER corpus: W_CDINS
  chains, keccak UFs, congruence conjuncts, the C3 global-spill path):
  per-candidate verdicts and batched search results, in every search mode.
"""
import os
import random

import numpy as np
import pytest

from mythril_amd import isa
from mythril_amd.compiler import compile_program
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.ir import BOOL, Ctx
from mythril_amd.smt2 import parse_file
from oracle import cdag

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


class compiled_interpreter:
    """MYTHRIL_AMD_ASM=0 for the duration (read by the library at each call)."""

    def __enter__(self):
        self.old = os.environ.get("MYTHRIL_AMD_ASM")
        os.environ["MYTHRIL_AMD_ASM"] = "0"

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop("MYTHRIL_AMD_ASM", None)
        else:
            os.environ["MYTHRIL_AMD_ASM"] = self.old


def both(dev, p, seed, begin, n):
    dp = dev.load(p)
    try:
        assert dev.engine_of(dp) == "asm"
        va, _ = dev.eval_generated(dp, seed, begin, n, trace=False)
        with compiled_interpreter():
            assert dev.engine_of(dp) == "interp"
            vi, _ = dev.eval_generated(dp, seed, begin, n, trace=False)
    finally:
        dp.free()
    return va.astype(np.uint8), vi.astype(np.uint8)


def test_asm_00_smoke(dev):
    """One small program first (a hang here stops the run early)."""
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 8)
    p = compile_program([c.app("bvult", x, c.const(1 << 255, 256)), c.app("bvugt", y, c.const(9, 8))])
    va, vi = both(dev, p, 7, 0, 1 << 12)
    assert np.array_equal(va, vi)
    _, _, vo = cdag.evaluate([c.app("bvult", x, c.const(1 << 255, 256)), c.app("bvugt", y, c.const(9, 8))],
                             7, 0, 1 << 12, want_verdict=True)
    assert np.array_equal(va, vo)
    assert 0 < int(va.sum()) < len(va)


WIDTHS = [1, 8, 16, 32, 33, 64, 160, 255, 256]


def _random_supported_dag(seed):
    """A random DAG over the asm interpreter's ops (no division, no variable shifts)."""
    r = random.Random(seed)
    c = Ctx()
    leaves = {w: [c.var(f"v{w}_{i}", w) for i in range(2)] for w in WIDTHS if w > 1}
    bools = [c.var(f"b{i}", BOOL) for i in range(2)]

    def bv(w, d):
        if d == 0 or r.random() < 0.25:
            if r.random() < 0.2:
                return c.const(r.getrandbits(w), w)
            if w in leaves:
                return r.choice(leaves[w])
            src = r.choice(leaves[256])
            return c.app("extract", src, params=(w - 1, 0)) if w > 1 else c.app("extract", src, params=(0, 0))
        k = r.random()
        a = bv(w, d - 1)
        if k < 0.35:
            return c.app(r.choice(["bvadd", "bvsub", "bvand", "bvor", "bvxor", "bvmul"]), a, bv(w, d - 1))
        if k < 0.45:
            return c.app("bvnot", a)
        if k < 0.55:
            return c.app("ite", boolean(d - 1), a, bv(w, d - 1))
        if k < 0.7 and w >= 2:
            amt = r.randrange(0, w)
            return c.app(r.choice(["bvshl", "bvlshr"]), a, c.const(amt, w))
        if k < 0.85:
            ww = r.choice([x for x in WIDTHS if x >= w])
            lo = r.randrange(0, ww - w + 1)
            return c.app("extract", bv(ww, d - 1), params=(lo + w - 1, lo)) if ww > w else a
        if w >= 2:
            hw = r.randrange(1, w)
            return c.app("concat", bv(hw, d - 1), bv(w - hw, d - 1)) if hw > 1 and w - hw > 1 else a
        return a

    def boolean(d):
        w = r.choice(WIDTHS[1:])
        k = r.random()
        if d == 0 or k < 0.15:
            return r.choice(bools)
        if k < 0.7:
            op = r.choice(["bvult", "bvule", "bvslt", "bvsle", "=", "bvugt", "bvsge"])
            return c.app(op, bv(w, d - 1), bv(w, d - 1))
        if k < 0.8:
            return c.app("bvumul_noovfl", bv(w, d - 1), bv(w, d - 1)) if w >= 33 else c.app("=", bv(w, 0), bv(w, 0))
        if k < 0.9:
            return c.app(r.choice(["and", "or", "xor"]), boolean(d - 1), boolean(d - 1))
        return c.app("not", boolean(d - 1))

    conj = [boolean(4) for _ in range(3)]
    return c, conj


@pytest.mark.parametrize("seed", range(24))
def test_asm_random_dags(dev, seed):
    c, conj = _random_supported_dag(9000 + seed)
    for pools in (False, True):
        q = prepare(conj, c, use_pools=pools)
        p = q.program
        if not isa.asm_eligible(p.code, p.leaves, p.consts):
            pytest.skip("lowered outside the asm opcode set")
        n = 1 << 12
        va, vi = both(dev, p, DEFAULT_SEED + seed, 1 << 20, n)
        assert np.array_equal(va, vi), (seed, pools, int(np.count_nonzero(va != vi)))
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED + seed, 1 << 20, n, want_verdict=True,
                                 specs=cdag.program_specs(p) if pools else None)
        assert np.array_equal(va, vo), (seed, pools)


def _corpus():
    out = []
    for d in ("solver_log", "laser"):
        base = os.path.join(ROOT, "tests", "golden", d)
        for f in sorted(os.listdir(base)):
            if f.endswith(".smt2") or f.endswith(".smt2.gz"):
                out.append(os.path.join(base, f))
    return out


@pytest.fixture(scope="module")
def corpus():
    qs = []
    for f in _corpus():
        s = parse_file(f)
        qs.append((os.path.basename(f), prepare(s.asserts, s.ctx)))
    return qs


def test_asm_corpus_verdicts(dev, corpus):
    n = 1 << 14
    for name, q in corpus:
        va, vi = both(dev, q.program, DEFAULT_SEED, 0, n)
        assert np.array_equal(va, vi), (name, int(np.count_nonzero(va != vi)))
    # and the oracle on a sample (C3 included: its global spill path)
    for name, q in corpus[:8] + corpus[-8:]:
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(q.program))
        va, _ = both(dev, q.program, DEFAULT_SEED, 0, n)
        assert np.array_equal(va, vo), name


class layout_env:
    """MYTHRIL_AMD_ASM_QUARTER / _NARROW for the programs loaded meanwhile
    (read by the library at each load: which register layout's kernel a
    program is predecoded for)."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("env", [{"MYTHRIL_AMD_ASM_QUARTER": "0"}, {"MYTHRIL_AMD_ASM_NARROW": "0"}])
def test_asm_corpus_verdicts_on_the_wider_layouts(dev, corpus, env):
    """Round 5: a program runs on the smallest register layout that holds it
    (quarter: 4 waves per SIMD, narrow: 3, wide: 2).  With the smaller
    layouts switched off the same programs run on the wider kernels: the
    same verdicts as the compiled interpreter there too."""
    n = 1 << 13
    for name, q in corpus[::3]:
        with layout_env(**env):
            va, vi = both(dev, q.program, DEFAULT_SEED, 0, n)
        assert np.array_equal(va, vi), (name, env, int(np.count_nonzero(va != vi)))


def test_asm_quarter_long_programs(dev, corpus):
    """Round 5: a long search runs Query.long_program, the constraints compiled
    again within the quarter layout's 4 W / 16 N slots (more spills, four
    waves per SIMD): per candidate the same verdicts as the search program,
    and the same lowest witness in a stop-after-hit search."""
    n = 1 << 13
    done = 0
    for name, q in corpus:
        lp = q.long_program
        if lp is q.program:
            continue
        dp, dl = dev.load(q.program), dev.load(lp)
        try:
            assert dev.engine_of(dl) == "asm"
            va, _ = dev.eval_generated(dp, DEFAULT_SEED, 0, n, trace=False)
            vl, _ = dev.eval_generated(dl, DEFAULT_SEED, 0, n, trace=False)
            assert np.array_equal(va, vl), (name, int(np.count_nonzero(va != vl)))
            fa, _ = dev.search([dp], DEFAULT_SEED, 0, 1 << 16, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT)
            fl, _ = dev.search([dl], DEFAULT_SEED, 0, 1 << 16, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT)
            assert fa == fl, name
        finally:
            dp.free()
            dl.free()
        done += 1
    assert done >= 20


def test_asm_corpus_search_modes(dev, corpus):
    """64 programs per launch, exhaustive / early exit / stop after hit: the
    same lowest witness index per program as the compiled interpreter."""
    dps = [dev.load(q.program) for _, q in corpus[:64]]
    try:
        for flags in (0, isa.FLAG_EARLY_EXIT, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            fa, sta = dev.search(dps, DEFAULT_SEED, 0, 1 << 16, flags)
            with compiled_interpreter():
                fi, sti = dev.search(dps, DEFAULT_SEED, 0, 1 << 16, flags)
            assert fa == fi, flags
            if flags == 0:
                assert sta["evals"] == sti["evals"] == 64 << 16
    finally:
        for dp in dps:
            dp.free()


@pytest.mark.parametrize("k", range(6))
def test_asm_search_reports_the_satisfying_lane(dev, k):
    """Witnesses in every wave of a 256-candidate chunk (not only its first
    64 lanes): an 8-bit Philox leaf equal to a constant, searched exhaustively
    and with early exit + stop-after-hit, gives the compiled interpreter's
    lowest index, and that index satisfies the program."""
    c = Ctx()
    x = c.var(f"x{k}", 8)
    p = compile_program([c.app("=", x, c.const(37 * k + 11, 8))])
    dp = dev.load(p)
    try:
        assert dev.engine_of(dp) == "asm"
        for flags in (0, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            (fa,), _ = dev.search([dp], 3 + k, 1000 * k, 1 << 16, flags)
            with compiled_interpreter():
                (fi,), _ = dev.search([dp], 3 + k, 1000 * k, 1 << 16, flags)
            assert fa == fi and fa is not None
            v, _ = dev.eval_generated(dp, 3 + k, fa, 1, trace=False)
            assert v[0] == 1
            if fa > 1000 * k:
                va, _ = dev.eval_generated(dp, 3 + k, 1000 * k, fa - 1000 * k, trace=False)
                assert not va.any()              # nothing lower
    finally:
        dp.free()


def both_traced(dev, p, seed, begin, n):
    dp = dev.load(p)
    try:
        assert dev.engine_of(dp) == "asm"
        va, ta = dev.eval_generated(dp, seed, begin, n)
        with compiled_interpreter():
            vi, ti = dev.eval_generated(dp, seed, begin, n)
    finally:
        dp.free()
    return va, ta, vi, ti


@pytest.mark.parametrize("seed", range(8))
def test_asm_trace_rows(dev, seed):
    """STORE_W / STORE_N on the asm interpreter (mg_eval_generated with a
    trace): every trace row of random DAG terms (widths 1..256, wide and
    narrow rows) equals the compiled interpreter's, at ragged counts (a last
    chunk with invalid lanes) and offsets past 2^32."""
    c, conj = _random_supported_dag(9100 + seed)
    r = random.Random(seed)
    terms, seen, stack = [], set(), list(conj)
    while stack:
        n = stack.pop()
        if n.id in seen:
            continue
        seen.add(n.id)
        if n.width and n.width > 0 and not n.is_array:
            terms.append(n)
        stack.extend(n.args or ())
    r.shuffle(terms)
    p = compile_program(conj, trace=terms[:12])
    if not isa.asm_eligible(p.code, p.leaves, p.consts):
        pytest.skip("lowered outside the asm opcode set")
    assert p.n_trace_rows > 0
    for begin, n in (((1 << 33) + 77, 4096 + 3 * seed + 1), (seed, 255)):
        va, ta, vi, ti = both_traced(dev, p, DEFAULT_SEED + seed, begin, n)
        assert np.array_equal(va, vi), (seed, begin)
        assert np.array_equal(ta, ti), (seed, begin, int(np.count_nonzero(ta != ti)))


def test_asm_witness_programs_of_the_corpus(dev, corpus):
    """The witness program of every corpus query (its leaves traced) on the
    asm interpreter gives the compiled interpreter's rows."""
    from mythril_amd.engine import _witness_program
    checked = 0
    for name, q in corpus[:16] + corpus[-16:]:
        p = q.program
        wp = _witness_program(p, list(p.leaf_nodes))
        if not isa.asm_eligible(wp.code, wp.leaves, wp.consts) or not wp.n_trace_rows:
            continue
        va, ta, vi, ti = both_traced(dev, wp, DEFAULT_SEED, 1 << 20, 1000)
        assert np.array_equal(va, vi), name
        assert np.array_equal(ta, ti), name
        checked += 1
    assert checked


def test_asm_search_of_a_traced_program(dev):
    """A program with STOREs searched on the asm interpreter (no trace buffer:
    every STORE is a no-op) finds the compiled interpreter's lowest witness."""
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 8)
    conj = [c.app("bvult", x, c.const(1 << 250, 256)), c.app("=", y, c.const(77, 8))]
    p = compile_program(conj, trace=[x, y, c.app("bvadd", x, c.const(5, 256))])
    assert p.n_trace_rows > 0 and isa.asm_eligible(p.code, p.leaves, p.consts)
    dp = dev.load(p)
    try:
        assert dev.engine_of(dp) == "asm"
        for flags in (0, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            (fa,), sta = dev.search([dp], 11, 0, 1 << 16, flags)
            with compiled_interpreter():
                (fi,), sti = dev.search([dp], 11, 0, 1 << 16, flags)
            assert fa == fi and fa is not None, flags
    finally:
        dp.free()


def _shift_dag(seed):
    """Shifts by per-lane amounts (W_SHL / W_LSHR / W_ASHR, round 5): amounts
    drawn below the width (masked leaves), at and just past it, and whole
    random 256-bit values (>= w: zero, or the sign fill for ashr)."""
    r = random.Random(seed)
    c = Ctx()
    terms, conj = [], []
    for i in range(10):
        w = r.choice([33, 64, 100, 160, 255, 256])
        a = c.var(f"a{i}_{w}", w)
        amt = c.var(f"s{i}_{w}", w)
        k = r.random()
        if k < 0.5:      # below the width: mask to 8 bits, then reduce mod w
            amt = c.app("bvurem", c.app("bvand", amt, c.const(0x1FF, w)), c.const(w, w)) if r.random() < 0.3 \
                else c.app("bvand", amt, c.const((1 << max(1, (w - 1).bit_length() - 1)) - 1, w))
        elif k < 0.7:    # at or past the width by a little
            amt = c.app("bvadd", c.app("bvand", amt, c.const(3, w)), c.const(w - 2, w))
        op = r.choice(["bvshl", "bvlshr", "bvashr"])
        t = c.app(op, a, amt)
        terms.append(t)
        conj.append(c.app(r.choice(["bvult", "bvule", "bvslt"]), t, c.var(f"b{i}_{w}", w))
                    if r.random() < 0.5 else c.app("not", c.app("=", t, c.const(0, w))))
    return c, conj, terms


@pytest.mark.parametrize("seed", range(6))
def test_asm_variable_shifts(dev, seed):
    c, conj, terms = _shift_dag(9300 + seed)
    p = compile_program(conj, trace=terms)
    ops = {int(x) & 0xFF for x in list(p.code)[0::4]}
    assert ops & {isa.OPCODES[n] for n in ("W_SHL", "W_LSHR", "W_ASHR")}
    if not isa.asm_eligible(p.code, p.leaves, p.consts):
        pytest.skip("lowered outside the asm opcode set")
    for begin, n in ((seed, 4096 + 7), ((1 << 33) + 5, 300)):
        va, ta, vi, ti = both_traced(dev, p, DEFAULT_SEED + seed, begin, n)
        assert np.array_equal(va, vi), (seed, begin)
        assert np.array_equal(ta, ti), (seed, begin, int(np.count_nonzero(ta != ti)))
    pair = conj[2 * (seed % 5):2 * (seed % 5) + 2]
    va, vi = both(dev, compile_program(pair), DEFAULT_SEED + seed, 0, 1 << 12)
    _, _, vo = cdag.evaluate(pair, DEFAULT_SEED + seed, 0, 1 << 12, want_verdict=True)
    assert np.array_equal(va, vo) and np.array_equal(vi, vo)
    assert int(vo.sum()) > 0
