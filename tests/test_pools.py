"""Candidate pools (mythril_amd/pools.py): domain restriction and word-tied
calldata bytes.  The generated candidates are checked with the oracle's leaf
generator (tests/helpers.oracle_models), which mirrors csrc/mw_leaf.h."""
import os

from mythril_amd.compiler import compile_program
from mythril_amd.ir import Ctx
from mythril_amd.pools import ACTORS, domains, harvest
from tests.helpers import oracle_models


def _calldata_word(c, base, size):
    return c.app("concat", *[c.app("ite", c.app("bvslt", c.const(base + i, 256), size),
                                   c.var(f"1_calldata@{base + i:x}", 8), c.const(0, 8)) for i in range(32)])


def test_domains_exact_interval_alignment():
    c = Ctx()
    s = c.var("sender_1", 256)
    size = c.var("1_calldatasize", 256)
    h = c.var("keccak256_512@s1", 256)
    word0 = _calldata_word(c, 0, size)
    conj = [c.app("or", *[c.app("=", s, c.const(a, 256)) for a in ACTORS]),
            c.app("=", c.app("extract", word0, params=(255, 224)), c.const(0xA9059CBB, 32)),
            c.app("bvule", c.const(68, 256), size), c.app("not", c.app("bvuge", size, c.const(4096, 256))),
            c.app("or", c.app("and", c.app("bvule", c.const(1000, 256), h), c.app("bvult", h, c.const(5000, 256)),
                              c.app("=", c.app("bvurem", h, c.const(64, 256)), c.const(0, 256))), c.false())]
    exact, interval, align = domains(conj)
    assert exact["sender_1"] == ACTORS
    assert [exact[f"1_calldata@{i}"] for i in range(4)] == [[0xA9], [0x05], [0x9C], [0xBB]]
    assert "1_calldata@4" not in exact
    assert interval["1_calldatasize"] == [68, 4095]
    assert interval["keccak256_512@s1"] == [1000, 4999] and align["keccak256_512@s1"] == 64
    specs = harvest(conj, [s, size, h] + [c.var(f"1_calldata@{i:x}", 8) for i in range(32)])
    assert sorted(set(specs["sender_1"].pool)) == sorted(ACTORS)
    assert set(specs["1_calldata@0"].pool) == {0xA9}
    assert all(v is not None and 68 <= v <= 4095 for v in specs["1_calldatasize"].pool)
    assert all(v is not None and 1000 <= v < 5000 and v % 64 == 0 for v in specs["keccak256_512@s1"].pool)


def test_word_bytes_draw_one_entry_together():
    """The 32 bytes of an ABI argument pick the same word-level pool entry, so
    a proposed word value (here: count <= 20, value with 2^255) appears whole."""
    c = Ctx()
    size = c.var("1_calldatasize", 256)
    cnt = _calldata_word(c, 4, size)
    value = _calldata_word(c, 36, size)
    conj = [c.app("bvule", cnt, c.const(20, 256)), c.app("bvugt", cnt, c.const(0, 256)),
            c.app("not", c.app("bvumul_noovfl", cnt, value)), c.app("bvult", size, c.const(4096, 256))]
    leaves = [size] + [c.var(f"1_calldata@{i:x}", 8) for i in range(4, 68)]
    specs = harvest(conj, leaves)
    assert specs["1_calldata@5"].tie == "1_calldata@4" and specs["1_calldata@4"].tie is None
    p = compile_program(conj, leaf_specs=specs)
    lay = {s.name: (s.bits, s.shift, s.stride, s.hashed, s.key_salt()) for s in p.leaf_specs}
    assert len({lay[f"1_calldata@{i:x}"] for i in range(4, 36)}) == 1
    wpool = set()
    for k in range(len(specs["1_calldata@4"].pool)):
        if specs["1_calldata@4"].pool[k] is not None:
            wpool.add(int.from_bytes(bytes(specs[f"1_calldata@{i:x}"].pool[k] for i in range(4, 36)), "big"))
    assert {20, 1 << 255} <= wpool | {1 << 255} and 20 in wpool
    hits = 0
    for m in oracle_models(p, 0x5EED0003, 0, 512):
        w = int.from_bytes(bytes(m[f"1_calldata@{i:x}"] for i in range(4, 36)), "big")
        hits += w in wpool
        v = int.from_bytes(bytes(m[f"1_calldata@{i:x}"] for i in range(36, 68)), "big")
        if 0 < w <= 20 and w * v >= 1 << 256:
            break
    else:
        raise AssertionError("no overflowing (count, value) pair in 512 candidates")
    assert hits > 0


def test_launch_count_bounds_ops_per_launch():
    """engine.WitnessEngine.launch_count: a miss on an expensive query costs at
    most op_budget u32 ops before z3 answers."""
    from types import SimpleNamespace
    from mythril_amd.engine import MIN_CANDIDATES, WitnessEngine
    from tests.fakedev import FakeDevice
    eng = WitnessEngine(dev=FakeDevice(), budget=1 << 22, op_budget=(1 << 22) * 2000)
    q = lambda ops: SimpleNamespace(ops_per_eval=ops)   # noqa: E731
    assert eng.launch_count([q(1187)]) == 1 << 22
    assert eng.launch_count([q(14000)]) == (1 << 22) * 2000 // 14000
    assert eng.launch_count([q(10 ** 9)]) == MIN_CANDIDATES
    assert eng.launch_count([q(1000), q(1000), q(1000)]) == (1 << 22) * 2000 // 3000
    eng.op_budget = None
    assert eng.launch_count([q(10 ** 9)]) == 1 << 22


def test_congruence_trimming_is_sound():
    """lower._never_equal / _fold_offsets: pairs skipped are unequal under every
    assignment, and folded premises are equivalent (checked with the oracle on
    random assignments, widths 8 and 256)."""
    import random
    from mythril_amd.lower import _fold_offsets, _never_equal
    from oracle.dag_eval import eval_nodes
    rng = random.Random(5)
    for w in (8, 256):
        c = Ctx()
        b = c.var("b", w)
        terms = [b] + [c.app("bvadd", b, c.const(k, w)) for k in (1, 3, (1 << w) - 1, 1 << (w - 1))] + \
                [c.app("bvadd", c.const(7, w), b), c.const(5, w), c.const(9, w)]
        for x in terms:
            for y in terms:
                fx, fy = _fold_offsets(c, x, y)
                eq, feq = c.app("=", x, y), c.app("=", fx, fy)
                for _ in range(40):
                    v = rng.choice([0, 1, 5, 9, (1 << w) - 1, rng.getrandbits(w)])
                    vals = eval_nodes([eq, feq], {"b": v})
                    assert vals[eq.id] == vals[feq.id], (x, y, v)
                    if _never_equal(x, y):
                        assert not vals[eq.id], (x, y, v)


def test_congruence_conjuncts_fuse_to_one_check():
    """compiler._fuse_checks: C3's congruence conjuncts (a => b) become single
    CHECK_IMP instructions in the interpreter bytecode; Program.ssa (the
    specialised-kernel input) keeps the unfused pair."""
    import os
    from mythril_amd import isa
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    s = parse_file(os.path.join(os.path.dirname(__file__), "golden", "solver_log",
                                "c3_bec_batchtransfer_overflow.smt2"))
    q = prepare(s.asserts, s.ctx)
    ops = [int(w) & 0xFF for w in q.program.code.reshape(-1, 4)[:, 0]]
    # (key = K) => (v = w) with keyed premises (lower._Rewriter.keyed): no premise
    # flags; over one key they form complete grids (compiler._form_grids), one
    # CHECK_GRID per concrete cell over a table of the symbolic bytes
    code = q.program.code.reshape(-1, 4)
    rows = [r for r in code if int(r[0]) & 0xFF == isa.OPCODES["CHECK_GRID"]]
    pairs = sum(((int(r[2]) >> 26) & 31) + 1 for r in rows)    # n of each row's table (c = T0 | (n-1) << 10)
    assert pairs == 2176, pairs
    assert ops.count(isa.OPCODES["CHECK_IMPEQK"]) == 0
    assert ops.count(isa.OPCODES["N_EQ"]) < 60
    assert len(ops) < 800 and q.program.n_spill <= 80
    assert all(not i.op.startswith("CHECK_IMP") for i in q.program.machine_ir())


def test_index_keys_are_exact():
    """lower._index_key: for a premise constant e < KEY_LIMIT, key(b) = e holds
    exactly when b = e - KEY_BIAS (mod 2^w), at the wrap-around, at the
    sentinel's neighbours and for random words (the keyed premise replaces
    b = K - k in the congruence conjuncts)."""
    import random
    from mythril_amd.ir import Ctx
    from mythril_amd.lower import _Rewriter, KEY_BIAS, KEY_LIMIT
    from oracle.dag_eval import eval_nodes
    rng = random.Random(7)
    c = Ctx()
    w = 256
    b = c.var("b", w)
    rw = _Rewriter(c)
    key = rw._index_key(b)
    M = (1 << w) - 1
    for d in (0, 1, 4, 31, 1234, M, M - 30, KEY_LIMIT - KEY_BIAS - 1):
        e = (d + KEY_BIAS) & M
        if e >= KEY_LIMIT:
            continue
        prem = c.app("=", key, c.const(e, 32))
        for v in (d, (d + 1) & M, (d - 1) & M, d ^ (1 << 40), (d + (1 << 32)) & M, M, 0,
                  (0xFFFFFFFF - KEY_BIAS) & M, rng.getrandbits(w)):
            vals = eval_nodes([prem], {"b": v})
            assert bool(vals[prem.id]) == (v == d), (d, v)


def test_check_imp_verdicts_all_input_combinations():
    """the fused CHECK_IMP against the oracle on every (p, q) row,
    with Bool and bv1 premises/conclusions and constant operands, including the
    rejecting row p=1, q=0; the unfused program (as jit.py sees it) agrees."""
    from mythril_amd import isa
    from mythril_amd.compiler import compile_program
    from mythril_amd.runtime import pack_inputs
    from oracle.dag_eval import eval_nodes
    from tests.helpers import emu_eval
    c = Ctx()
    a, b = c.var("a", 0), c.var("b", 0)
    u, v = c.var("u", 1), c.var("v", 1)
    x = c.var("x", 8)
    t, f = c.true(), c.false()
    shapes = [
        [c.app("=>", a, b)],
        [c.app("=>", c.app("=", u, c.const(1, 1)), c.app("=", v, c.const(1, 1)))],
        [c.app("=>", c.app("bvule", u, v), b)],
        [c.app("=>", a, c.app("=", x, c.const(7, 8)))],
        [c.app("=>", t, b)], [c.app("=>", a, f)], [c.app("=>", f, b)], [c.app("=>", a, t)],
        [c.app("=>", a, b), c.app("=>", b, a)],
    ]
    models = [{"a": p, "b": q, "u": p, "v": q, "x": 7 if q else 3} for p in (0, 1) for q in (0, 1)]
    for conj in shapes:
        prog = compile_program(conj)
        ops = {int(w) & 0xFF for w in prog.code.reshape(-1, 4)[:, 0]}
        want = [int(all(eval_nodes(conj, m)[k.id] for k in conj)) for m in models]
        got, _ = emu_eval(prog, pack_inputs(prog, models), len(models))
        assert list(map(int, got)) == want, conj
        if not any(k.args[0].op == "const" or k.args[1].op == "const" for k in conj):
            assert ops & {isa.OPCODES[n] for n in ("CHECK_IMP", "CHECK_IMPEQ", "CHECK_IMPEQW", "CHECK_IMPEQK")}, conj
    assert [int(all(eval_nodes(shapes[0], m)[k.id] for k in shapes[0])) for m in models] == [1, 1, 0, 1]


def test_long_lived_prepare_replays_memoised_walks_and_scans():
    """C3 through a long-lived context (z3bridge.ConjunctCache's): its parent
    set, the full set and the full set again (the kept topo walks and the
    harvest's congruence-segment scan replayed, lower._topo_memo /
    pools._scan) compile to the program a fresh context gives."""
    from mythril_amd import z3bridge
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_script, to_smt2
    from tests import fakez3
    from tools.replay_latency import program_bytes
    import sys as _sys
    z = fakez3.module()
    old = _sys.modules.get("z3")
    _sys.modules["z3"] = z
    saved = z3bridge.solver_sexpr
    z3bridge.solver_sexpr = lambda raws: to_smt2([r.node for r in raws])
    try:
        text = open(os.path.join(os.path.dirname(__file__), "golden", "solver_log",
                                 "c3_bec_batchtransfer_overflow.smt2")).read()
        fresh = parse_script(text)
        want = program_bytes(prepare(fresh.asserts, fresh.ctx).program)
        ws = parse_script(text)
        raws = [z.ast(n) for n in ws.asserts]
        cache = z3bridge.ConjunctCache()
        sp = cache.to_ir(raws[:-1])
        prepare(sp.asserts, sp.ctx)
        for _ in range(2):
            sc = cache.to_ir(raws)
            q = prepare(sc.asserts, sc.ctx)
            assert q.lowered.harvest_split is not None
            assert program_bytes(q.program) == want
        assert any(isinstance(k, tuple) and k and k[0] == "seg" for k in sc.ctx._harvest)
    finally:
        z3bridge.solver_sexpr = saved
        if old is None:
            _sys.modules.pop("z3", None)
        else:
            _sys.modules["z3"] = old
