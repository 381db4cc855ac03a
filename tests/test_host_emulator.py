"""CPU parity: compiler + bytecode + the interpreter/ALU code (host build) vs the oracle.

The host emulator (build/host/libmw_host_emu.so) is the *same* mw_interp.h /
mw_alu.h / mw_leaf.h / mw_keccak.h source the gfx950 kernels run, compiled
for x86; the GPU tests (test_gpu_parity.py) then repeat these checks on the
device.  Random DAGs cover every lowered op at widths 1..256.
"""
import random

import numpy as np
import pytest

from mythril_amd.compiler import compile_program
from mythril_amd.ir import BOOL, topo
from mythril_amd.runtime import pack_inputs, unpack_trace
from oracle.dag_eval import eval_nodes
from oracle.keccak import keccak256
from tests.helpers import RandDag, emu_eval, host_emu, oracle_models, random_assignments


def _check_program(dag, conj, extra, ncand, rng):
    nodes = [n for n in topo(conj + extra) if not n.is_array]
    p = compile_program(conj, trace=nodes)
    models = random_assignments(dag.vars + dag.bvars, ncand, rng, dag)
    inp = pack_inputs(p, models)
    verdict, trace = emu_eval(p, inp, ncand)
    for j, m in enumerate(models):
        vals = eval_nodes(conj + extra, m)
        exp_verdict = int(all(vals[c.id] for c in conj))
        assert verdict[j] == exp_verdict, f"verdict cand {j}"
    for n in nodes:
        got = unpack_trace(p, trace, n)
        for j, m in enumerate(models):
            exp = eval_nodes([n], m)[n.id]
            assert got[j] == exp, f"node {n!r} cand {j}: got {got[j]:#x} want {exp:#x}"
    return p


@pytest.mark.parametrize("seed", range(40))
def test_random_dag_parity(seed):
    rng = random.Random(seed)
    dag = RandDag(seed)
    conj = [dag.boolean(4) for _ in range(3)]
    extra = [dag.bv(rng.choice(dag.widths), 4) for _ in range(4)]
    _check_program(dag, conj, extra, 24, rng)


@pytest.mark.parametrize("w", [8, 32, 64, 160, 256])
@pytest.mark.parametrize("op", ["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvmul", "bvshl",
                                "bvlshr", "bvashr"])
def test_binary_op_edge_values(op, w):
    rng = random.Random(hash((op, w)) & 0xFFFF)
    dag = RandDag(1, widths=[w], nvars=2)
    a, b = dag.ctx.var("a", w), dag.ctx.var("b", w)
    t = dag.ctx.app(op, a, b)
    p = compile_program([dag.ctx.true()], trace=[t])
    m = (1 << w) - 1
    specials = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, (1 << (w - 1)) + 1, w, w - 1, w + 1]
    models = [{"a": x, "b": y} for x in specials for y in specials]
    models += [{"a": rng.getrandbits(w), "b": rng.getrandbits(rng.randint(1, w))} for _ in range(200)]
    # divisor-shape stress for Knuth D: divisors with 1..8 significant limbs, quotient digits near 2^32
    for _ in range(200):
        nb = rng.randint(1, w)
        y = rng.getrandbits(nb) | (1 << (nb - 1))
        x = (y * rng.getrandbits(max(1, w - nb + 1)) + rng.getrandbits(max(1, nb - 1))) & m
        models.append({"a": x, "b": y})
    inp = pack_inputs(p, [{"a": mm["a"] & m, "b": mm["b"] & m} for mm in models])
    _, trace = emu_eval(p, inp, len(models))
    got = unpack_trace(p, trace, t)
    for j, mm in enumerate(models):
        exp = eval_nodes([t], {"a": mm["a"] & m, "b": mm["b"] & m})[t.id]
        assert got[j] == exp, f"{op}/{w} a={mm['a']:#x} b={mm['b']:#x}: {got[j]:#x} != {exp:#x}"


def test_generated_candidates_match_oracle_philox_and_pools():
    dag = RandDag(7, widths=[8, 64, 256])
    x, y, z = dag.ctx.var("x", 256), dag.ctx.var("y", 8), dag.ctx.var("z", 64)
    conj = [dag.ctx.app("bvult", x, dag.ctx.const(1 << 255, 256)), dag.ctx.app("=", y, dag.ctx.const(3, 8))]
    pools = {"y": [0, 1, 2, 3, None, 255], "z": [None, 7]}
    p = compile_program(conj, trace=[x, y, z], pools=pools)
    seed, begin, n = 0x5EED0002, 1000, 64
    verdict, trace = emu_eval(p, None, n, seed=seed, begin=begin)
    models = oracle_models(p, seed, begin, n)
    for node in (x, y, z):
        got = unpack_trace(p, trace, node)
        assert got == [m[node.name] for m in models]
    for j, m in enumerate(models):
        assert verdict[j] == int(m["x"] < (1 << 255) and m["y"] == 3)


def test_hashed_pools_match_oracle():
    from mythril_amd.compiler import LeafSpec
    dag = RandDag(8, widths=[8, 256])
    c = dag.ctx
    xs = [c.var(f"h{i}", 8) for i in range(6)]
    big = c.var("big", 256)
    specs = {f"h{i}": LeafSpec(f"h{i}", 8, pool=[i, 0x41, None, 0xFF, 7], hashed=True) for i in range(6)}
    specs["big"] = LeafSpec("big", 256, pool=[None, 1 << 200, 5], hashed=True)
    p = compile_program([c.true()], trace=xs + [big], leaf_specs=specs)
    seed, begin, n = 3, (1 << 50) + 9, 300
    _, trace = emu_eval(p, None, n, seed=seed, begin=begin)
    models = oracle_models(p, seed, begin, n)
    for node in xs + [big]:
        assert unpack_trace(p, trace, node) == [m[node.name] for m in models]


def test_spilling_under_pressure():
    """More simultaneously-live wide values than W slots forces SPILL/FILL."""
    dag = RandDag(3, widths=[256])
    c = dag.ctx
    vs = [c.var(f"s{i}", 256) for i in range(40)]
    prods = [c.app("bvmul", vs[i], vs[(i + 1) % 40]) for i in range(40)]
    total = c.app("bvadd", *prods)
    xorall = c.app("bvxor", *prods)
    conj = [c.app("bvult", total, xorall)]
    p = compile_program(conj, trace=[total, xorall])
    assert p.n_spill > 0 and p.stats["spills"] > 0
    rng = random.Random(5)
    models = [{v.name: rng.getrandbits(256) for v in vs} for _ in range(16)]
    _, trace = emu_eval(p, pack_inputs(p, models), 16)
    for node in (total, xorall):
        got = unpack_trace(p, trace, node)
        for j, m in enumerate(models):
            assert got[j] == eval_nodes([node], m)[node.id]


def test_host_keccak_matches_oracle():
    import ctypes
    lib = host_emu()
    rng = random.Random(11)
    msgs = [b"", b"\x00" * 5, b"a" * 135, b"b" * 136, b"c" * 137, bytes(rng.getrandbits(8) for _ in range(700))]
    data = b"".join(msgs)
    off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint64)
    ln = np.array([len(m) for m in msgs], dtype=np.uint32)
    out = np.zeros(32 * len(msgs), dtype=np.uint8)
    lib.mwh_keccak256(ctypes.c_char_p(data), off.ctypes.data, ln.ctypes.data, len(msgs), out.ctypes.data)
    for i, m in enumerate(msgs):
        assert out[32 * i:32 * i + 32].tobytes() == keccak256(m)


def test_division_rare_correction_paths():
    """Quotient estimates one too large (add-back) and equal top words (qhat =
    B-1) are rare on random operands; these pairs reach both (udivrem8)."""
    from tests.helpers import division_stress_pairs
    dag = RandDag(1, widths=[256], nvars=2)
    a, b = dag.ctx.var("a", 256), dag.ctx.var("b", 256)
    terms = [dag.ctx.app(op, a, b) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    p = compile_program([dag.ctx.true()], trace=terms)
    pairs = division_stress_pairs(400, 11)
    models = [{"a": x, "b": y} for x, y in pairs]
    _, trace = emu_eval(p, pack_inputs(p, models), len(models))
    for t in terms:
        got = unpack_trace(p, trace, t)
        for j, mm in enumerate(models):
            assert got[j] == eval_nodes([t], mm)[t.id], f"{t.op} a={mm['a']:#x} b={mm['b']:#x}"


@pytest.mark.parametrize("seed", range(3))
def test_full_width_divisors(seed):
    """The one-digit path for divisors with a nonzero top limb (udivrem8_full):
    estimate never too small, add-back corrections, digits near 2^32-1."""
    from tests.helpers import full_width_division_models, short_division_models
    dag = RandDag(1, widths=[256], nvars=2)
    a, b = dag.ctx.var("a", 256), dag.ctx.var("b", 256)
    terms = [dag.ctx.app(op, a, b) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    p = compile_program([dag.ctx.true()], trace=terms)
    models = full_width_division_models(seed, 64 * 12) + short_division_models(seed, 64 * 12)
    _, trace = emu_eval(p, pack_inputs(p, models), len(models))
    for t in terms:
        got = unpack_trace(p, trace, t)
        for j, mm in enumerate(models):
            assert got[j] == eval_nodes([t], mm)[t.id], f"{t.op} a={mm['a']:#x} b={mm['b']:#x}"
