"""GPU parity: the gfx950 kernels (through the C-ABI) vs the oracle.

Every check compares device results with the CPU restatement in oracle/ on the
same inputs: random DAGs (all ops, widths 1..256), division/shift edge
values, generated candidates (Philox + pools), the reference's VMTests
post-storage values and vmSha3Test Keccak vectors, and witness search
(planted witness, early-exit == exhaustive, batched == individual).
"""
import json
import os
import random

import numpy as np
import pytest

from mythril_amd.compiler import LeafSpec, compile_program
from mythril_amd.ir import BOOL, Ctx, topo
from mythril_amd.runtime import LIB_PATH, Device, pack_inputs, unpack_trace
from mythril_amd import isa
from oracle.dag_eval import eval_nodes
from oracle.keccak import keccak256
from oracle.vmtest_runner import run_case, env_of
from tests.helpers import (RandDag, full_width_division_models, oracle_models, random_assignments,
                           short_division_models)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    d = Device(0)
    yield d
    d.close()


def test_native_library_is_the_in_tree_build(dev):
    maps = open("/proc/self/maps").read()
    assert os.path.realpath(LIB_PATH) in maps


def _parity(dev, conj, extra, models):
    nodes = [n for n in topo(conj + extra) if not n.is_array]
    p = compile_program(conj, trace=nodes)
    dp = dev.load(p)
    verdict, trace = dev.eval(dp, pack_inputs(p, models), len(models))
    for j, m in enumerate(models):
        vals = eval_nodes(conj + extra, m)
        assert verdict[j] == int(all(vals[c.id] for c in conj)), f"verdict {j}"
    for n in nodes:
        got = unpack_trace(p, trace, n)
        for j, m in enumerate(models):
            exp = eval_nodes([n], m)[n.id]
            assert got[j] == exp, f"{n!r}[{j}]: {got[j]:#x} != {exp:#x}"


@pytest.mark.parametrize("seed", range(30))
def test_random_dag_parity_gpu(dev, seed):
    rng = random.Random(1000 + seed)
    dag = RandDag(1000 + seed)
    conj = [dag.boolean(4) for _ in range(3)]
    extra = [dag.bv(rng.choice(dag.widths), 4) for _ in range(4)]
    _parity(dev, conj, extra, random_assignments(dag.vars + dag.bvars, 96, rng, dag))


@pytest.mark.parametrize("w", [8, 32, 64, 160, 256])
def test_division_and_shift_edges_gpu(dev, w):
    c = Ctx()
    a, b = c.var("a", w), c.var("b", w)
    ops = ["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvmul", "bvshl", "bvlshr", "bvashr"]
    terms = [c.app(op, a, b) for op in ops] + [c.app("bvumul_noovfl", a, b)]
    m = (1 << w) - 1
    sp = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, w, w + 1]
    rng = random.Random(w)
    models = [{"a": x & m, "b": y & m} for x in sp for y in sp]
    for _ in range(400):
        nb = rng.randint(1, w)
        y = rng.getrandbits(nb) | (1 << (nb - 1))
        models.append({"a": rng.getrandbits(w), "b": y & m})
    _parity(dev, [c.true()], terms, models)


@pytest.mark.parametrize("seed", range(3))
def test_full_width_divisors_gpu(dev, seed):
    """Waves whose every divisor is full width take the one-digit path
    (udivrem8_full, f64 estimate + add-back), waves of one-limb divisors the
    short division (udivrem8_short); the models come in blocks of 64, so every
    wave of each batch takes its path."""
    c = Ctx()
    a, b = c.var("a", 256), c.var("b", 256)
    terms = [c.app(op, a, b) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    _parity(dev, [c.true()], terms, full_width_division_models(seed, 64 * 12))
    _parity(dev, [c.true()], terms, short_division_models(seed, 64 * 12))


def test_generated_candidates_gpu(dev):
    c = Ctx()
    x, y, z = c.var("x", 256), c.var("y", 8), c.var("z", 160)
    conj = [c.app("bvult", x, c.const(1 << 255, 256)), c.app("=", y, c.const(3, 8))]
    p = compile_program(conj, trace=[x, y, z], pools={"y": [0, 1, 2, 3, None, 255], "z": [None, 7, 1 << 159]})
    dp = dev.load(p)
    seed, begin, n = 0x5EED0002, (1 << 40) + 12345, 4096
    verdict, trace = dev.eval_generated(dp, seed, begin, n)
    models = oracle_models(p, seed, begin, n)
    for node in (x, y, z):
        assert unpack_trace(p, trace, node) == [m[node.name] for m in models]
    assert [int(v) for v in verdict] == [int(m["x"] < (1 << 255) and m["y"] == 3) for m in models]


VMTESTS = [t for t in json.load(open(os.path.join(GOLD, "vmtests.json"))) if t["post_storage"]]


def test_vmtests_post_storage_on_gpu(dev):
    """The reference's VMTests, each SSTOREd value evaluated as a DAG on the device."""
    checked = 0
    for case in VMTESTS:
        ctx = Ctx()
        status, evm, checks = run_case(case, ctx)
        if status != "ok" or not checks:
            continue
        terms = [t for _, t, _ in checks]
        p = compile_program([ctx.true()], trace=terms)
        dp = dev.load(p)
        _, trace = dev.eval(dp, pack_inputs(p, [evm.model]), 1)
        for (slot, t, expected) in checks:
            got = unpack_trace(p, trace, t)[0]
            assert got == expected, f"{case['name']} slot {slot}: {got:#x} != {expected:#x}"
            checked += 1
        dp.free()
    assert checked >= 300


def test_keccak_gpu(dev):
    rng = random.Random(3)
    msgs = [b"", b"\0" * 5, b"a" * 135, b"b" * 136, b"c" * 137, bytes(range(256)) * 3]
    msgs += [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300))) for _ in range(2000)]
    out, st = dev.keccak256(msgs)
    assert out == [keccak256(m) for m in msgs]
    assert out[0].hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"


def _small_planted(n_nodes=600, n_conj=8, density_log2=10, seed=0x5EED0005):
    from mythril_amd.synth import build_c5
    from tests.helpers import oracle_models as om

    def ev(terms, index, sd):
        p = compile_program([], trace=list(terms))
        m = om(p, sd, index, 1)[0]
        vals = eval_nodes(list(terms), m)
        return [vals[t.id] for t in terms]
    return build_c5(ev, n_nodes=n_nodes, n_leaves=16, n_conj=n_conj, seed=seed,
                    witness_index=(1 << 17) + 77, density_log2=density_log2)


def test_search_finds_lowest_witness(dev):
    s = _small_planted()
    p = compile_program(s.conjuncts)
    dp = dev.load(p)
    count = 1 << 18
    (found,), st = dev.search([dp], s.seed, 0, count, 0)
    assert found is not None and found <= s.witness_index
    # the found index is a witness (oracle) and no lower index satisfies (device sweep)
    m = oracle_models(p, s.seed, found, 1)[0]
    vals = eval_nodes(s.conjuncts, m)
    assert all(vals[c.id] for c in s.conjuncts)
    v, _ = dev.eval_generated(dp, s.seed, 0, found, trace=False)
    assert int(v.sum()) == 0
    # oracle spot-check of the sweep on random indices below the witness
    rng = random.Random(9)
    for idx in rng.sample(range(found), 24):
        mm = oracle_models(p, s.seed, idx, 1)[0]
        vv = eval_nodes(s.conjuncts, mm)
        assert not all(vv[c.id] for c in s.conjuncts)
    assert st["evals"] == count


def test_early_exit_and_batching_agree_with_exhaustive(dev):
    progs = []
    for k in range(4):
        s = _small_planted(n_nodes=300, n_conj=6, density_log2=8 + k, seed=0x5EED0005 + k)
        progs.append(dev.load(compile_program(s.conjuncts)))
    count = 1 << 17
    ex, _ = dev.search(progs, 0x5EED0005, 0, count, 0)
    ee, _ = dev.search(progs, 0x5EED0005, 0, count, isa.FLAG_EARLY_EXIT)
    st, _ = dev.search(progs, 0x5EED0005, 0, count, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT)
    singles = [dev.search([p], 0x5EED0005, 0, count, 0)[0][0] for p in progs]
    assert ex == ee == st == singles


def test_invalid_program_rejected(dev):
    c = Ctx()
    p = compile_program([c.app("bvult", c.var("a", 256), c.const(5, 256))])
    p.code = p.code.copy()
    p.code[0] = (int(p.code[0]) & 0xFFFFFF00) | 200  # unknown opcode
    with pytest.raises(Exception):
        dev.load(p)


def test_division_rare_paths_gpu(dev):
    from tests.helpers import division_check_programs
    for p in division_check_programs():
        dp = dev.load(p)
        v, _ = dev.eval_generated(dp, 1, 0, 256, trace=False)
        assert int(v.sum()) == 256
        dp.free()


def test_keccak_service_on_device(dev):
    """mythril_amd.keccak_service over mg_keccak256: one launch for a batch of
    distinct messages, memo answers repeats, replace_with_actual_sha output
    identical to the per-window reference loop (tests/test_keccak_service.py)."""
    from mythril_amd.keccak_service import KeccakService, replace_with_actual_sha
    from tests.test_keccak_service import _placeholder, _reference_replace
    svc = KeccakService(device=dev, reference=None, min_batch=1)
    rng = random.Random(17)
    # mapping-slot preimages of the three LASER actors x 300 slots (512-bit concat(key, slot))
    actors = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
              0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]
    pre = [(512, (a << 256) | s) for a in actors for s in range(300)]
    assert svc.prefetch_values(pre) == len(pre)
    assert svc.stats["launches"] == 1 and svc.stats["gpu_hashes"] == len(pre)
    for size, v in pre[::37]:
        assert svc.find_concrete_keccak_int(v, size) == int.from_bytes(keccak256(v.to_bytes(64, "big")), "big")
    assert svc.stats["launches"] == 1
    holders = [_placeholder(rng) for _ in range(40)]
    table = {h: (256, rng.getrandbits(256)) for h in holders[:30]}
    txs = [{"input": "0x" + "a9059cbb" + "".join("%064x" % rng.choice(holders) for _ in range(6))}
           for _ in range(8)]
    ref = [dict(t) for t in txs]
    replace_with_actual_sha(txs, table.get, svc)
    _reference_replace(ref, table.get)
    assert txs == ref
    assert svc.stats["launches"] == 2
