"""GPU parity of the specialised-kernel tier (mythril_amd/jit.py) through the C-ABI.

A program with an attached specialised kernel must give exactly the
interpreter's verdicts and witness indices (and the oracle's, spot-checked)
on the same generated candidates, in exhaustive, early-exit and
stop-after-hit modes, alone and batched with interpreted programs; a code
object generated for another program is refused.
"""
import random

import numpy as np
import pytest

from mythril_amd import isa, jit
from mythril_amd.compiler import compile_program
from mythril_amd.ir import topo
from oracle.dag_eval import eval_nodes
from tests.helpers import oracle_models


def small_planted(n_nodes=600, n_conj=8, density_log2=10, seed=0x5EED0005, witness_index=(1 << 17) + 77):
    from mythril_amd.synth import build_c5

    def ev(terms, index, sd):
        p = compile_program([], trace=list(terms))
        m = oracle_models(p, sd, index, 1)[0]
        vals = eval_nodes(list(terms), m)
        return [vals[t.id] for t in terms]
    return build_c5(ev, n_nodes=n_nodes, n_leaves=16, n_conj=n_conj, seed=seed,
                    witness_index=witness_index, density_log2=density_log2)


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def planted():
    return [small_planted(n_nodes=300, n_conj=6, density_log2=8 + k, seed=0x5EED0005 + k) for k in range(3)]


@pytest.fixture(scope="module")
def random_progs():
    from tests.test_jit import _random_programs
    return _random_programs(8, 9100)


@pytest.fixture(scope="module")
def images(planted, random_progs):
    from tests.helpers import division_check_programs
    progs = [compile_program(s.conjuncts) for s in planted] + [p for *_, p in random_progs] + \
        division_check_programs()
    image, names, _ = jit.compile_device(progs)  # one module, one hipcc run
    return progs, image, names


pytestmark = pytest.mark.gpu


def planted_names(images):
    return images[2][:3]


def _pair(dev, p, image, name):
    a = dev.load(p)
    b = dev.load(p)
    dev.attach_kernel(b, image, name)
    assert dev.has_kernel(b) and not dev.has_kernel(a)
    return a, b


def test_random_dag_verdicts_match_interpreter_and_oracle(dev, images, random_progs):
    progs, image, names = images
    k0 = len(planted_names(images))
    seed, begin, n = 0x5EED0009, (1 << 36) + 5, 8192
    for (dag, conj, extra, nodes, p), name in zip(random_progs, names[k0:]):
        a, b = _pair(dev, p, image, name)
        va, _ = dev.eval_generated(a, seed, begin, n, trace=False)
        vb, _ = dev.eval_generated(b, seed, begin, n, trace=False)
        assert np.array_equal(va, vb), name
        rng = random.Random(1)
        idx = rng.sample(range(n), 64)
        models = oracle_models(p, seed, begin, n)
        for j in idx:
            vals = eval_nodes(conj, models[j])
            assert int(vb[j]) == int(all(vals[c.id] for c in conj)), f"{name} cand {j}"
        a.free()
        b.free()


def test_division_rare_paths(dev, images):
    progs, image, names = images
    for p, name in zip(progs[-5:], names[-5:]):
        dp = dev.load(p)
        dev.attach_kernel(dp, image, name)
        v, _ = dev.eval_generated(dp, 1, 0, 256, trace=False)
        assert int(v.sum()) == 256, name
        dp.free()


def test_search_modes_match_interpreter(dev, images, planted):
    progs, image, names = images
    count = 1 << 18
    for s, p, name in zip(planted, progs, names):
        a, b = _pair(dev, p, image, name)
        for flags in (0, isa.FLAG_EARLY_EXIT, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            (fa,), sa = dev.search([a], s.seed, 0, count, flags)
            (fb,), sb = dev.search([b], s.seed, 0, count, flags)
            assert fa == fb, (name, flags)
            if flags == 0:
                assert sa["evals"] == sb["evals"] == count
        assert fb is not None and fb <= s.witness_index
        m = oracle_models(p, s.seed, fb, 1)[0]
        vals = eval_nodes(s.conjuncts, m)
        assert all(vals[c.id] for c in s.conjuncts)
        a.free()
        b.free()


def test_mixed_batch(dev, images, planted):
    progs, image, names = images
    dps = []
    for k, (p, name) in enumerate(zip(progs[:3], names[:3])):
        dp = dev.load(p)
        if k != 1:  # programs 0 and 2 specialised, 1 interpreted
            dev.attach_kernel(dp, image, name)
        dps.append(dp)
    count = 1 << 17
    got, st = dev.search(dps, 0x5EED0005, 0, count, 0)
    singles = [dev.search([dev.load(p)], 0x5EED0005, 0, count, 0)[0][0] for p in progs[:3]]
    assert got == singles
    assert st["launches"] == 3 and st["evals"] == 3 * count


def test_signature_mismatch_refused(dev, images):
    progs, image, names = images
    dp = dev.load(progs[0])
    with pytest.raises(Exception):
        dev.attach_kernel(dp, image, names[1])  # kernel of another program
    assert not dev.has_kernel(dp)


@pytest.fixture(scope="module")
def images_lds(planted, random_progs):
    progs = [compile_program(s.conjuncts) for s in planted] + [p for *_, p in random_progs]
    image, names, _ = jit.compile_device(progs, lds_leaves=4)
    return progs, image, names


def test_lds_leaves_match_interpreter(dev, images_lds, planted):
    """Specialised kernels that keep leaves in LDS: same verdicts and witnesses."""
    progs, image, names = images_lds
    seed, n = 0x5EED0009, 8192
    for p, name in zip(progs[3:], names[3:]):
        a, b = _pair(dev, p, image, name)
        va, _ = dev.eval_generated(a, seed, 5, n, trace=False)
        vb, _ = dev.eval_generated(b, seed, 5, n, trace=False)
        assert np.array_equal(va, vb), name
        a.free()
        b.free()
    for s, p, name in zip(planted, progs[:3], names[:3]):
        a, b = _pair(dev, p, image, name)
        for flags in (0, isa.FLAG_EARLY_EXIT):
            assert dev.search([a], s.seed, 0, 1 << 17, flags)[0] == dev.search([b], s.seed, 0, 1 << 17, flags)[0]
        a.free()
        b.free()


def test_split_program_parts_match_interpreter(dev, planted):
    """A program run as several part kernels (alive bits passed between them)
    gives the interpreter's witnesses and verdicts, in every search mode."""
    for s in planted[:2]:
        p = compile_program(s.conjuncts)
        a = dev.load(p)
        b = dev.load(p)
        jit.attach(dev, [b], split=True, part_weight=3000, lds_leaves=2)
        assert dev.has_kernel(b) and "parts" in b.kernel
        for flags in (0, isa.FLAG_EARLY_EXIT, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT):
            assert dev.search([a], s.seed, 0, 1 << 18, flags)[0] == dev.search([b], s.seed, 0, 1 << 18, flags)[0]
        va, _ = dev.eval_generated(a, s.seed, s.witness_index - 5000, 6000, trace=False)
        vb, _ = dev.eval_generated(b, s.seed, s.witness_index - 5000, 6000, trace=False)
        assert np.array_equal(va, vb) and vb[5000] == 1
        a.free()
        b.free()


def test_constant_divisors_specialised(dev):
    """Divisions by literal divisors (folded by LLVM in the specialised kernel),
    d = 2^31 after normalisation included: every pooled candidate satisfies."""
    from tests.helpers import constant_divisor_programs
    progs = constant_divisor_programs()
    image, names, _ = jit.compile_device(progs)
    for p, name in zip(progs, names):
        for special in (True, False):
            dp = dev.load(p)
            if special:
                dev.attach_kernel(dp, image, name)
            v, _ = dev.eval_generated(dp, 1, 0, 256, trace=False)
            assert int(v.sum()) == 256, (name, special)
            dp.free()


def test_mul_cols_against_oracle(dev):
    """mw_jit.h mul8_cols (the column multiply of two register operands) on
    carry-heavy operand pairs: every candidate asserts bvmul(a, b) == e with e
    the oracle's product (tests/helpers.mul_check_programs), so every verdict
    over the pool must be 1, on the kernel built with and without the columns
    and on the interpreter."""
    from tests.helpers import mul_check_programs
    (p,) = mul_check_programs()
    src = jit.generate([p], [jit.kernel_name(p)], mul_cols=True)
    assert "jit::w_mulv(" in src
    n = 4096
    for cols in (True, False):
        image, names, _ = jit.compile_device([p], mul_cols=cols)
        a, b = _pair(dev, p, image, names[0])
        va, _ = dev.eval_generated(a, 1, 0, n, trace=False)
        vb, _ = dev.eval_generated(b, 1, 0, n, trace=False)
        assert int(va.sum()) == n, "interpreter"
        assert int(vb.sum()) == n, f"specialised kernel, mul_cols={cols}: {n - int(vb.sum())} wrong products"
        a.free()
        b.free()
