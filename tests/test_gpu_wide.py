"""Wide (> 256-bit) terms on gfx950: the programs of tests/test_wide.py (257-bit
BVAddNoOverflow, 257/300/512/1024-bit add/sub/compare, structure and constant
shifts, random wide DAGs) evaluated by the device interpreter through the
C-ABI (mg_eval) must match the oracle's evaluation of the original formula."""
import pytest

from tests import test_wide as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device_eval():
    from mythril_amd.runtime import Device
    dev = Device(0)

    def run(p, inputs, n):
        dp = dev.load(p)
        try:
            v, _ = dev.eval(dp, inputs, n, trace=False)
        finally:
            dp.free()
        return v
    W.RUN["eval"] = run
    yield
    W.RUN["eval"] = W.host_run
    dev.close()


def test_bvadd_no_overflow_257():
    W.test_bvadd_no_overflow_257_bit_pattern()


@pytest.mark.parametrize("w", [257, 300, 512, 1024])
def test_add_sub_compare(w):
    W.test_wide_add_sub_compare(w)


@pytest.mark.parametrize("w", [257, 512])
def test_structure_and_shifts(w):
    W.test_wide_structure_and_constant_shifts(w)


@pytest.mark.parametrize("seed", range(16))
def test_random_wide_dags(seed):
    W.test_random_wide_dags(seed)
