"""The engine scenarios of tests/test_engine_cpu.py on the device, through the C-ABI.

Same formulas (the reference's keccak UF and calldata sat/unsat expectations,
tests/laser/keccak_tests.py:7-145 and tests/laser/state/calldata_test.py:42-91,
plus the dispatcher-selector shape), same soundness check of every witness
against the oracle on the ORIGINAL formula; only the engine's device is the
MI355X instead of the host emulator.
"""
import pytest

import tests.test_engine_cpu as cpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_engine():
    from mythril_amd.engine import WitnessEngine
    from mythril_amd.runtime import Device
    dev = Device(0)
    yield lambda budget=1 << 14: WitnessEngine(dev=dev, seed=0x5EED0001, budget=budget)
    dev.close()


@pytest.fixture(autouse=True)
def on_gpu(monkeypatch, gpu_engine):
    monkeypatch.setattr(cpu, "engine", gpu_engine)


test_keccak_basic = cpu.test_keccak_basic
test_keccak_symbol_and_val_unsat = cpu.test_keccak_symbol_and_val_unsat
test_keccak_simple_number_unsat = cpu.test_keccak_simple_number_unsat
test_keccak_complex_eq_unsat = cpu.test_keccak_complex_eq_unsat
test_keccak_other_num_sat_witness_is_sound = cpu.test_keccak_other_num_sat_witness_is_sound
test_symbolic_calldata_constrain_index_unsat = cpu.test_symbolic_calldata_constrain_index_unsat
test_symbolic_calldata_equal_indices_unsat = cpu.test_symbolic_calldata_equal_indices_unsat
test_function_selector_dispatch_sat = cpu.test_function_selector_dispatch_sat
test_batched_search_equals_individual = cpu.test_batched_search_equals_individual


def test_engine_runs_on_the_device(gpu_engine):
    from mythril_amd.runtime import Device
    assert isinstance(gpu_engine().dev, Device)
