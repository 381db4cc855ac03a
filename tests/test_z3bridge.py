"""mythril_amd/z3bridge.py without z3 (not installable here): a
minimal stand-in z3 module exercises the bridge's own code paths - to_ir's
print-and-parse, model_from_witness's pinning of scalars, array cells and
function points and its sat/unknown handling - and the drop-in must fail
closed (the reference answers) whenever the re-check raises or declines.
Bit-exactness against the real z3 stays unpinned."""
import sys
import types

import pytest

from mythril_amd import model as dropin
from mythril_amd import z3bridge
from mythril_amd.engine import Witness
from mythril_amd.smt2 import parse_script

DUMP = """(declare-fun x () (_ BitVec 8))
(declare-fun cd () (Array (_ BitVec 256) (_ BitVec 8)))
(declare-fun f ((_ BitVec 256)) (_ BitVec 256))
(declare-fun b () Bool)
(assert (bvugt x #x05))
"""


class FakeZ3(types.ModuleType):
    """Records what the bridge asks of z3; check() returns the configured answer."""

    def __init__(self, answer="sat"):
        super().__init__("z3")
        self.sat, self.unknown = "sat", "unknown"
        self.answer = answer
        self.pins = []
        self.Z3_OP_UNINTERPRETED = 2345
        z = self

        class Solver:
            def __init__(self):
                self.items = []

            def set(self, **kw):
                z.timeout = kw.get("timeout")

            def add(self, items):
                self.items.extend(items if isinstance(items, list) else [items])
                z.pins = self.items

            def sexpr(self):
                return DUMP

            def check(self):
                return z.answer

            def model(self):
                return ("z3-model", len(self.items))
        self.Solver = Solver
        self.BitVecSort = lambda w: ("sort", w)
        self.BitVecVal = lambda v, w: ("val", v, w)
        self.BoolVal = lambda v: ("bool", v)
        self.BitVec = lambda n, w: _Sym(n)
        self.Bool = lambda n: _Sym(n)
        self.Array = lambda n, d, r: _Sym(n)
        self.Select = lambda a, i: _Sym(("select", a.name, i))
        self.Function = lambda n, *sorts: (lambda *args: _Sym((n,) + args))


class _Sym:
    def __init__(self, name):
        self.name = name

    def __eq__(self, other):
        return ("pin", self.name, other)

    __hash__ = object.__hash__


@pytest.fixture
def fake_z3(monkeypatch):
    z = FakeZ3()
    monkeypatch.setitem(sys.modules, "z3", z)
    return z


def test_to_ir_parses_the_solver_text(fake_z3):
    from mythril_amd.ir import Ctx
    s = z3bridge.to_ir(["raw-assertion"], Ctx())     # the text route (a context of the caller's)
    assert [d for d in s.decls] == ["x", "cd", "f", "b"] and len(s.asserts) == 1


def test_model_from_witness_pins_every_kind_of_leaf(fake_z3):
    script = parse_script(DUMP)
    w = Witness(7, {"x": 9, "b": 1}, arrays={"cd": {4: 0xAB}}, functions={"f": {(3,): 77}})
    got = z3bridge.model_from_witness(["raw"], script, w, timeout_ms=123)
    assert got == ("z3-model", 5) and fake_z3.timeout == 123
    pins = fake_z3.pins[1:]
    assert ("pin", "x", ("val", 9, 8)) in pins and ("pin", "b", ("bool", True)) in pins
    assert ("pin", ("select", "cd", ("val", 4, 256)), ("val", 0xAB, 8)) in pins
    assert ("pin", ("f", ("val", 3, 256)), ("val", 77, 256)) in pins


def test_unconfirmed_witness_returns_none(fake_z3):
    fake_z3.answer = "unknown"
    assert z3bridge.model_from_witness(["raw"], parse_script(DUMP), Witness(0, {"x": 9})) is None


@pytest.mark.usefixtures("mythril")
def test_recheck_exception_goes_to_reference(monkeypatch, mythril):
    from tests.test_dropin import SAT

    def boom(*a, **k):
        raise RuntimeError("z3 exception during check")
    monkeypatch.setattr(z3bridge, "model_from_witness", boom)
    res = dropin.get_model(SAT)
    assert res.raw[0] == "ref" and dropin.STATS["recheck_errors"] >= 1


@pytest.mark.usefixtures("mythril")
def test_translation_exception_goes_to_reference(monkeypatch, mythril):
    from tests.test_dropin import SAT

    def boom(*a, **k):
        raise TypeError("sexpr of an unexpected AST")
    monkeypatch.setattr(z3bridge, "to_ir", boom)
    assert dropin.get_model(SAT).raw[0] == "ref"


from tests.test_dropin import mythril  # noqa: E402,F401  (the stand-in Mythril fixture)
