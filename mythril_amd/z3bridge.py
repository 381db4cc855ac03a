"""z3 <-> witness-engine glue (used only inside a Mythril process, where z3 exists).

* ``to_ir``: a list of z3 ``BoolRef`` -> the solver script text (exactly the
  ``Optimize.sexpr()`` form ``--solver-log`` writes, ``mythril/support/model.py:45-56``)
  -> :mod:`mythril_amd.smt2` -> IR conjuncts.
* ``model_from_witness``: re-checks a GPU witness *in z3* on the exact same
  constraints (including the current keccak conditions) by pinning every free
  symbol / array cell / function application to the witness values, and
  returns z3's model of that query — so the caller gets a genuine
  ``z3.ModelRef`` (what ``Optimize.model()`` returns, ``solver.py:68-77``),
  or ``None`` if z3 does not confirm it (then the reference path runs).
"""
from __future__ import annotations

import logging
from typing import List, Optional, Sequence

from .engine import Witness
from .ir import Ctx
from .smt2 import Script, parse_script

log = logging.getLogger(__name__)


def _z3():
    import z3  # noqa: WPS433 - only available inside Mythril's environment
    return z3


def var_name(raw) -> Optional[str]:
    """The declaration name of a z3 constant (an uninterpreted 0-ary symbol), else None."""
    try:
        if raw.num_args() == 0 and raw.decl().kind() == _z3().Z3_OP_UNINTERPRETED:
            return raw.decl().name()
    except Exception:
        return None
    return None


def to_ir(raws: Sequence, ctx: Optional[Ctx] = None) -> Script:
    z3 = _z3()
    s = z3.Solver()
    s.add(list(raws))
    return parse_script(s.sexpr(), ctx)


def model_from_witness(raws: Sequence, script: Script, w: Witness, timeout_ms: int = 2000):
    z3 = _z3()
    s = z3.Solver()
    s.set(timeout=max(1, int(timeout_ms)))
    s.add(list(raws))
    pins: List = []
    for name, d in script.decls.items():
        if d.args:
            fn_vals = w.functions.get(name)
            if not fn_vals:
                continue
            f = z3.Function(name, *[z3.BitVecSort(a.width) for a in d.args], z3.BitVecSort(d.sort.width))
            for args, val in fn_vals.items():
                zargs = [z3.BitVecVal(a, srt.width) for a, srt in zip(args, d.args)]
                pins.append(f(*zargs) == z3.BitVecVal(val, d.sort.width))
            continue
        if d.sort.kind == "array":
            cells = w.arrays.get(name)
            if not cells:
                continue
            arr = z3.Array(name, z3.BitVecSort(d.sort.dom), z3.BitVecSort(d.sort.width))
            for idx, val in cells.items():
                pins.append(z3.Select(arr, z3.BitVecVal(idx, d.sort.dom)) == z3.BitVecVal(val, d.sort.width))
        elif name in w.values:
            if d.sort.kind == "bool":
                pins.append(z3.Bool(name) == z3.BoolVal(bool(w.values[name])))
            else:
                pins.append(z3.BitVec(name, d.sort.width) == z3.BitVecVal(w.values[name], d.sort.width))
    s.add(pins)
    r = s.check()
    if r == z3.sat:
        return s.model()
    log.warning("z3 did not confirm a GPU witness (%s); falling back to the reference solver", r)
    return None
