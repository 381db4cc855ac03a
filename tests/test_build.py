"""CPU checks of the native boundary: the C-ABI library exists, exports every
entry point include/mythril_witness.h declares, the Python ISA mirror matches
csrc/mw_isa.h, and program validation rejects malformed programs (no GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from mythril_amd import isa
from mythril_amd.compiler import compile_program
from mythril_amd.ir import Ctx
from mythril_amd.runtime import LIB_PATH, SIGNATURES, make_desc
from tests.helpers import host_emu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mythril_witness.h")
ISA_H = os.path.join(ROOT, "mythril_amd", "csrc", "mw_isa.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mg_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB_PATH), "run python -m mythril_amd.build"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, re.M))
    decl = declared_symbols()
    assert len(decl) >= 12
    missing = [s for s in decl if s not in exported]
    assert not missing, missing
    assert set(decl) == set(SIGNATURES), "runtime.py binds exactly the declared C-ABI"


def test_library_loads_without_gpu():
    lib = ctypes.CDLL(LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_library_contains_gfx950_code_object():
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_isa_header_matches_python_mirror():
    txt = open(ISA_H).read()
    found = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"MW_(\w+)\s*=\s*(\d+)", txt))
    for name, code in isa.OPCODES.items():
        assert found.get(name) == code, name
    assert int(re.search(r"#define MW_NW (\d+)", txt).group(1)) == isa.NW
    assert int(re.search(r"#define MW_NN (\d+)", txt).group(1)) == isa.NN
    assert int(re.search(r"#define MW_KBIT (0x[0-9a-f]+)u", txt).group(1), 16) == isa.KBIT


def _validate(p):
    lib = host_emu()
    d, keep = make_desc(p)
    return lib.mg_validate_desc(ctypes.byref(d))


def test_validation_accepts_compiled_and_rejects_malformed():
    c = Ctx()
    p = compile_program([c.app("bvult", c.var("a", 256), c.const(5, 256))])
    assert _validate(p) == 0
    bad = [
        lambda q: q.code.__setitem__(0, (int(q.code[0]) & 0xFFFFFF00) | 200),          # unknown opcode
        lambda q: q.code.__setitem__(-4, isa.OPCODES["CHECK"]),              # missing END
        lambda q: q.code.__setitem__(1, (q.code[1] & 0xFFFF0000) | 99),      # W dst slot 99
        lambda q: q.leaves.__setitem__(0, 0),                                # leaf width 0
    ]
    for f in bad:
        q = compile_program([c.app("bvult", c.var("a", 256), c.const(5, 256))])
        q.code = q.code.copy()
        q.leaves = q.leaves.copy()
        f(q)
        assert _validate(q) != 0
