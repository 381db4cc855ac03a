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
    prog_h = open(os.path.join(os.path.dirname(ISA_H), "mw_prog.h")).read()   # not in the jit cache key
    assert int(re.search(r"#define MW_ASM_NK (\d+)u", prog_h).group(1)) == isa.ASM_NK
    from mythril_amd import asmgen
    assert int(re.search(r"#define MW_ASM_NK_INDEX (\d+)u", prog_h).group(1)) == asmgen.NK_INDEX


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


def test_reserved_write_back_slots():
    """W7 and N31/N63 are the interpreter's write-back scratch slots: the
    allocator never hands them out and the validator rejects them."""
    c = Ctx()
    # enough live values to use every allocatable slot of both files
    ws = [c.var(f"w{i}", 256) for i in range(20)]
    ns = [c.var(f"n{i}", 8) for i in range(90)]
    conj = [c.app("bvult", c.app("bvadd", *ws), c.app("bvxor", *ws)),
            c.app("=", c.app("bvadd", *ns), c.app("bvxor", *ns))]
    p = compile_program(conj)
    assert _validate(p) == 0
    from mythril_amd.isa import SHAPES
    inv = {v: k for k, v in isa.OPCODES.items()}
    used_w, used_n = set(), set()
    for w0, w1, w2, _ in p.code.reshape(-1, 4):
        op = inv[int(w0) & 0xFF]
        dcls, srcs = SHAPES[op]
        wd, nd = isa.decode_dst(int(w1) & 0xFFFF)
        if dcls == "W":
            used_w.add(wd)
        elif dcls == "N":
            used_n.add(nd)
        else:
            assert (wd, nd) == (None, None)
        fields = [int(w1) >> 16, int(w2) & 0xFFFF, int(w2) >> 16]
        for cls, f in zip(srcs, fields):
            if cls and not f & isa.KBIT:
                (used_w if cls == "W" else used_n).add(f)
    assert isa.W_RESERVED not in used_w and len(used_w) == isa.NW - 1
    assert isa.N_RESERVED not in used_n and 63 not in used_n and len(used_n) > 32
    for bad_dst in (isa.W_RESERVED,):
        q = compile_program([c.app("bvult", c.var("a", 256), c.const(5, 256))])
        q.code = q.code.copy()
        k = next(i for i in range(0, q.code.size, 4) if inv[int(q.code[i]) & 0xFF] == "LEAF_W")
        q.code[k + 1] = (int(q.code[k + 1]) & 0xFFFF0000) | isa.encode_dst("W", bad_dst)
        assert _validate(q) != 0


def test_spill_words_hottest_first():
    """Spill slots are word offsets (W: 8 words, N: 1), most-accessed first, so
    the LDS-resident prefix of the spill area holds the hot ones."""
    from mythril_amd.compiler import _layout_spills, MInsn
    insns = ([MInsn("SPILL_W", 0, None, [], imm=0)] + [MInsn("FILL_N", 0, None, [], imm=1)] * 5
             + [MInsn("SPILL_N", 0, None, [], imm=2)] + [MInsn("FILL_W", 0, None, [], imm=0)] * 3)
    out, words = _layout_spills([MInsn(i.op, 0, None, [], imm=i.imm) for i in insns], ["W", "N", "N"])
    assert words == 10
    offs = {(i.op, i.imm) for i in out}
    # N slot 1 (6 accesses / 1 word) first, then N slot 2 (1/1), then W slot 0 (4/8)
    assert ("FILL_N", 0) in offs and ("SPILL_N", 1) in offs and ("SPILL_W", 2) in offs and ("FILL_W", 2) in offs


def test_cdins_chain_flag_set_and_validated():
    """W_CDINS chains (a calldata word built byte by byte) carry MW_FLAG_CHAIN
    on every link whose result only feeds the next link; the validator rejects
    the flag anywhere else."""
    from mythril_amd.smt2 import parse_file
    from mythril_amd.engine import prepare
    s = parse_file(os.path.join(ROOT, "tests", "golden", "solver_log", "c2_token_transfer_ok.smt2"))
    p = prepare(s.asserts, s.ctx).program
    code = p.code.reshape(-1, 4)
    inv = {v: k for k, v in isa.OPCODES.items()}
    links = [k for k in range(len(code)) if (int(code[k][0]) >> 8) & 0xFF]
    assert len(links) >= 16
    for k in links:
        assert inv[int(code[k][0]) & 0xFF] == "W_CDINS" and inv[int(code[k + 1][0]) & 0xFF] == "W_CDINS"
        assert int(code[k + 1][1]) >> 16 == isa.decode_dst(int(code[k][1]) & 0xFFFF)[0]
    assert _validate(p) == 0
    q = compile_program([Ctx().app("bvult", Ctx().var("a", 256), Ctx().const(5, 256))])
    q.code = q.code.copy()
    q.code[0] = int(q.code[0]) | (isa.FLAG_CHAIN << 8)    # a flag on a non-W_CDINS instruction
    assert _validate(q) != 0
    p.code = p.code.copy()
    last = links[-1] + 1                                  # the chain's last link: next is not a W_CDINS
    p.code[4 * last] = int(p.code[4 * last]) | (isa.FLAG_CHAIN << 8)
    assert _validate(p) != 0


def test_chain_link_result_read_as_size_is_rejected():
    """a chain link's result stays in registers; a consumer that also
    names that slot as its size operand would read the stale slot."""
    from mythril_amd.smt2 import parse_file
    from mythril_amd.engine import prepare
    s = parse_file(os.path.join(ROOT, "tests", "golden", "solver_log", "c2_token_transfer_ok.smt2"))
    p = prepare(s.asserts, s.ctx).program
    code = p.code.copy().reshape(-1, 4)
    k = next(k for k in range(len(code)) if (int(code[k][0]) >> 8) & 0xFF)
    slot = isa.decode_dst(int(code[k][1]) & 0xFFFF)[0]
    code[k + 1][2] = (int(code[k + 1][2]) & 0xFFFF0000) | slot
    p.code = code.reshape(-1)
    assert _validate(p) != 0


def test_dead_handles_are_rejected_without_a_gpu():
    """the library keeps a registry of live handles, so a
    program freed with (or after) its context, a double free, or a foreign
    pointer is an MG_E_ARG and is never dereferenced (checked here without a
    GPU: no such handle can be live)."""
    from mythril_amd.runtime import bind
    lib = bind(ctypes.CDLL(LIB_PATH))
    bogus = ctypes.c_void_p(0xDEAD0000)
    assert lib.mg_prog_free(bogus) == -1
    assert b"not a live program" in lib.mg_last_error()
    assert lib.mg_free(bogus) == -1
    assert b"not a live context" in lib.mg_last_error()
    assert lib.mg_prog_has_kernel(bogus) == 0
    out = (ctypes.c_uint64 * 1)()
    arr = (ctypes.c_void_p * 1)(0xDEAD1000)
    assert lib.mg_search(bogus, arr, 1, 0, 0, 1, 0, out, None) == -1
    assert lib.mg_free(None) == 0 and lib.mg_prog_free(None) == 0
