"""Assembled kernels: a program as straight-line gfx950 code, in milliseconds.

The asm interpreter (csrc/mw_asm_interp.inc) pays a dispatch and an indexed
operand fetch per bytecode instruction.  An assembled kernel is the same
kernel with the program itself in place of the dispatch loop: every
instruction is its handler instantiated with literal registers and constants
(mythril_amd/asmgen.py static_body).  The template - prologue, chunk loop,
result protocol, leaf subroutines - is compiled once by hipcc at build time
(csrc/mw_asmjit_shell.hip -> build/asmjit/template.s); here the program's body
replaces its marker line and llvm-mc + ld.lld turn the text into a code
object, about 1 ms per hundred instructions, where hipcc's specialised
kernels (mythril_amd/jit.py) take seconds to minutes.  Results are the
interpreter's: same handlers, same records, same candidate generator
(tests/test_gpu_asmjit.py).

    image, name, seconds = assemble(program)
    attach(dev, dp)            # dev.attach_asm(dp, image, name)
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import tempfile
import time
from pathlib import Path
from typing import Optional, Tuple

from . import asmgen, isa
from .compiler import Program
from .jit import signature

ROOT = Path(__file__).resolve().parent.parent
TEMPLATE = ROOT / "build" / "asmjit" / "template.s"
CACHE = ROOT / "build" / "asmjit" / "cache"
LLVM_BIN = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "llvm" / "bin"
TEMPLATE_NAME = "mwa_TEMPLATE"
TEMPLATE_SIG = str(0x0123456789ABCDEF)   # the shell's placeholder signature, as the .s prints it

_template: Optional[Tuple[str, str, str]] = None   # (text, asm-statement number, hash)


class Unavailable(RuntimeError):
    """No template or no assembler: programs stay on the asm interpreter."""


def _load_template() -> Tuple[str, str, str]:
    global _template
    if _template is None:
        if not TEMPLATE.exists():
            raise Unavailable(f"{TEMPLATE} missing: run python -m mythril_amd.build")
        text = TEMPLATE.read_text()
        if asmgen.MARKER not in text:
            raise Unavailable("template has no body marker")
        m = re.search(r"^Lstop_(\d+):", text, re.M)   # hipcc's number for the asm statement's %=
        if not m or TEMPLATE_SIG not in text:
            raise Unavailable("template lacks its labels or signature placeholder")
        _template = (text, m.group(1), hashlib.sha256(text.encode()).hexdigest()[:16])
    return _template


def available() -> bool:
    try:
        _load_template()
    except Unavailable:
        return False
    return (LLVM_BIN / "llvm-mc").exists() and (LLVM_BIN / "ld.lld").exists()


def eligible(p: Program) -> bool:
    return isa.asm_eligible(p.code, p.leaves)


def kernel_name(p: Program) -> str:
    return f"mwa_{signature(p):016x}"


def source(p: Program) -> Tuple[str, str]:
    """(kernel name, assembly text) of the program's assembled kernel."""
    text, num, _ = _load_template()
    name = kernel_name(p)
    body = "\n".join("\t" + ln if not ln.endswith(":") else ln
                     for ln in asmgen.static_body(p.code, p.consts, p.leaves,
                                                  nlds=asmgen.lds_spill_words(p.n_spill, len(p.pool)),
                                                  pool=p.pool)).replace("%=", num)
    out = text.replace(asmgen.MARKER, body, 1).replace(TEMPLATE_NAME, name)
    return name, out.replace(TEMPLATE_SIG, str(signature(p)), 1)


def assemble(p: Program, cache: bool = True) -> Tuple[bytes, str, float]:
    """(code object, kernel name, seconds spent assembling; 0 when cached)."""
    if not eligible(p):
        raise Unavailable("program has opcodes or leaf kinds the asm engines lack")
    _, _, thash = _load_template()
    name = kernel_name(p)
    key = hashlib.sha256((thash + name).encode() + p.code.tobytes() + p.consts.tobytes()
                         + p.leaves.tobytes() + p.pool.tobytes()).hexdigest()[:24]
    path = CACHE / f"{key}.hsaco"
    if cache and path.exists():
        return path.read_bytes(), name, 0.0
    t0 = time.perf_counter()
    name, src = source(p)
    with tempfile.TemporaryDirectory(prefix="mwa_") as tmp:
        s_path, o_path, co_path = (os.path.join(tmp, f) for f in ("k.s", "k.o", "k.hsaco"))
        with open(s_path, "w") as f:
            f.write(src)
        for cmd in ([str(LLVM_BIN / "llvm-mc"), "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-filetype=obj",
                     s_path, "-o", o_path],
                    [str(LLVM_BIN / "ld.lld"), "-shared", o_path, "-o", co_path]):
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"{os.path.basename(cmd[0])} failed for {name}: {r.stderr[:2000]}")
        image = open(co_path, "rb").read()
    dt = time.perf_counter() - t0
    if cache:
        CACHE.mkdir(parents=True, exist_ok=True)
        tmp_path = path.with_suffix(f".tmp{os.getpid()}")
        tmp_path.write_bytes(image)
        os.replace(tmp_path, path)
    return image, name, dt


def attach(dev, dp, cache: bool = True) -> float:
    """Assemble dp's program and attach the kernel; returns the assembly seconds."""
    image, name, dt = assemble(dp.prog, cache=cache)
    dev.attach_asm(dp, image, name)
    return dt
