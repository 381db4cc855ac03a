"""Assembled kernels: a program as straight-line gfx950 code, in milliseconds.

The asm interpreter (csrc/mw_asm_interp.inc) pays a dispatch and an indexed
operand fetch per bytecode instruction.  An assembled kernel is the same
kernel with the program itself in place of the dispatch loop: every
instruction is its handler instantiated with literal registers and constants
(mythril_amd/asmgen.py static_body).  The template - prologue, chunk loop,
result protocol, leaf subroutines - is compiled once by hipcc at build time
(csrc/mw_asmjit_shell.hip -> lib/asmjit_template.s, package data); here the program's body
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

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
# shipped with the package (setup.py package_data), beside the product library
TEMPLATE = PKG / "lib" / "asmjit_template.s"
# in a source tree: build/asmjit/cache; installed: the user's cache directory
CACHE = Path(os.environ.get("MYTHRIL_AMD_ASMJIT_CACHE") or (
    ROOT / "build" / "asmjit" / "cache" if (ROOT / "setup.py").exists()
    else Path.home() / ".cache" / "mythril_amd" / "asmjit"))
LLVM_BIN = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "llvm" / "bin"
TEMPLATE_NAME = "mwa_TEMPLATE"
TEMPLATE_SIG = str(0x0123456789ABCDEF)   # the shell's placeholder signature, as the .s prints it

_template: Optional[Tuple[str, str, str]] = None   # (text, asm-statement number, hash)
_generator: Optional[str] = None


def generator_hash() -> str:
    """Hash of everything that turns a program into assembly text besides the
    template: the body generator's sources and the assembler's version.  Part
    of the on-disk cache key, so a changed generator never reuses a stale
    code object."""
    global _generator
    if _generator is None:
        h = hashlib.sha256()
        here = Path(__file__).resolve().parent
        for f in ("asmgen.py", "asmjit.py", "isa.py"):
            h.update((here / f).read_bytes())
        try:
            r = subprocess.run([str(LLVM_BIN / "llvm-mc"), "--version"], capture_output=True, text=True)
            h.update(r.stdout.encode())
        except OSError:
            pass
        _generator = h.hexdigest()[:16]
    return _generator


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


def why_unavailable() -> Optional[str]:
    """None when programs can be assembled, else the reason they stay on the
    asm interpreter (missing template or assembler)."""
    try:
        _load_template()
    except Unavailable as e:
        return str(e)
    for tool in ("llvm-mc", "ld.lld"):
        if not (LLVM_BIN / tool).exists():
            return f"{LLVM_BIN / tool} missing (ROCm's LLVM tools)"
    return None


def available() -> bool:
    return why_unavailable() is None


_STORE_OPS = (isa.OPCODES["STORE_W"], isa.OPCODES["STORE_N"])


def eligible(p: Program) -> bool:
    """asm-eligible search programs: trace rows (STORE_*) are written by the
    asm interpreter only (mg_eval_generated), never by an assembled body"""
    return (isa.asm_eligible(p.code, p.leaves, p.consts)
            and not any(int(w) & 0xFF in _STORE_OPS for w in list(p.code)[0::4]))


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
    key = hashlib.sha256((thash + generator_hash() + name).encode() + p.code.tobytes() + p.consts.tobytes()
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
