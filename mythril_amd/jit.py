"""Specialised search kernels: one straight-line gfx950 kernel per program.

The interpreter (``csrc/mw_interp.h``) runs any program, but for every
bytecode instruction it pays a scalar dispatch and indexed register-file
moves (``s_set_gpr_idx``) around a handful of VALU ops.  On the C5 workload
that overhead is about two thirds of the kernel time (performance
log).  For long searches the program is instead emitted as HIP source: one
straight-line function over the compiler's SSA machine IR (``Program.machine_ir()``),
every value a register array, every constant a literal, every leaf
descriptor folded into the generator call.  hipcc compiles it for gfx950 into
a code object, and ``mg_prog_attach_kernel`` binds it to the loaded program;
``mg_search`` / ``mg_eval_generated`` then launch it instead of the
interpreter.  The op helpers (``csrc/mw_jit.h``) have the interpreter's exact
semantics over the same ALU and candidate generator, so verdicts and witness
indices are identical (tests/test_jit.py on the CPU, tests/test_gpu_jit.py on
the device).

The code object carries the program's signature (FNV-1a 64 over its code,
constant, leaf and pool words); the library refuses to attach it to any
other program.  Compiles are cached on disk by source hash (``MW_JIT_CACHE``,
default ``build/jit``).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .compiler import Const, MInsn, Program, VReg, compile_program

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "mythril_amd" / "csrc"
ARCH = os.environ.get("MW_OFFLOAD_ARCH", "gfx950")
HEADERS = ["mw_jit.h", "mw_alu.h", "mw_isa.h", "mw_leaf.h"]
M256 = (1 << 256) - 1
# A straight-line body is cut into basic blocks at every CHECK and at least every
# SPLIT_EVERY instructions (JIT_SPLIT, mw_jit.h).  In one giant block LLVM's
# scheduler interleaves far-apart computations and spills heavily (C5-1k:
# 1121 VGPR spills in one block, 25 with a block per conjunct).
SPLIT_EVERY = 48
# how a region boundary is emitted: "branch" (JIT_SPLIT of mw_jit.h) or
# "sched_barrier" (MW_JIT_SPLIT env: experiments)
SPLIT_KIND = os.environ.get("MW_JIT_SPLIT", "branch")
# experiments (tools/ab_c5.py): a workgroup barrier after every conjunct of the
# exhaustive variant, keeping a block's waves at the same place in the code
CHECK_SYNC = os.environ.get("MW_JIT_CHECK_SYNC", "0") == "1"
CHECK_SYNC_EVERY = int(os.environ.get("MW_JIT_CHECK_SYNC_EVERY", "1"))   # ... after every k-th conjunct
# 256-bit products of two register operands by columns (mw_jit.h mul8_cols:
# v_mad_u64_u32 carry-outs counted per column) instead of mul8's rows; C5
# 17.51 -> 17.40 ms per 2^22 launch (profiles/r6k/ab_c5_mulcols.json)
MUL_COLS = os.environ.get("MW_JIT_MUL_COLS", "1") == "1"
# An LDS leaf's reload is placed up to this many body lines before its use
# (not before the leaf's own store, and not above a division: LDS_AHEAD_STOP),
# so its latency overlaps the instructions in between; 0 reloads right before
# the use.  C5 per 2^22 launch (tools/ab_c5.py, profiles/r6p): right before
# the use 17.41 ms; 8 / 16 / 32 lines 16.91 / 16.88 / 16.85 ms, but hoisted
# into the divisions' register pressure LLVM spills to scratch (+25 / +300 /
# +350 MB of HBM writes per launch) and 64 lines spill so much it is slower
# (20.93 ms).  Stopping at divisions: 8 / 16 / 32 lines 16.98 / 16.95 /
# 16.94 ms with 3 / 2 / 11 VGPRs spilled (the unhoisted kernel: 2); 16 lines
# keeps the unhoisted kernel's 12 scratch bytes per lane, so that is the default
LDS_AHEAD = int(os.environ.get("MW_JIT_LDS_AHEAD", "16"))
# ... or (when > 0) as far back as that much estimated work (insn_weight, in
# machine instructions) of the lines in between
LDS_AHEAD_W = int(os.environ.get("MW_JIT_LDS_AHEAD_W", "0"))
# ... and never above a line at least this heavy (insn_weight: the divisions,
# where LLVM already runs short of registers)
LDS_AHEAD_STOP = int(os.environ.get("MW_JIT_LDS_AHEAD_STOP", "500"))
# A use within this many body lines of the leaf's last reload reads that
# copy instead of reloading (0: every use reloads).  C5 per 2^22 launch
# (profiles/r6ze-r6zg, against 0 on the same box): 4 / 12 / 24 / 48 / 96 / 192
# lines -0.5 / -0.8 / -1.0 / -1.5 / -2.1 / -2.3 %, with the unreused kernel's
# spills up to 96 lines (12 bytes per lane) and 68 bytes at 192: 96
LDS_REUSE = int(os.environ.get("MW_JIT_LDS_REUSE", "96"))
M32 = 0xFFFFFFFF

_WBIN = {"W_ADD": "w_add", "W_SUB": "w_sub", "W_MUL": "w_mul", "W_AND": "w_and", "W_OR": "w_or",
         "W_XOR": "w_xor", "W_SHL": "w_shl", "W_LSHR": "w_lshr", "W_ASHR": "w_ashr"}
_DIV = {"UDIV": 0, "UREM": 1, "SDIV": 2, "SREM": 3, "SMOD": 4}
_NBIN = {"N_ADD": "jit::nn_add({a}, {b}, {w})", "N_SUB": "jit::nn_sub({a}, {b}, {w})",
         "N_MUL": "jit::nn_mul({a}, {b}, {w})", "N_AND": "({a} & {b})", "N_OR": "({a} | {b})",
         "N_XOR": "({a} ^ {b})", "N_SHL": "n_shl({a}, {b}, {w})", "N_LSHR": "n_lshr({a}, {b}, {w})",
         "N_ASHR": "n_ashr({a}, {b}, {w})", "N_ULTN": "(u32)({a} < {b})", "N_ULEN": "(u32)({a} <= {b})",
         "N_SLTN": "(u32)n_slt({a}, {b}, {w})", "N_SLEN": "(u32)n_sle({a}, {b}, {w})",
         "N_EQN": "(u32)({a} == {b})", "N_UMULNON": "(u32)n_umulno({a}, {b}, {w})",
         "N_ADDCN": "jit::nn_addc({a}, {b}, {w})"}


def _cache_dir() -> Path:
    return Path(os.environ.get("MW_JIT_CACHE", str(ROOT / "build" / "jit")))


def signature(p: Program) -> int:
    """FNV-1a 64 over the program's words, as mg_prog_load computes it."""
    h = 0xCBF29CE484222325
    for arr in (p.code, p.consts, p.leaves, p.pool):
        a = np.ascontiguousarray(arr, dtype=np.uint32)
        h = _fnv_words(h, a)
    return h


def _fnv_words(h: int, a: np.ndarray) -> int:
    # FNV-1a over the little-endian bytes of each word; vectorised per byte lane
    b = a.astype("<u4").view(np.uint8)
    P = 0x100000001B3
    M = (1 << 64) - 1
    for x in b.tobytes():
        h = ((h ^ x) * P) & M
    return h


def interleave_conjuncts(insns: List[MInsn], k: int) -> List[MInsn]:
    """Merge each run of k consecutive conjuncts (SSA segments ending at a
    CHECK) into one instruction stream, round-robin, so independent dependency
    chains sit side by side in every basic block.

    A conjunct alone is one serial chain (C5: every node consumes its
    predecessor; a 256-bit add is an 8-deep carry chain).  gfx950 needs wait
    states between a VALU that writes a carry/mask SGPR and the VALU reading
    it, and LLVM pads a serial chain with s_nop; a second, independent chain in
    the same block fills those slots and the VALU latency instead.  The merge
    keeps every operand defined before its use: a segment whose next
    instruction reads a value another segment of the group has not produced
    yet (a leaf first generated there) waits while that segment advances."""
    if k <= 1:
        return list(insns)
    segs: List[List[MInsn]] = []
    cur: List[MInsn] = []
    tail: List[MInsn] = []
    for ins in insns:
        if ins.op == "END":
            tail.append(ins)
            continue
        cur.append(ins)
        if ins.op == "CHECK":
            segs.append(cur)
            cur = []
    if cur:
        segs.append(cur)
    out: List[MInsn] = []
    defined = set()
    for g in range(0, len(segs), k):
        group = segs[g:g + k]
        pos = [0] * len(group)
        left = sum(len(sg) for sg in group)
        while left:
            # round-robin; a head whose operand is still pending waits.  The
            # earliest unfinished segment can always issue (the original order
            # is topological), so every round makes progress.
            for j, sg in enumerate(group):
                if pos[j] >= len(sg):
                    continue
                ins = sg[pos[j]]
                if any(isinstance(s_, VReg) and s_.id not in defined for s_ in ins.srcs):
                    continue
                out.append(ins)
                if ins.dst is not None:
                    defined.add(ins.dst.id)
                pos[j] += 1
                left -= 1
    return out + tail


class _Gen:
    """Emit the body of one program as straight-line HIP."""

    def __init__(self, p: Program, name: str, fence_first: bool = False, lds_leaves: int = 0,
                 insns: Optional[List[MInsn]] = None, interleave: int = 1, mul_cols: Optional[bool] = None):
        self.fence_first = fence_first  # diagnostics (tools/opbench.py): no folding across nodes
        self.mul_cols = MUL_COLS if mul_cols is None else mul_cols
        self.p = p
        self.insns = interleave_conjuncts(p.machine_ir() if insns is None else insns, interleave)
        # the lds_leaves most-used wide leaves live in LDS (mw_jit.h lds_put8/lds_get8)
        uses: Dict[int, int] = {}
        defs: Dict[int, int] = {}
        for ins in self.insns:
            if ins.op == "LEAF_W":
                defs[ins.dst.id] = ins.imm
            for s_ in ins.srcs:
                if isinstance(s_, VReg) and s_.id in defs:
                    uses[s_.id] = uses.get(s_.id, 0) + 1
        hot = sorted(uses, key=lambda v: -uses[v])[:lds_leaves]
        self.lds_slot: Dict[int, int] = {v: k for k, v in enumerate(hot)}
        self.pre: List[str] = []
        self.nl = 0
        self.name = name
        self.wconst: Dict[int, str] = {}
        self.lines: List[str] = []
        self.since_split = 0
        self.nf = 0
        self.put_at: Dict[int, int] = {}     # LDS leaf vreg -> index of its store line
        self.line_w: List[int] = []          # estimated work of each line (_place_reloads)
        self.nchecks = 0
        self.last_reload: Dict[int, Tuple[str, int]] = {}   # LDS leaf -> (its last reload, line)

    def W(self, s) -> str:
        if isinstance(s, Const):
            v = s.value & M256
            n = self.wconst.get(v)
            if n is None:
                n = f"k{len(self.wconst)}"
                self.wconst[v] = n
            return n
        if s.cls != "W":
            raise ValueError("N register in a W operand")
        slot = self.lds_slot.get(s.id)
        if slot is not None:
            last = self.last_reload.get(s.id)
            if LDS_REUSE and last is not None and len(self.lines) - last[1] <= LDS_REUSE:
                return last[0]      # reloaded a few lines ago: that copy again
            self.nl += 1
            self.last_reload[s.id] = (f"L{self.nl}", len(self.lines))
            self.pre.append(("R", f"u32 L{self.nl}[8]; jit::lds_get8({slot}u, L{self.nl});", s.id))
            return f"L{self.nl}"
        return f"v{s.id}"

    def N(self, s) -> str:
        if isinstance(s, Const):
            return f"{s.value & M32:#x}u"
        if s.cls != "N":
            raise ValueError("W register in an N operand")
        return f"n{s.id}"

    def leaf(self, li: int, dst: str):
        L = [int(x) for x in self.p.leaves[li * isa.LEAF_WORDS:(li + 1) * isa.LEAF_WORDS]]
        w, kind, lid, shift, bits, poff, _inrow, stride = L
        return (f"leaf_fields({w}u, {kind}u, {lid:#x}u, {shift}u, {bits}u, {poff}u, {stride}u, "
                f"pool, seed, cand, {dst});")

    def emit(self, ins) -> None:
        n0 = len(self.lines)
        self._emit(ins)
        self.line_w.extend([0] * (len(self.lines) - len(self.line_w)))
        if len(self.lines) > n0:
            self.line_w[-1] = insn_weight(ins)

    def _emit(self, ins) -> None:
        op, w, d, S, imm = ins.op, ins.width, ins.dst, ins.srcs, ins.imm
        self.since_split += 1
        if self.since_split > SPLIT_EVERY and op != "CHECK":
            self.lines.append("JIT_SPLIT();")
            self.since_split = 0
        if op == "END":
            return
        shape = isa.SHAPES[op]
        A = [self.W(s) if c == "W" else self.N(s) for s, c in zip(S, shape[1])]
        out = self.lines.append
        for x in self.pre:
            out(x)
        self.pre = []
        fence = getattr(ins, "remat", False)
        if fence or (self.fence_first and S and op not in ("CHECK", "STORE_W", "STORE_N")):
            for j, (s, c) in enumerate(zip(S, shape[1])):
                if not fence and j > 0:
                    break
                if isinstance(s, VReg):
                    self.nf += 1
                    if c == "W":
                        out(f"u32 f{self.nf}[8]; jit::fence8({A[j]}, f{self.nf});")
                        A[j] = f"f{self.nf}"
                    else:
                        out(f"const u32 f{self.nf} = jit::fence1({A[j]});")
                        A[j] = f"f{self.nf}"
        dn = None
        if d is not None:
            dn = f"v{d.id}" if d.cls == "W" else f"n{d.id}"
        if op == "CHECK":
            self.nchecks += 1
            sync = CHECK_SYNC and self.nchecks % CHECK_SYNC_EVERY == 0
            tail = "{ JIT_SPLIT(); JIT_SYNC(); }" if sync else "JIT_SPLIT();"
            out(f"alive = jit::check(alive, {A[0]}); if (EARLY) {{ if (jit::none(alive)) break; }} else {tail}")
            self.since_split = 0
        elif op == "LEAF_W" and d.id in self.lds_slot:
            out(f"{{ u32 t_[8]; {self.leaf(imm, 't_')} jit::lds_put8({self.lds_slot[d.id]}u, t_); }}")
            self.put_at[d.id] = len(self.lines)
        elif op == "LEAF_W":
            out(f"u32 {dn}[8]; {self.leaf(imm, dn)}")
        elif op == "LEAF_N":
            out(f"u32 {dn}; {{ u32 t_[8]; {self.leaf(imm, 't_')} {dn} = t_[0]; }}")
        elif op in ("STORE_W", "STORE_N"):
            row = self.p.trace_map[-imm - 1][0]
            if op == "STORE_W":
                out(f"jit::tstore(trace, tstride, tidx, {row}u, {A[0]}, 8);")
            else:
                out(f"{{ const u32 t_ = {A[0]}; jit::tstore(trace, tstride, tidx, {row}u, &t_, 1); }}")
        elif op == "MOV_W":
            out(f"u32 {dn}[8]; jit::w_mov({A[0]}, {w}u, {dn});")
        elif op == "MOV_N":
            out(f"const u32 {dn} = {A[0]};")
        elif op == "W_MUL" and self.mul_cols and all(isinstance(s, VReg) for s in S):
            out(f"u32 {dn}[8]; jit::w_mulv({A[0]}, {A[1]}, {w}u, {dn});")
        elif op in _WBIN:
            out(f"u32 {dn}[8]; jit::{_WBIN[op]}({A[0]}, {A[1]}, {w}u, {dn});")
        elif op.startswith("W_") and op[2:] in _DIV:
            out(f"u32 {dn}[8]; jit::w_div({_DIV[op[2:]]}, {A[0]}, {A[1]}, {w}u, {dn}, dsteps);")
        elif op == "W_NOT":
            out(f"u32 {dn}[8]; jit::w_not({A[0]}, {w}u, {dn});")
        elif op == "W_ITE":
            out(f"u32 {dn}[8]; jit::w_ite({A[2]}, {A[0]}, {A[1]}, {w}u, {dn});")
        elif op == "W_SHLI":
            out(f"u32 {dn}[8]; jit::w_shli({A[0]}, {imm}u, {w}u, {dn});")
        elif op == "W_LSHRI":
            out(f"u32 {dn}[8]; jit::w_lshri({A[0]}, {imm}u, {w}u, {dn});")
        elif op == "W_ZEXTN":
            out(f"u32 {dn}[8]; jit::w_zextn({A[0]}, {w}u, {dn});")
        elif op == "W_SEXT":
            out(f"u32 {dn}[8]; jit::w_sext({A[0]}, {imm}u, {w}u, {dn});")
        elif op == "W_SEXTN":
            out(f"u32 {dn}[8]; jit::w_sextn({A[0]}, {imm}u, {w}u, {dn});")
        elif op == "W_INSN":
            out(f"u32 {dn}[8]; jit::w_insn({A[0]}, {A[1]}, {imm}u, {w}u, {dn});")
        elif op == "N_EXTRACTW":
            out(f"const u32 {dn} = jit::n_extractw({A[0]}, {imm}u, {w}u);")
        elif op == "N_ULT":
            out(f"const u32 {dn} = jit::n_ult({A[0]}, {A[1]});")
        elif op == "N_ULE":
            out(f"const u32 {dn} = jit::n_ule({A[0]}, {A[1]});")
        elif op in ("N_SLT", "N_SLE"):
            le = "true" if op == "N_SLE" else "false"
            out(f"const u32 {dn} = jit::n_scmp({A[0]}, {A[1]}, {w}u, {le});")
        elif op == "N_EQ":
            out(f"const u32 {dn} = jit::n_eq({A[0]}, {A[1]});")
        elif op == "N_UMULNO":
            out(f"const u32 {dn} = jit::n_umulno({A[0]}, {A[1]}, {w}u);")
        elif op == "N_ADDC":
            out(f"const u32 {dn} = jit::n_addc({A[0]}, {A[1]}, {w}u);")
        elif op in _NBIN:
            out(f"const u32 {dn} = " + _NBIN[op].format(a=A[0], b=A[1], w=f"{w}u") + ";")
        elif op.startswith("N_") and op[2:] in _DIV:
            out(f"const u32 {dn} = n_div({_DIV[op[2:]]}, {A[0]}, {A[1]}, {w}u);")
        elif op == "N_NOT":
            out(f"const u32 {dn} = jit::nn_not({A[0]}, {w}u);")
        elif op == "N_ITE":
            out(f"const u32 {dn} = {A[2]} ? {A[0]} : {A[1]};")
        elif op == "N_SHLI":
            out(f"const u32 {dn} = jit::nn_shli({A[0]}, {imm}u, {w}u);")
        elif op == "N_LSHRI":
            out(f"const u32 {dn} = jit::nn_lshri({A[0]}, {imm}u, {w}u);")
        elif op == "N_SEXT":
            out(f"const u32 {dn} = jit::nn_sext({A[0]}, {imm}u, {w}u);")
        else:
            raise ValueError(f"jit: no emitter for {op}")

    def _place_reloads(self) -> List[str]:
        """self.lines with every LDS reload ("R", text, leaf) moved LDS_AHEAD
        lines earlier (never above its leaf's store): it goes before the
        first other line at or after that point, in the order met."""
        if LDS_AHEAD <= 0 and LDS_AHEAD_W <= 0:
            return [x[1] if isinstance(x, tuple) else x for x in self.lines]
        before: Dict[int, List[str]] = {}
        rest: List[Tuple[int, str]] = []
        for i, x in enumerate(self.lines):
            if isinstance(x, tuple):
                floor = self.put_at.get(x[2], -1) + 1
                if LDS_AHEAD_W > 0:
                    j, acc = i, 0
                    while j > floor and acc < LDS_AHEAD_W:
                        j -= 1
                        acc += self.line_w[j]
                elif LDS_AHEAD_STOP < (1 << 30):
                    j = i
                    while j > floor and i - j < LDS_AHEAD and self.line_w[j - 1] < LDS_AHEAD_STOP:
                        j -= 1
                else:
                    j = max(i - LDS_AHEAD, floor)
                before.setdefault(j, []).append(x[1])
            else:
                rest.append((i, x))
        out: List[str] = []
        pend = sorted(before)
        k = 0
        for i, x in rest:
            while k < len(pend) and pend[k] <= i:
                out += before[pend[k]]
                k += 1
            out.append(x)
        while k < len(pend):
            out += before[pend[k]]
            k += 1
        return out

    def body(self) -> str:
        for ins in self.insns:
            self.emit(ins)
        self.lines = self._place_reloads()
        head = [f"template <bool EARLY>",
                f"MW_HD bool {self.name}_body(const u32* __restrict__ pool, u64 seed, u64 cand, bool alive,",
                f"                             u32 ctl, u32* __restrict__ trace, u64 tstride, u64 tidx,",
                f"                             DivCount& dsteps) {{"]
        consts = []
        for v, n in self.wconst.items():
            limbs = ", ".join(f"{(v >> (32 * k)) & M32:#x}u" for k in range(8))
            consts.append(f"  const u32 {n}[8] = {{{limbs}}};")
        return "\n".join(head + consts + ["  do {"] + ["    " + x for x in self.lines] +
                         ["  } while (0);", "  return alive;", "}"])


# --------------------------------------------------------------------------- program parts
# Large programs are split at conjunct boundaries into parts of about
# PART_WEIGHT estimated machine instructions, each its own kernel and code
# object (compiled in parallel), launched in order over the same candidates
# with the alive bits passed through a buffer (mw_jit.h MW_JIT_FIRST/LAST).
# LLVM allocates a part like a small program (C5: 3k-node programs compile
# without spills at 2 waves/SIMD, the 10k whole program does not) and each
# part compiles in a fraction of the time.  A part regenerates the leaves it
# uses (and recomputes any other value live across its boundary; boundaries
# are chosen where there is none).
PART_WEIGHT = 110_000
_WEIGHT = {"W_UDIV": 900, "W_UREM": 900, "W_SDIV": 950, "W_SREM": 950, "W_SMOD": 950, "W_MUL": 110,
           "W_SHL": 45, "W_LSHR": 45, "W_ASHR": 45, "LEAF_W": 200, "LEAF_N": 100, "N_ULT": 25, "N_ULE": 25,
           "N_SLT": 30, "N_SLE": 30, "N_EQ": 16, "N_UMULNO": 150, "N_ADDC": 12}


def insn_weight(ins: MInsn) -> int:
    w = _WEIGHT.get(ins.op)
    if w is not None:
        return w
    return 10 if ins.op.startswith("W_") else 3


def split_ssa(p: Program, part_weight: int = PART_WEIGHT) -> List[List[MInsn]]:
    """Instruction lists of the program's parts (one list when it is small)."""
    ssa = [i for i in p.machine_ir() if i.op != "END"]
    n = len(ssa)
    total = sum(insn_weight(i) for i in ssa)
    if total <= part_weight * 1.25 or n < 2:
        return [p.machine_ir()]
    defs: Dict[int, int] = {}
    last: Dict[int, int] = {}
    for i, ins in enumerate(ssa):
        if ins.dst is not None:
            defs[ins.dst.id] = i
        for s_ in ins.srcs:
            if isinstance(s_, VReg):
                last[s_.id] = i
    delta = [0] * (n + 2)  # non-leaf values live across boundary b (before insn b)
    for vid, d in defs.items():
        if ssa[d].op.startswith("LEAF"):
            continue
        l = last.get(vid, d)
        if l > d:
            delta[d + 1] += 1
            delta[l + 1] -= 1
    cuts, acc, cross = [], 0, 0
    target = total / max(2, round(total / part_weight))
    for b in range(1, n):
        cross += delta[b]
        acc += insn_weight(ssa[b - 1])
        if acc >= target and ssa[b - 1].op == "CHECK" and cross == 0:
            cuts.append(b)
            acc = 0
    if not cuts:
        return [p.machine_ir()]
    bounds = [0] + cuts + [n]
    parts = []
    for a, b in zip(bounds, bounds[1:]):
        seg = ssa[a:b]
        inside = {ins.dst.id for ins in seg if ins.dst is not None}
        need, stack = set(), [s_.id for ins in seg for s_ in ins.srcs if isinstance(s_, VReg)]
        while stack:  # defining instructions of values from earlier parts (leaves, in practice)
            v = stack.pop()
            if v in inside or v in need:
                continue
            need.add(v)
            stack.extend(s_.id for s_ in ssa[defs[v]].srcs if isinstance(s_, VReg))
        pre = [ssa[defs[v]] for v in sorted(need, key=lambda v: defs[v])]
        parts.append(pre + seg + [MInsn("END")])
    return parts


def generate(progs: Sequence[Program], names: Sequence[str], variants: str = "xe",
             fence_first: bool = False, lds_leaves: int = 0,
             parts: Optional[Sequence[Tuple[List[MInsn], int, int]]] = None, interleave: int = 1,
             mul_cols: Optional[bool] = None) -> str:
    """HIP source for a module holding one specialised kernel set per program
    (with `parts`: per program, its (instructions, part index, part count))."""
    out = ["// generated by mythril_amd/jit.py: specialised witness-search kernels"]
    if lds_leaves:
        out.append(f"#define MW_JIT_LDS_SLOTS {lds_leaves}")
    out += ['#include "mw_jit.h"', "using namespace mw;", ""]
    if SPLIT_KIND == "sched_barrier":
        # region boundaries as scheduling barriers instead of never-taken branches:
        # no branch (and no long-jump sequence past a cold block at the end of a
        # multi-MiB body), the scheduler still cannot move code across them
        out += ["#if defined(__HIP_DEVICE_COMPILE__)", "#undef JIT_SPLIT",
                "#define JIT_SPLIT() __builtin_amdgcn_sched_barrier(0)", "#endif", ""]
    if CHECK_SYNC:
        out += ["#if defined(__HIP_DEVICE_COMPILE__)", "#define JIT_SYNC() __syncthreads()", "#else",
                "#define JIT_SYNC() ((void)0)", "#endif", ""]
    done = set()
    for k, (p, name) in enumerate(zip(progs, names)):
        if name in done:   # two queries that compile to the same program share one kernel
            continue
        done.add(name)
        if not p.machine_ir():
            raise ValueError("program has no SSA machine IR (compiled by an older compiler?)")
        part = parts[k] if parts else None
        out.append(f"// program {name}: {p.n_insn} bytecode insns, {p.ops_per_eval} u32 ops/eval"
                   + (f", part {part[1]} of {part[2]}" if part else ""))
        out.append(_Gen(p, name, fence_first, lds_leaves, part[0] if part else None, interleave, mul_cols).body())
        out.append(f"MW_JIT_SIG({name}, {signature(p):#x}ull)")
        if part:
            out.append(f"MW_JIT_PART({name}, {part[1]}u, {part[2]}u)")
        if "x" in variants:
            out.append(f"MW_JIT_KERNEL({name}, _x, {name}_body, false)")
        if "e" in variants:
            out.append(f"MW_JIT_KERNEL({name}, _e, {name}_body, true)")
        out.append(f"MW_JIT_HOST_ENTRY({name}, {name}_body)")
        out.append("")
    return "\n".join(out)


def kernel_name(p: Program) -> str:
    return f"mwj_{signature(p):016x}"


def _hipcc() -> str:
    return "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else "hipcc"


def _key(src: str, flags: Sequence[str]) -> str:
    h = hashlib.sha256(src.encode())
    h.update(" ".join(flags).encode())
    for hd in HEADERS:
        h.update((CSRC / hd).read_bytes())
    return h.hexdigest()[:24]


DEVICE_FLAGS = ["--genco", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wno-unused-variable"]
HOST_FLAGS = ["-O1", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-DMW_JIT_HOST",
              "-Wno-unused-variable"]


_USED: set = set()  # cache files this process produced or read (prune_cache keeps them)


def prune_cache(keep: Optional[set] = None) -> int:
    """Delete cache entries not used by this process (the cache ships with every
    GPU run); returns the number removed."""
    keep = _USED if keep is None else keep
    n = 0
    for f in _cache_dir().glob("*"):
        if f not in keep:
            f.unlink()
            n += 1
    return n


def _compile(src: str, flags: Sequence[str], suffix: str, ext: str) -> Tuple[Path, float]:
    cache = _cache_dir()
    cache.mkdir(parents=True, exist_ok=True)
    out = cache / f"{_key(src, flags)}{suffix}"
    _USED.add(out)
    if out.exists():
        return out, 0.0
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / f"k{ext}"
        f.write_text(src)
        tmp = Path(td) / ("out" + suffix)
        proc = subprocess.Popen([_hipcc(), *flags, f"-I{CSRC}", str(f), "-o", str(tmp)],
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        while True:  # large programs take minutes: keep a heartbeat on stderr
            try:
                _, err = proc.communicate(timeout=30)
                break
            except subprocess.TimeoutExpired:
                print(f"[jit] compiling {len(src) // 1024} KiB of HIP for {ARCH}: "
                      f"{time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
        if proc.returncode != 0:
            raise RuntimeError(f"jit compile failed:\n{err[-4000:]}")
        os.replace(tmp, out)
    return out, time.perf_counter() - t0


def is_cached(progs: Sequence[Program], variants: str = "xe", waves: int = 2, lds_leaves: int = 0,
              interleave: int = 1, mul_cols: Optional[bool] = None) -> bool:
    """Whether compile_device(...) with these arguments would be a cache hit."""
    names = [kernel_name(p) for p in progs]
    src = generate(progs, names, variants, lds_leaves=lds_leaves, interleave=interleave, mul_cols=mul_cols)
    return (_cache_dir() / f"{_key(src, _device_flags(waves))}.hsaco").exists()


def compile_device(progs: Sequence[Program], variants: str = "xe", fence_first: bool = False,
                   waves: int = 2, lds_leaves: int = 0, interleave: int = 1,
                   mul_cols: Optional[bool] = None) -> Tuple[bytes, List[str], float]:
    """gfx950 code object for `progs`; returns (image, kernel names, compile seconds; 0 if cached).

    waves: waves per SIMD the kernels are built for (launch bounds): 2 gives
    each lane 256 registers, 1 gives 512 (AGPRs become spill space instead of
    scratch memory) at half the latency hiding."""
    names = [kernel_name(p) for p in progs]
    src = generate(progs, names, variants, fence_first, lds_leaves, interleave=interleave, mul_cols=mul_cols)
    path, dt = _compile(src, _device_flags(waves), ".hsaco", ".hip")
    return path.read_bytes(), names, dt


HOST_OMP_FLAGS = ["-fopenmp", "-Wl,-rpath,/opt/rocm/llvm/lib"]


def _omp_entries(names: Sequence[str]) -> str:
    """<name>_host_omp: the exhaustive verdicts of candidates [begin,
    begin+count) on every host core (OpenMP), for bench.py's CPU baseline."""
    out = []
    for name in dict.fromkeys(names):
        out += [f'extern "C" int {name}_host_omp(const mw::u32* pool, mw::u64 seed, mw::u64 begin, mw::u64 count,',
                "                               mw::u32* verdict) {",
                "#pragma omp parallel for schedule(dynamic, 64)",
                "  for (long long i = 0; i < (long long)count; ++i) {",
                "    mw::DivCount ds;",
                f"    verdict[i] = {name}_body<false>(pool, seed, begin + (mw::u64)i, true, 0u, nullptr, count,",
                "                                    (mw::u64)i, ds) ? 1u : 0u;",
                "  }",
                "  return 0;",
                "}"]
    return "\n".join(out) + "\n"


def is_host_cached(progs: Sequence[Program], openmp: bool = True) -> bool:
    """Whether compile_host(progs, openmp=...) would be a cache hit."""
    names = [kernel_name(p) for p in progs]
    src = generate(progs, names, "") + (_omp_entries(names) if openmp else "")
    return (_cache_dir() / f"{_key(src, HOST_FLAGS + (HOST_OMP_FLAGS if openmp else []))}.so").exists()


def compile_host(progs: Sequence[Program], lds_leaves: int = 0,
                 part_weight: Optional[int] = None, openmp: bool = False) -> Tuple[Path, List[str]]:
    """TEST ONLY: x86 build of the same generated source (verdicts + trace rows).
    With part_weight, every part of every program gets a host entry
    (<name>_p<k>_host; the program's verdict is the AND over its parts).
    openmp: the candidate loop on every host core (bench.py's CPU baseline)."""
    names = [kernel_name(p) for p in progs]
    if openmp:
        src = generate(progs, names, "", lds_leaves=lds_leaves) + _omp_entries(names)
        path, _ = _compile(src, HOST_FLAGS + HOST_OMP_FLAGS, ".so", ".cpp")
        return path, names
    if part_weight is not None:
        allp, alln, spec = [], [], []
        for p, name in zip(progs, names):
            segs = split_ssa(p, part_weight)
            for k, seg in enumerate(segs):
                allp.append(p)
                alln.append(f"{name}_p{k}")
                spec.append((seg, k, len(segs)))
        src = generate(allp, alln, "", lds_leaves=lds_leaves, parts=spec)
        path, _ = _compile(src, HOST_FLAGS, ".so", ".cpp")
        return path, alln
    src = generate(progs, names, "", lds_leaves=lds_leaves)
    path, _ = _compile(src, HOST_FLAGS, ".so", ".cpp")
    return path, names


# extra device flags for experiments (tools/ab_c5.py ablations); empty in the product
# experiments only (tools/leaf_ablate.py, tools/ab_c5.py): extra -D flags, part of the cache key
EXTRA_FLAGS: List[str] = os.environ.get("MYTHRIL_AMD_JIT_FLAGS", "").split()


def _device_flags(waves: int) -> List[str]:
    return DEVICE_FLAGS + ([f"-DMW_JIT_WAVES={waves}"] if waves != 2 else []) + list(EXTRA_FLAGS)


def compile_parts(p: Program, variants: str = "xe", waves: int = 2, lds_leaves: int = 0,
                  part_weight: int = PART_WEIGHT, interleave: int = 1) -> Tuple[List[Tuple[bytes, str]], float]:
    """Code objects of a program's parts (split_ssa), compiled in parallel hipcc
    processes; returns ([(image, kernel name)], wall seconds, 0 if all cached)."""
    from concurrent.futures import ThreadPoolExecutor
    segs = split_ssa(p, part_weight)
    base = kernel_name(p)
    n = len(segs)
    jobs = []
    for k, seg in enumerate(segs):
        name = base if n == 1 else f"{base}_p{k}"
        spec = None if n == 1 else [(seg, k, n)]
        jobs.append((name, generate([p], [name], variants, lds_leaves=lds_leaves, parts=spec,
                                    interleave=interleave)))
    t0 = time.perf_counter()
    workers = max(1, min(n, int(os.environ.get("MW_JIT_JOBS", "8"))))
    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(lambda j: _compile(j[1], _device_flags(waves), ".hsaco", ".hip"), jobs))
    dt = time.perf_counter() - t0 if any(d for _, d in res) else 0.0
    return [(path.read_bytes(), name) for (path, _), (name, _) in zip(res, jobs)], dt


def attach(dev, dps, variants: str = "xe", waves: int = 2, lds_leaves: int = 0,
           split: bool = False, part_weight: int = PART_WEIGHT, interleave: int = 1) -> float:
    """Compile and attach specialised kernels to loaded programs (DevicePrograms); returns
    the compile seconds (0 when every code object came from the cache).  split: large
    programs become several part kernels (compile_parts) instead of one."""
    dps = list(dps)
    if split:
        total = 0.0
        for dp in dps:
            objs, dt = compile_parts(dp.prog, variants, waves, lds_leaves, part_weight, interleave)
            for image, name in objs:
                dev.attach_kernel(dp, image, name)
            dp.kernel = objs[0][1].rsplit("_p", 1)[0] + (f" ({len(objs)} parts)" if len(objs) > 1 else "")
            total += dt
        return total
    image, names, dt = compile_device([dp.prog for dp in dps], variants, waves=waves, lds_leaves=lds_leaves,
                                      interleave=interleave)
    for dp, name in zip(dps, names):
        dev.attach_kernel(dp, image, name)
    return dt


def bench_programs(n_nodes: int = 10000) -> Dict[int, Program]:
    """bench.py's C5 program (density 2^-24) and its mixed-verdict variant
    (density 2^-1 without the leftover comparisons, about half satisfied, for
    tests/test_gpu_fullsize.py), keyed by density.

    The C5 witness is planted with the host build of the interpreter
    (mythril_amd/hostemu.py), which gives bit for bit the values bench.py gets
    from the device interpreter, so the generated source — and the cache key —
    are the ones the benchmark computes on the GPU box."""
    from . import hostemu
    from .synth import build_c5
    out = {}
    for dens in (24, 1):
        syn = build_c5(hostemu.term_values, n_nodes=n_nodes, density_log2=dens, keep_pending=dens == 24)
        out[dens] = compile_program(syn.conjuncts)
    return out


# leaves of the C5 benchmark kernel kept in LDS at 2 waves per SIMD (8 KiB per
# slot and block). One A/B run (profiles/r3z/ab_c5.json): 10 slots 17.55 ms,
# 8 17.39 ms, 6 18.12 ms, 12 32.5 ms (one block per CU).  8 is 1 % faster but
# spills 100 bytes per lane instead of 12: 401 MB of scratch traffic per
# launch against 32 MB (profiles/r3za) - 10 stays.
BENCH_LDS_LEAVES = 10


def bench_warm_jobs(n_nodes: int = 10000, waves: int = 2, lds_leaves: int = BENCH_LDS_LEAVES, log=print):
    """Independent compile jobs (callables) that put bench.py's C5 kernels in the
    in-tree cache: the single kernel of each density, and the benchmark
    program's split parts (bench.py falls back to them when the single
    kernel's code object is missing)."""
    progs = bench_programs(n_nodes)

    def single(dens):
        _, names, dt = compile_device([progs[dens]], "x", waves=waves, lds_leaves=lds_leaves)
        log(f"[jit] C5 (density 2^-{dens}) kernel {names[0]}: {'compiled in %.0f s' % dt if dt else 'cached'}")

    def parts():
        objs, dt = compile_parts(progs[24], "x", waves=waves, lds_leaves=lds_leaves)
        log(f"[jit] C5 split kernels ({len(objs)} parts): {'compiled in %.0f s' % dt if dt else 'cached'}")

    def host():   # bench.py's CPU baseline (mythril_amd/host_baseline.py)
        cached = is_host_cached([progs[24]], openmp=True)
        t0 = time.perf_counter()
        compile_host([progs[24]], openmp=True)
        log(f"[jit] C5 x86 OpenMP build (CPU baseline): "
            f"{'cached' if cached else 'compiled in %.0f s' % (time.perf_counter() - t0)}")
    return [lambda: single(24), lambda: single(1), parts, host]


def warm_bench_cache(n_nodes: int = 10000, log=print, waves: int = 2, lds_leaves: int = BENCH_LDS_LEAVES) -> float:
    """Pre-compile bench.py's C5 kernels into the in-tree cache, one job after
    the other (tools/jit_warm.py runs the same jobs in parallel)."""
    t0 = time.perf_counter()
    for job in bench_warm_jobs(n_nodes, waves, lds_leaves, log):
        job()
    return time.perf_counter() - t0
