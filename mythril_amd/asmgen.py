"""gfx950 assembly generator for the witness engine's two asm engines:

* the threaded-dispatch interpreter core (``render_interp`` ->
  csrc/mw_asm_interp.inc, written by tools/gen_asm_interp.py): one inline-asm
  block that runs any eligible program.  Every handler ends in its own copy
  of the dispatch, which takes the next instruction (prefetched one ahead
  with s_load_dwordx4) and jumps with s_setpc_b64 to the handler offset
  predecoded into its word 0.  The register files live in fixed VGPRs and are
  indexed with s_set_gpr_idx_on; operands come predecoded (mw_validate.cpp
  mw_asm_predecode), narrow constants as registers of their own (NK0);
* assembled kernels (``render_template`` + ``static_body``, used by
  mythril_amd/asmjit.py): the same prologue, chunk loop, result protocol and
  leaf subroutines, with the program itself emitted as straight-line code -
  every handler instantiated with its operands as literal registers and
  constants, no dispatch and no operand indexing - and assembled by llvm-mc
  in milliseconds (hipcc's specialised kernels take seconds to minutes).

Semantics are the interpreter's, opcode by opcode (mw_interp.h).  Programs
qualify when every opcode and leaf kind is listed in ASM_OPCODES /
ASM_LEAF_KINDS (mythril_amd/isa.py, checked by tests/test_asm_interp.py);
the GPU tests compare both engines' verdicts with the compiled interpreter's
and the oracle's.

Registers (per lane; all clobbered by the block):
  v0..v63     W file: slot s, limb k at v[8s + k]
  v64..v127   N file: slot s at v[64 + s]
  v128..v135  zeros (shift padding below XA)   v136..v143 XA (operand a)
  v144..v151  zeros (padding above XA)         v152..v159 XB (operand b)
  v160/v161 candidate index lo/hi  v162 alive (0/1)  v163 LDS lane byte offset
  v164 global-spill lane byte offset  v165 thread id  v168..v175 XR (result)
  v176..v183 XC (third operand / Philox output)  v184..v191 temporaries
  v240..v255  the program's narrow constants (interpreter)
  s16..s98    chunk loop and interpreter state (see the constants below)
"""
import os
import re
import sys

from mythril_amd import isa

# opcodes / leaf kinds with an asm handler (the list lives in mythril_amd/isa.py)
ASM_OPCODES = isa.ASM_OPCODES
ASM_LEAF_KINDS = isa.ASM_LEAF_KINDS

# ---------------------------------------------------------------- registers
# Two register layouts (round 5).  "wide": the files above, 256 VGPRs, two
# waves per SIMD.  "narrow" (the asm interpreter's second kernel,
# mw_search_asm_kernel_n): the same structure with a 24-slot N file and the
# narrow constants right after the temporaries - 168 VGPRs, three waves per
# SIMD - for programs whose N slots all lie below NFILE (95 % of the LASER
# corpus).  A dispatch is a chain of dependent instructions (profiles/r4m):
# a third wave per SIMD hides more of it.  variant("narrow") builds this
# module again with that layout (render_interp emits both bodies).
# "quarter" (mw_search_asm_kernel_q): 5 W slots, 16 N slots and 4 narrow
# constants (no corpus program has more than 3), 124 VGPRs in
# the asm block, four waves per SIMD, for programs whose registers all lie
# in those files (about half of the LASER corpus as compiled).
_LAYOUT_NAME = globals().get("_LAYOUT_OVERRIDE", "wide")
WFILE = 5 if _LAYOUT_NAME == "quarter" else 8     # W slots the layout holds
W0, N0 = 0, 8 * WFILE
NFILE = {"wide": 64, "narrow": 24, "quarter": 16}[_LAYOUT_NAME]   # N slots the layout holds
_OPB = N0 + NFILE                                # first register after the files: the shift padding
XA, XB, XR, XC, T = _OPB + 8, _OPB + 24, _OPB + 40, _OPB + 48, _OPB + 56
CLO, CHI, ALIVE, LDSOFF, GOFF = _OPB + 32, _OPB + 33, _OPB + 34, _OPB + 35, _OPB + 36
# scalar state
# The interpreter keeps two instructions in SGPRs, in two banks: instruction
# i of the predecoded stream always lives in bank i & 1 (s40..s43 for even i,
# s44..s47 for odd).  While the handler of i runs, i + 1 is already in (or on
# its way to) the other bank; dispatching to it loads i + 2 into the bank i
# vacates and jumps through the other bank's word 0 - the handler's absolute
# address, low word (mw_asm_predecode) - with no register moves.  Every
# handler is generated once per bank (Gen.CUR names the bank it reads).
# DISPATCH "single" (MYTHRIL_AMD_ASM_DISPATCH at generation time) keeps one
# current bank and copies the prefetched words into it instead: the handlers
# are emitted once and both banks' entries of the offset table name them.
CUR = 40          # s40..s43 bank A: the current instruction of even index (or of every index, "single")
NXT = 44          # s44..s47 bank B: the odd instructions (the prefetched one, "single")
DISPATCH = os.environ.get("MYTHRIL_AMD_ASM_DISPATCH", "pingpong")
SOFF = 48         # byte offset of the instruction last loaded, from CODE0
TABLO = 49        # address of the handlers' base (Lpc0), low / high word
TABHI = 58
SIDX = 19         # register-file index of an operand / write-back
# assembled kernels (template mode): addresses the straight-line body leaves
# through (it can outgrow a branch's reach); the interpreter's CUR/NXT words
# are unused there (only CUR + 3, the immediate, is)
LEAFADDR = 44     # s[44:45] Lleaf
PHILOXADDR = 48   # s[48:49] Lphilox
STOPADDR = 46     # s[46:47] Lstop
ENDADDR = 40      # s[40:41] Lh_END
CPOOL = 50        # s[50:51] constant pool
LEAVES = 52       # s[52:53] leaf table
POOLB = 54        # pool LDS byte base
FLAGS = 55
SEED = 56         # s[56:57]
NLDS = 59         # spill words in LDS
GSP = 60          # s[60:61] global spill base
GSTRIDE = 62      # bytes between consecutive global spill words (nthreads x 4)
PM0, PM1 = 63, 64  # Philox multipliers
PK0, PK1 = 65, 66  # Philox keys
S67 = 67
LRET = 68         # s[68:69] leaf return address
PRET = 70         # s[70:71] Philox / canon return address
S = list(range(72, 80))   # scratch s72..s79
DESC = 80         # s[80:87] leaf descriptor / wide constant
MSK = 88          # s[88:89] saved lane mask
MSK2 = 90         # s[90:91]
JMP = 92          # s[92:93] the dispatch target: s92 the handler's low word, s93 the code's high word
SX = 94           # s[94:95] scratch pair
AM = 100          # s[100:101] the chunk's live lanes (valid, every check so far held)
POLL = 99         # chunks this wave has started (stop-after-hit polls every POLL_EVERY-th)
POLL_EVERY = 16

# chunk loop state (s16..s39)
CH, NCH, GDX = 16, 17, 18
BEGIN = 20        # s[20:21]
END = 22          # s[22:23]
BASE = 24         # s[24:25]
OUTMIN = 26       # s[26:27] this program's witness slot
VERD = 28         # s[28:29] verdict array or 0
EVALS = 30        # s[30:31]
CODE0 = 32        # s[32:33]
EXECSV = 34       # s[34:35]
VALID = 36        # s[36:37] valid lanes of the chunk
ARGP = 36         # s[36:37] AsmArgs (prologue only; then VALID)
PROGP = 38        # s[38:39] ProgDev (prologue only)
HIT = 38          # after the prologue: this wave has reported a witness (chunks only grow)
TID, LO_SREG = _OPB + 37, 0
TRACE = 96        # s[96:97] trace rows (AsmArgs.trace; 0 in searches: STORE is then a no-op)
NCAND = 98        # candidates per trace row (AsmArgs.ncand)
# the pool digit of the last pooled leaf drawn in this chunk (Lleaf) and its
# digit group (the asm leaf table's word 6, mw_kernels.hip asm_leaf_table;
# reset to -1 at every chunk)
DIGV = _OPB + 38
DIGKEY = 39

NTAB = 128
CHAIN_BIT = 31     # predecoded word 3 (the immediate): W_CDINS's FLAG_CHAIN (mw_asm_predecode)
# narrow constants: v240..v255, filled once per block from the table after the
# predecoded code; a constant N operand is predecoded as index NK0 - N0 + k
# (mw_isa.h MW_ASM_NK / MW_ASM_NK_INDEX)
NK0 = 240 if _LAYOUT_NAME == "wide" else T + 8
NK_INDEX = NK0 - N0
# the narrow layout holds two constants fewer: the kernel's own two inputs
# (thread id, spill offset) need VGPRs outside the asm block's 168
NKN = {"wide": isa.ASM_NK, "narrow": isa.ASM_NK - 2, "quarter": 4}[_LAYOUT_NAME]
NVGPR = NK0 + NKN                                # registers the interpreter's asm block uses
assert (NK_INDEX, NVGPR) == {"wide": (176, 256), "narrow": (88, 166), "quarter": (80, 124)}[_LAYOUT_NAME]
INTROSPECT_FLAG = 7   # AsmArgs.flags bit: report the handler offsets and exit


def v(i):
    return f"v{i}"


def s(i):
    return f"s{i}"


def vr(a, n):
    return f"v[{a}:{a + n - 1}]"


def sr(a, n):
    return f"s[{a}:{a + n - 1}]"


class Gen:
    inline_leaf = True   # W_CDINS inlines the Lleaf code (leaf_inline) instead of calling it
    chains = True        # CHECK_IMPEQ runs chain (the interpreter; an assembled body has no dispatch)

    def __init__(self):
        self.lines = []
        self.tail = []      # out-of-line blocks (constant operands), emitted after the handler
        self.n = 0
        self.bound = {}     # name -> operand field (field())
        self.CUR = CUR      # the bank holding the current instruction (s40 or s44; consume() flips it)

    def L(self, base):
        self.n += 1
        return f"L{base}{self.n}_%="

    def __call__(self, *xs):
        self.lines.extend(xs)

    def label(self, lab):
        self.lines.append(f"{lab}:")

    def flush_tail(self):
        self.lines.extend(self.tail)
        self.tail = []

    # ------------------------------------------------------------ operands
    # Operands come from the asm engine's predecoded copy of the program
    # (mw_validate.cpp mw_asm_predecode): a register operand field holds the
    # N slot (0..63), the W slot x 8 or a narrow constant's VGPR (NK0), so it
    # is the VGPR index relative to the file's base as it stands; bit 15 flags
    # a W constant (word offset).  Word 1 is a [15:0] | dst [31:16], word 2
    # b [15:0] | c [31:16].  s_set_gpr_idx_on reads only bits [7:0] of its
    # SGPR (tools/exp/gpridx_probe.hip), so a and b index straight from their
    # word; c and dst take one shift.
    # field() only binds an operand to a name; fetch_n / fetch_w read it.
    c_in_imm = False   # the current opcode's c operand is in word 3 (C_IN_IMM, mw_asm_predecode)

    def word(self, which):
        """(SGPR, half) holding operand field `which` of the current instruction"""
        if which == "c" and self.c_in_imm:
            return self.CUR + 3, "lo"
        return {"a": (self.CUR + 1, "lo"), "b": (self.CUR + 2, "lo"), "c": (self.CUR + 2, "hi")}[which]

    def field(self, which, dst):
        """bind operand field a/b/c to the name dst (no code)"""
        self.bound[dst] = which

    def _index(self, which):
        """the SGPR to hand s_set_gpr_idx_on for operand field `which`"""
        wd, half = self.word(which)
        if half == "hi":
            self(f"s_lshr_b32 {s(SIDX)}, {s(wd)}, 16")
            return s(SIDX)
        return s(wd)

    def _is_const(self, which, label):
        wd, half = self.word(which)
        self(f"s_bitcmp1_b32 {s(wd)}, {31 if half == 'hi' else 15}", f"s_cbranch_scc1 {label}")

    def fetch_n(self, f, dst):
        """N operand bound to f -> VGPR dst: one indexed move, registers and
        constants alike (a constant is predecoded as its VGPR above the N
        file, NK0)"""
        idx = self._index(self.bound[f])
        self(f"s_set_gpr_idx_on {idx}, gpr_idx(SRC0)", f"v_mov_b32_e32 {v(dst)}, {v(N0)}", "s_set_gpr_idx_off")

    def op_n(self, f, fmt, scratch, mode="SRC0"):
        """emit fmt with {a} = the N operand bound to f, read in place through
        the index register (gpr_idx(mode): fmt's instruction reads {a} as that
        source and no other file register); scratch: the VGPR an assembled
        body may stage it in"""
        idx = self._index(self.bound[f])
        self(f"s_set_gpr_idx_on {idx}, gpr_idx({mode})", fmt.format(a=v(N0)), "s_set_gpr_idx_off")

    def fetch_w(self, f, dst):
        """W/K operand bound to f -> VGPRs dst..dst+7"""
        which = self.bound[f]
        lk, lr = self.L("kw"), self.L("rw")
        self._is_const(which, lk)
        idx = self._index(which)
        self(f"s_set_gpr_idx_on {idx}, gpr_idx(SRC0)")
        for k in range(8):
            self(f"v_mov_b32_e32 {v(dst + k)}, {v(W0 + k)}")
        self("s_set_gpr_idx_off")
        self.label(lr)
        wd, half = self.word(which)
        off = f"s_bfe_u32 {s(SX)}, {s(wd)}, {(15 << 16) | (16 if half == 'hi' else 0):#x}"   # the word offset
        t = [f"{lk}:", off, f"s_lshl_b32 {s(SX)}, {s(SX)}, 2",
             f"s_load_dwordx8 {sr(DESC, 8)}, {sr(CPOOL, 2)}, {s(SX)}", "s_waitcnt lgkmcnt(0)"]
        t += [f"v_mov_b32_e32 {v(dst + k)}, {s(DESC + k)}" for k in range(8)]
        self.tail += t + [f"s_branch {lr}"]

    def w_indexed(self, f, mode, emit, scratch=XA):
        """emit(base): an operation reading the W operand bound to f as VGPRs
        base..base+7 - a register straight from the W file through the index
        (gpr_idx(mode): the emitted instructions read it as that operand, and
        no move copies it out first), a constant from `scratch` after its
        load (out of line)"""
        which = self.bound[f]
        lk, lr = self.L("kx"), self.L("rx")
        self._is_const(which, lk)
        self(f"s_set_gpr_idx_on {self._index(which)}, gpr_idx({mode})")
        emit(W0)
        self("s_set_gpr_idx_off")
        self.label(lr)
        wd, half = self.word(which)
        main, self.lines = self.lines, [f"{lk}:", f"s_bfe_u32 {s(SX)}, {s(wd)}, {(15 << 16) | (16 if half == 'hi' else 0):#x}",
                                        f"s_lshl_b32 {s(SX)}, {s(SX)}, 2",
                                        f"s_load_dwordx8 {sr(DESC, 8)}, {sr(CPOOL, 2)}, {s(SX)}", "s_waitcnt lgkmcnt(0)"]
        self(*[f"v_mov_b32_e32 {v(scratch + k)}, {s(DESC + k)}" for k in range(8)])
        emit(scratch)
        self(f"s_branch {lr}")
        self.tail += self.lines
        self.lines = main

    def width(self, dst):
        # predecoded word 1 [31:24]: the width - 1
        self(f"s_lshr_b32 {s(dst)}, {s(self.CUR + 1)}, 24", f"s_add_u32 {s(dst)}, {s(dst)}, 1")

    def nmask(self, w, dst):
        """dst = w >= 32 ? ~0 : (1 << w) - 1 (w in SGPR, <= 32): the low word of
        the 64-bit field mask (dst must start an aligned SGPR pair)"""
        assert dst % 2 == 0
        self(f"s_bfm_b64 {sr(dst, 2)}, {s(w)}, 0")

    def insn_mask(self, dst):
        """the SGPR holding this instruction's result mask: word 3, where
        mw_asm_predecode puts it for N_ADD / N_SUB / N_MUL / N_NOT (no code)"""
        return s(self.CUR + 3)

    def write_n(self, src):
        """N result in VGPR src -> the N slot in the predecoded dst field (word 1 [31:16])"""
        self(f"s_lshr_b32 {s(SIDX)}, {s(self.CUR + 1)}, 16", f"s_set_gpr_idx_on {s(SIDX)}, gpr_idx(DST)",
             f"v_mov_b32_e32 {v(N0)}, {v(src)}", "s_set_gpr_idx_off")

    def write_w(self, src):
        """W result in VGPRs src.. -> the W slot x 8 in the predecoded dst field (word 1 [31:16])"""
        self(f"s_lshr_b32 {s(SIDX)}, {s(self.CUR + 1)}, 16", f"s_set_gpr_idx_on {s(SIDX)}, gpr_idx(DST)")
        for k in range(8):
            self(f"v_mov_b32_e32 {v(W0 + k)}, {v(src + k)}")
        self("s_set_gpr_idx_off")

    def canon(self, base, w):
        """clear the bits >= w (SGPR) of the 8 limbs at VGPR base (no-op for w >= 256)"""
        done = self.L("cd")
        q, r = S[4], S[5]
        self(f"s_cmp_ge_u32 {s(w)}, 256", f"s_cbranch_scc1 {done}",
             f"s_lshr_b32 {s(q)}, {s(w)}, 5", f"s_and_b32 {s(r)}, {s(w)}, 31")
        for k in range(1, 8):
            sk = self.L("cz")
            # zero limb k when k > q, i.e. q < k
            self(f"s_cmp_lt_u32 {s(q)}, {k}", f"s_cbranch_scc0 {sk}", f"v_mov_b32_e32 {v(base + k)}, 0")
            self.label(sk)
        # partial limb q: keep its low r bits (r == 0: the limb is above w, zero it)
        self(f"s_bfm_b32 {s(r)}, {s(r)}, 0", f"s_set_gpr_idx_on {s(q)}, gpr_idx(SRC1,DST)",
             f"v_and_b32_e32 {v(base)}, {s(r)}, {v(base)}", "s_set_gpr_idx_off")
        self.label(done)

    def nop_vcc(self):
        """a VALU reading the vcc the previous VALU wrote needs no wait states
        (carry chains measured exact without them)"""

    def all_dead_exit(self):
        """SCC = AM != 0 (just ANDed): no live lane -> the dead stub of this
        bank (the chunk ends, or with early exit off, the next instruction)"""
        self(f"s_cbranch_scc0 Ldead{'AB'[self.CUR == NXT and DISPATCH != 'single']}_%=")

    def bit_at(self, base, w, dst):
        """v(dst) = bit w (SGPR) of the limbs at VGPR base (limb w >> 5 read
        through the index register)"""
        q, r = S[3], S[4]
        self(f"s_lshr_b32 {s(q)}, {s(w)}, 5", f"s_and_b32 {s(r)}, {s(w)}, 31",
             f"s_set_gpr_idx_on {s(q)}, gpr_idx(SRC1)", f"v_lshrrev_b32_e64 {v(dst)}, {s(r)}, {v(base)}",
             "s_set_gpr_idx_off", f"v_and_b32_e32 {v(dst)}, 1, {v(dst)}")

    def static_imm(self):
        """the instruction's immediate word when known at generation time"""
        return None

    def flip_sign_bits(self, w, t):
        """flip bit w-1 (w: SGPR holding the width) of XA and XB; t: scratch SGPR"""
        self(f"s_sub_u32 {s(w)}, {s(w)}, 1", f"s_lshr_b32 {s(t)}, {s(w)}, 5",
             f"s_and_b32 {s(w)}, {s(w)}, 31", f"s_lshl_b32 {s(w)}, 1, {s(w)}",
             f"s_set_gpr_idx_on {s(t)}, gpr_idx(SRC1,DST)", f"v_xor_b32_e32 {v(XA)}, {s(w)}, {v(XA)}",
             "s_set_gpr_idx_off", f"s_set_gpr_idx_on {s(t)}, gpr_idx(SRC1,DST)",
             f"v_xor_b32_e32 {v(XB)}, {s(w)}, {v(XB)}", "s_set_gpr_idx_off")

    def extract_limb(self, q, r):
        """XR = bits imm..imm+31 of XA (imm: the instruction's immediate word;
        limb 8 reads v144, zeroed once per block); q, r: scratch SGPRs"""
        self(f"s_lshr_b32 {s(q)}, {s(self.CUR + 3)}, 5", f"s_and_b32 {s(r)}, {s(self.CUR + 3)}, 31",
             f"s_set_gpr_idx_on {s(q)}, gpr_idx(SRC0,SRC1)",
             f"v_alignbit_b32 {v(XR)}, {v(XA + 1)}, {v(XA)}, {s(r)}", "s_set_gpr_idx_off")

    def sub_chain(self, a, b, dst=None, borrow_only=False):
        """a - b over 8 limbs (VGPR bases); borrow out in vcc"""
        for k in range(8):
            d = v(T) if dst is None else v(dst + k)
            if k == 0:
                self(f"v_sub_co_u32_e32 {d}, vcc, {v(a)}, {v(b)}")
            else:
                self.nop_vcc()
                self(f"v_subb_co_u32_e32 {d}, vcc, {v(a + k)}, {v(b + k)}, vcc")

    def add_chain(self, a, b, dst):
        for k in range(8):
            if k == 0:
                self(f"v_add_co_u32_e32 {v(dst)}, vcc, {v(a)}, {v(b)}")
            else:
                self.nop_vcc()
                self(f"v_addc_co_u32_e32 {v(dst + k)}, vcc, {v(a + k)}, {v(b + k)}, vcc")

    def bool_from_vcc(self, dst, invert=False):
        self.nop_vcc()
        self(f"v_cndmask_b32_e64 {v(dst)}, {1 if invert else 0}, {0 if invert else 1}, vcc")

    def long_addr(self, reg, label):
        """s[reg:reg+1] = the address of label (any distance)"""
        here = self.L("pc")
        self(f"s_getpc_b64 {sr(reg, 2)}")
        self.label(here)
        self(f"s_add_u32 {s(reg)}, {s(reg)}, ({label} - {here})", f"s_addc_u32 {s(reg + 1)}, {s(reg + 1)}, 0")

    def stop_if_scc1(self):
        """end this chunk's evaluation (every lane dead) when SCC is set"""
        self("s_cbranch_scc1 Lstop_%=")

    def call_leaf_sub(self):
        self(f"s_call_b64 {sr(LRET, 2)}, Lleaf_%=")

    def other(self):
        """the bank that is not CUR"""
        return CUR + NXT - self.CUR

    _WRITE_MOV = re.compile(r"v_mov_b32_e32 v(\d+), v(\d+)")

    def fuse_write(self):
        """Before a dispatch: `v_op vR, ...` then write_n's `s_lshr; on(DST);
        v_mov vN0, vR; off` becomes `s_lshr; on(DST); v_op vN0, ...; off` -
        the producer writes the N slot through the index register itself (vR
        is dead once the handler ends; the op's sources are not indexed in
        DST mode)."""
        L = self.lines
        if len(L) < 5:
            return
        op, sh, on, mv, off = L[-5:]
        m = self._WRITE_MOV.fullmatch(mv)
        if not (m and int(m.group(1)) == N0 and on.endswith("gpr_idx(DST)") and off == "s_set_gpr_idx_off"
                and sh.startswith(f"s_lshr_b32 {s(SIDX)}, ")):
            return
        mo = re.fullmatch(rf"(v_\w+) v{m.group(2)}, (.*)", op)
        if not mo or "gpr_idx" in op:
            return
        L[-5:] = [sh, on, f"{mo.group(1)} {v(N0)}, {mo.group(2)}", off]

    def consume(self):
        """make the next instruction current without a dispatch (the next link
        of a W_CDINS chain, the next handler of a fused sequence) and prefetch
        the one after it into the bank this one vacates"""
        self.fuse_write()
        if DISPATCH == "single":
            self("s_waitcnt lgkmcnt(0)", f"s_mov_b64 {sr(CUR, 2)}, {sr(NXT, 2)}", f"s_mov_b64 {sr(CUR + 2, 2)}, {sr(NXT + 2, 2)}",
                 f"s_add_u32 {s(SOFF)}, {s(SOFF)}, 16", f"s_load_dwordx4 {sr(NXT, 4)}, {sr(CODE0, 2)}, {s(SOFF)}")
            return
        self("s_waitcnt lgkmcnt(0)", f"s_add_u32 {s(SOFF)}, {s(SOFF)}, 16",
             f"s_load_dwordx4 {sr(self.CUR, 4)}, {sr(CODE0, 2)}, {s(SOFF)}")
        self.CUR = self.other()

    def next(self):
        """dispatch the next instruction (each handler ends in its own copy:
        no jump back to a shared dispatch block).  It was prefetched one ahead;
        the stream ends in a validated END and no instruction jumps, so the
        offset only grows to it.  The predecoded word 0 holds the handler's
        word offset from Lpc0 in bits [14:0] (mw_asm_predecode, from the
        offsets the kernel reports in its introspection mode): one jump, no
        table."""
        self.fuse_write()
        if DISPATCH == "single":
            self("s_waitcnt lgkmcnt(0)", f"s_mov_b32 {s(JMP)}, {s(NXT)}", f"s_mov_b64 {sr(CUR, 2)}, {sr(NXT, 2)}",
                 f"s_mov_b64 {sr(CUR + 2, 2)}, {sr(NXT + 2, 2)}",
                 f"s_add_u32 {s(SOFF)}, {s(SOFF)}, 16", f"s_load_dwordx4 {sr(NXT, 4)}, {sr(CODE0, 2)}, {s(SOFF)}",
                 f"s_setpc_b64 {sr(JMP, 2)}")
            return
        self("s_waitcnt lgkmcnt(0)", f"s_add_u32 {s(SOFF)}, {s(SOFF)}, 16",
             f"s_load_dwordx4 {sr(self.CUR, 4)}, {sr(CODE0, 2)}, {s(SOFF)}",
             f"s_mov_b32 {s(JMP)}, {s(self.other())}", f"s_setpc_b64 {sr(JMP, 2)}")


# opcodes with a c operand and no immediate: mw_asm_predecode copies the c
# field into word 3, where s_set_gpr_idx_on takes it with no shift
C_IN_IMM = ("N_ITE", "W_ITE", "CHECK_IMPEQ", "CHECK_IMPEQW")


def build_handlers():
    """{opcode name: fn(g)} emitting that opcode's semantics with g's operand
    access (runtime-indexed in the interpreter, literal in assembled kernels)"""
    handlers = {}

    def handler(name):
        def deco(fn):
            handlers[name] = fn
            return fn
        return deco

    # -------------------------------------------------------- narrow
    for name, expr, masked in (("N_ADD", "v_add_u32_e32 {d}, {a}, {b}", True),
                               ("N_SUB", "v_sub_u32_e32 {d}, {a}, {b}", True),
                               ("N_AND", "v_and_b32_e32 {d}, {a}, {b}", False),
                               ("N_OR", "v_or_b32_e32 {d}, {a}, {b}", False),
                               ("N_XOR", "v_xor_b32_e32 {d}, {a}, {b}", False)):
        def h(g, expr=expr, masked=masked):
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_n(S[1], T + 1)
            g.op_n(S[0], expr.format(d=v(XR), a="{a}", b=v(T + 1)), T)
            if masked:
                g(f"v_and_b32_e32 {v(XR)}, {g.insn_mask(S[4])}, {v(XR)}")
            g.write_n(XR)
        handlers[name] = h

    @handler("N_MUL")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_n(S[1], T + 1)
        g.op_n(S[0], f"v_mul_lo_u32 {v(XR)}, {{a}}, {v(T + 1)}", T)
        g(f"v_and_b32_e32 {v(XR)}, {g.insn_mask(S[4])}, {v(XR)}")
        g.write_n(XR)

    for name, cmp in (("N_SLTN", "v_cmp_lt_u32_e32"), ("N_SLEN", "v_cmp_le_u32_e32")):
        def h(g, cmp=cmp):
            # signed w-bit compare of canonical values: flip bit w-1, compare unsigned
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_n(S[0], T), g.fetch_n(S[1], T + 1)
            g.width(S[2])
            g(f"s_sub_u32 {s(S[2])}, {s(S[2])}, 1", f"s_lshl_b32 {s(S[2])}, 1, {s(S[2])}",
              f"v_xor_b32_e32 {v(T)}, {s(S[2])}, {v(T)}", f"v_xor_b32_e32 {v(T + 1)}, {s(S[2])}, {v(T + 1)}",
              f"{cmp} vcc, {v(T)}, {v(T + 1)}")
            g.bool_from_vcc(XR)
            g.write_n(XR)
        handlers[name] = h

    @handler("N_UMULNON")
    def _(g):
        # a * b < 2^w: the high word is 0 and (w < 32) the low word has no bit >= w
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_n(S[0], T), g.fetch_n(S[1], T + 1)
        g.width(S[2]), g.nmask(S[2], S[4])
        g(f"v_mul_hi_u32 {v(T + 2)}, {v(T)}, {v(T + 1)}", f"v_mul_lo_u32 {v(T + 3)}, {v(T)}, {v(T + 1)}",
          f"s_not_b32 {s(S[4])}, {s(S[4])}", f"v_and_b32_e32 {v(T + 3)}, {s(S[4])}, {v(T + 3)}",
          f"v_or_b32_e32 {v(T + 2)}, {v(T + 2)}, {v(T + 3)}", f"v_cmp_eq_u32_e32 vcc, 0, {v(T + 2)}")
        g.bool_from_vcc(XR)
        g.write_n(XR)

    @handler("N_NOT")
    def _(g):
        g.field("a", S[0])
        g.op_n(S[0], f"v_xor_b32_e32 {v(XR)}, {g.insn_mask(S[4])}, {{a}}", T, "SRC1")   # ~a & m == a ^ m (a canonical)
        g.write_n(XR)

    for name, cmp in (("N_EQN", "v_cmp_eq_u32_e32"), ("N_ULTN", "v_cmp_lt_u32_e32"), ("N_ULEN", "v_cmp_le_u32_e32")):
        def h(g, cmp=cmp):
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_n(S[1], T + 1)
            g.op_n(S[0], f"{cmp} vcc, {{a}}, {v(T + 1)}", T)
            g.bool_from_vcc(XR)
            g.write_n(XR)
        handlers[name] = h

    @handler("N_ITE")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1]), g.field("c", S[2])
        g.fetch_n(S[0], T)
        g.op_n(S[2], "v_cmp_ne_u32_e32 vcc, 0, {a}", T + 2, "SRC1")
        g.nop_vcc()
        g.op_n(S[1], f"v_cndmask_b32_e32 {v(XR)}, {{a}}, {v(T)}, vcc", T + 1)
        g.write_n(XR)

    for name, op in (("N_SHLI", "v_lshlrev_b32_e32"), ("N_LSHRI", "v_lshrrev_b32_e32")):
        def h(g, op=op):
            g.field("a", S[0])
            big, j = g.L("sb"), g.L("sj")
            g(f"s_cmp_ge_u32 {s(g.CUR + 3)}, 32", f"s_cbranch_scc1 {big}")
            g.op_n(S[0], f"{op} {v(XR)}, {s(g.CUR + 3)}, {{a}}", T, "SRC1")
            g.width(S[2]), g.nmask(S[2], S[4])
            g(f"v_and_b32_e32 {v(XR)}, {s(S[4])}, {v(XR)}", f"s_branch {j}")
            g.label(big)
            g(f"v_mov_b32_e32 {v(XR)}, 0")
            g.label(j)
            g.write_n(XR)
        handlers[name] = h

    @handler("MOV_N")
    def _(g):
        g.field("a", S[0]), g.fetch_n(S[0], XR), g.write_n(XR)

    # -------------------------------------------------------- checks
    def update_alive(g):
        """alive &= vcc, then the early-exit test"""
        g(f"s_and_b64 {sr(AM, 2)}, {sr(AM, 2)}, vcc")
        g.all_dead_exit()

    @handler("CHECK")
    def _(g):
        g.field("a", S[0])
        g.op_n(S[0], "v_cmp_ne_u32_e32 vcc, 0, {a}", T, "SRC1")
        update_alive(g)

    @handler("CHECK_IMP")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.op_n(S[0], f"v_cmp_eq_u32_e64 {sr(MSK, 2)}, 0, {{a}}", T, "SRC1")
        g.op_n(S[1], "v_cmp_ne_u32_e32 vcc, 0, {a}", T + 1, "SRC1")
        g(f"s_or_b64 vcc, vcc, {sr(MSK, 2)}")
        update_alive(g)

    def impeq(g, keyed=False):
        """alive &= (a == 0) | (b == c) for the current bank's instruction
        (keyed, CHECK_IMPEQK: (a != imm) | (b == c)).  The premise is an
        index equality of a congruence pair, false in every lane for most
        pairs: then the check holds in every lane and b, c are not read (the
        interpreter; an assembled body's check runs fold the masks without
        branches)"""
        g.field("a", S[0]), g.field("b", S[1]), g.field("c", S[2])
        if keyed:
            g.op_n(S[0], f"v_cmp_ne_u32_e64 {sr(MSK, 2)}, {s(g.CUR + 3)}, {{a}}", T, "SRC1")
        else:
            g.op_n(S[0], f"v_cmp_eq_u32_e64 {sr(MSK, 2)}, 0, {{a}}", T, "SRC1")
        skip = g.L("iqskip") if g.chains else None
        if skip:
            g(f"s_cmp_eq_u64 {sr(MSK, 2)}, -1", f"s_cbranch_scc1 {skip}")
        g.fetch_n(S[2], T + 2)
        g.op_n(S[1], f"v_cmp_eq_u32_e32 vcc, {{a}}, {v(T + 2)}", T + 1)
        g(f"s_or_b64 vcc, vcc, {sr(MSK, 2)}")
        update_alive(g)
        if skip:
            g.label(skip)

    def impeq_run(g, keyed):
        # congruence checks come in runs (a C3 program: 2 176 of its 2 747
        # instructions): mw_asm_predecode flags a CHECK_IMPEQ followed by
        # another with bit 31 of word 3 (its c field sits in the low bits; a
        # CHECK_IMPEQK, whose word 3 is the premise constant: bit 31 of word
        # 1), and the handler takes the next one itself - a branch not taken
        # per link instead of a jump per instruction, two links per loop
        # trip, one per bank, each with its own exit (as W_CDINS chains)
        if not g.chains:
            impeq(g, keyed)
            return
        nlinks = 1 if DISPATCH == "single" else 2
        tops, exits = [g.L("iqtop") for _ in range(nlinks)], []
        for j in range(nlinks):
            g.label(tops[j])
            impeq(g, keyed)
            exits.append((g.L("iqlast"), g.CUR))
            g(f"s_bitcmp1_b32 {s(g.CUR + (1 if keyed else 3))}, 31", f"s_cbranch_scc0 {exits[-1][0]}")
            g.consume()
        g(f"s_branch {tops[0]}")
        for lab, bank in exits[1:]:
            g.label(lab)
            g.CUR = bank
            g.next()
        g.label(exits[0][0])
        g.CUR = exits[0][1]

    @handler("CHECK_IMPEQ")
    def _(g):
        impeq_run(g, False)

    @handler("CHECK_IMPEQK")
    def _(g):
        impeq_run(g, True)

    def eq8(g, a, b, dst_v):
        """dst_v = OR of the limb XORs (0 iff equal)"""
        for k in range(8):
            g(f"v_xor_b32_e32 {v(T + k)}, {v(a + k)}, {v(b + k)}")
        g(f"v_or3_b32 {v(T)}, {v(T)}, {v(T + 1)}, {v(T + 2)}", f"v_or3_b32 {v(T + 3)}, {v(T + 3)}, {v(T + 4)}, {v(T + 5)}",
          f"v_or3_b32 {v(dst_v)}, {v(T + 6)}, {v(T + 7)}, {v(T)}", f"v_or_b32_e32 {v(dst_v)}, {v(dst_v)}, {v(T + 3)}")

    @handler("CHECK_IMPEQW")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1]), g.field("c", S[2])
        g.fetch_n(S[0], XC), g.fetch_w(S[1], XA), g.fetch_w(S[2], XB)
        eq8(g, XA, XB, XC + 1)
        g(f"v_cmp_eq_u32_e64 {sr(MSK, 2)}, 0, {v(XC)}", f"v_cmp_eq_u32_e32 vcc, 0, {v(XC + 1)}",
          "s_nop 1", f"s_or_b64 vcc, vcc, {sr(MSK, 2)}")
        update_alive(g)

    @handler("CHECK_GRID")
    def _(g):
        """One row of a congruence grid (compiler.py _form_grids): j = imm - key;
        the live lanes with j < n read word T0 + j of their own spill area (LDS
        [word][lane] below nlds, else the global buffer, as spill_word) and
        must find b there.  c (raw): T0 = c & 1023, n - 1 = c >> 10 & 31."""
        g.field("a", S[0]), g.field("b", S[1])
        done, nolds, noglob = g.L("gd"), g.L("gl"), g.L("gg")
        if g.static_imm() is not None:     # an assembled body: the field is known
            g(f"s_mov_b32 {s(S[2])}, {_lit(g.cur['c'])}")
        else:
            g(f"s_lshr_b32 {s(S[2])}, {s(g.CUR + 2)}, 16")
        g.op_n(S[0], f"v_sub_u32_e32 {v(T)}, {s(g.CUR + 3)}, {{a}}", T + 4, "SRC1")
        g(f"s_and_b32 {s(S[3])}, {s(S[2])}, 1023", f"s_bfe_u32 {s(S[4])}, {s(S[2])}, 0x5000a",
          f"v_cmp_ge_u32_e32 vcc, {s(S[4])}, {v(T)}", f"s_and_b64 {sr(MSK2, 2)}, vcc, {sr(AM, 2)}",
          f"s_cbranch_scc0 {done}",
          f"v_add_u32_e32 {v(T + 1)}, {s(S[3])}, {v(T)}",
          f"s_mov_b64 {sr(EXECSV, 2)}, exec",
          f"v_cmp_gt_u32_e32 vcc, {s(NLDS)}, {v(T + 1)}",
          f"s_and_b64 exec, {sr(MSK2, 2)}, vcc", f"s_cbranch_scc0 {nolds}",
          f"v_lshlrev_b32_e32 {v(T + 2)}, 10, {v(T + 1)}", f"v_add_u32_e32 {v(T + 2)}, {v(T + 2)}, {v(LDSOFF)}",
          f"ds_read_b32 {v(T + 3)}, {v(T + 2)}")
        g.label(nolds)
        g(f"s_andn2_b64 exec, {sr(MSK2, 2)}, vcc", f"s_cbranch_scc0 {noglob}",
          f"v_subrev_u32_e32 {v(T + 2)}, {s(NLDS)}, {v(T + 1)}",
          f"v_mul_lo_u32 {v(T + 2)}, {v(T + 2)}, {s(GSTRIDE)}", f"v_add_u32_e32 {v(T + 2)}, {v(T + 2)}, {v(GOFF)}",
          f"global_load_dword {v(T + 3)}, {v(T + 2)}, {sr(GSP, 2)}")
        g.label(noglob)
        g(f"s_mov_b64 exec, {sr(MSK2, 2)}", "s_waitcnt vmcnt(0) lgkmcnt(0)")
        g.op_n(S[1], f"v_cmp_ne_u32_e32 vcc, {{a}}, {v(T + 3)}", T + 4)
        g(f"s_mov_b64 exec, {sr(EXECSV, 2)}", f"s_andn2_b64 {sr(AM, 2)}, {sr(AM, 2)}, vcc")
        g.all_dead_exit()
        g.label(done)

    # -------------------------------------------------------- wide -> narrow
    # N_EQ / N_ULT / N_ULE read operand a (N_ULE: b) as the VALU source
    # itself (Gen.w_indexed): no eight-move copy out of the W file
    @handler("N_EQ")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[1], XB)
        g.w_indexed(S[0], "SRC0", lambda base: g(*[f"v_xor_b32_e32 {v(T + k)}, {v(base + k)}, {v(XB + k)}"
                                                   for k in range(8)]))
        g(f"v_or3_b32 {v(T)}, {v(T)}, {v(T + 1)}, {v(T + 2)}", f"v_or3_b32 {v(T + 3)}, {v(T + 3)}, {v(T + 4)}, {v(T + 5)}",
          f"v_or3_b32 {v(XC)}, {v(T + 6)}, {v(T + 7)}, {v(T)}", f"v_or_b32_e32 {v(XC)}, {v(XC)}, {v(T + 3)}")
        g(f"v_cmp_eq_u32_e32 vcc, 0, {v(XC)}")
        g.bool_from_vcc(XR)
        g.write_n(XR)

    @handler("N_ULT")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[1], XB)
        g.w_indexed(S[0], "SRC0", lambda base: g.sub_chain(base, XB))
        g.bool_from_vcc(XR)
        g.write_n(XR)

    @handler("N_ULE")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XA)
        g.w_indexed(S[1], "SRC0", lambda base: g.sub_chain(base, XA), scratch=XB)   # b < a  ->  not (a <= b)
        g.bool_from_vcc(XR, invert=True)
        g.write_n(XR)

    for name, le in (("N_SLT", False), ("N_SLE", True)):
        def h(g, le=le):
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
            # flip bit w-1 of both (width = operand width), then compare unsigned
            g.width(S[2])
            g.flip_sign_bits(S[2], S[3])
            if le:
                g.sub_chain(XB, XA)
                g.bool_from_vcc(XR, invert=True)
            else:
                g.sub_chain(XA, XB)
                g.bool_from_vcc(XR)
            g.write_n(XR)
        handlers[name] = h

    @handler("N_EXTRACTW")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XA)
        # (x >> imm)[0] & nmask(w): limb q = imm >> 5 and the next, funnel by imm & 31
        g.extract_limb(S[1], S[2])
        g.width(S[3]), g.nmask(S[3], S[4])
        g(f"v_and_b32_e32 {v(XR)}, {s(S[4])}, {v(XR)}")
        g.write_n(XR)

    @handler("N_UMULNO")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
        mul_full(g, hi=True)
        # overflow iff any product bit >= w: low limbs above w (masked by ~limb_mask), or any high limb
        g.width(S[2])
        g(f"v_or3_b32 {v(T)}, {v(XC)}, {v(XC + 1)}, {v(XC + 2)}", f"v_or3_b32 {v(T)}, {v(T)}, {v(XC + 3)}, {v(XC + 4)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XC + 5)}, {v(XC + 6)}", f"v_or_b32_e32 {v(T)}, {v(T)}, {v(XC + 7)}")
        # low part: copy XR, canon it to w, and compare with XR (a difference = bits >= w)
        for k in range(8):
            g(f"v_mov_b32_e32 {v(XB + k)}, {v(XR + k)}")
        g.canon(XB, S[2])
        for k in range(8):
            g(f"v_xor_b32_e32 {v(XB + k)}, {v(XB + k)}, {v(XR + k)}")
        g(f"v_or3_b32 {v(T)}, {v(T)}, {v(XB)}, {v(XB + 1)}", f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 2)}, {v(XB + 3)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 4)}, {v(XB + 5)}", f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 6)}, {v(XB + 7)}",
          f"v_cmp_eq_u32_e32 vcc, 0, {v(T)}")
        g.bool_from_vcc(XR)
        g.write_n(XR)

    def udivrem(g):
        """XR = XA / XB, XC = XA % XB over 256 bits (canonical operands, so the
        w-bit results follow): restoring division, one quotient bit per step,
        most significant first, a uniform 256 steps.  A zero divisor gives all
        ones and the dividend: bvudiv / bvurem's definition (SMT-LIB, z3)."""
        for k in range(8):
            g(f"v_mov_b32_e32 {v(XC + k)}, 0", f"v_mov_b32_e32 {v(XR + k)}, {v(XA + k)}")
        g(f"s_movk_i32 {s(S[5])}, 0x100")
        top = g.L("dv")
        g.label(top)
        # (R:Q) <<= 1: funnel each limb with the top bit of the one below
        for k in range(7, 0, -1):
            g(f"v_alignbit_b32 {v(XC + k)}, {v(XC + k)}, {v(XC + k - 1)}, 31")
        g(f"v_alignbit_b32 {v(XC)}, {v(XC)}, {v(XR + 7)}, 31")
        for k in range(7, 0, -1):
            g(f"v_alignbit_b32 {v(XR + k)}, {v(XR + k)}, {v(XR + k - 1)}, 31")
        g(f"v_lshlrev_b32_e32 {v(XR)}, 1, {v(XR)}")
        g.sub_chain(XC, XB, T)                   # borrow (vcc): R < B
        g.nop_vcc()
        for k in range(8):
            g(f"v_cndmask_b32_e32 {v(XC + k)}, {v(T + k)}, {v(XC + k)}, vcc")
        g(f"v_cndmask_b32_e64 {v(T)}, 1, 0, vcc")
        g(f"v_or_b32_e32 {v(XR)}, {v(XR)}, {v(T)}")
        g(f"s_sub_u32 {s(S[5])}, {s(S[5])}, 1", f"s_cmp_lg_u32 {s(S[5])}, 0", f"s_cbranch_scc1 {top}")

    @handler("W_UDIV")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
        udivrem(g)
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    @handler("W_UREM")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
        udivrem(g)
        g.write_w(XC)

    @handler("N_ADDC")
    def _(g):
        # carry out of the w-bit add a + b of canonical operands: bit w of the
        # 257-bit sum (lower.py's bvaddc: BVAddNoOverflow's 257-bit add)
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
        g.add_chain(XA, XB, XR)
        g.bool_from_vcc(XR + 8)                 # bit 256 (XR + 8 is XC)
        g.width(S[2])
        g.bit_at(XR, S[2], T)
        g.write_n(T)

    @handler("N_ADDCN")
    def _(g):
        # ((a + b) >> w) & 1 for w <= 32: the 33-bit sum in T+2 (low), T+3 (carry)
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_n(S[0], T), g.fetch_n(S[1], T + 1)
        g(f"v_add_co_u32_e32 {v(T + 2)}, vcc, {v(T)}, {v(T + 1)}")
        g.bool_from_vcc(T + 3)
        g.width(S[2])
        g.bit_at(T + 2, S[2], XR)
        g.write_n(XR)

    # -------------------------------------------------------- wide
    def wbin(name, fn, canon=True):
        def h(g):
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
            fn(g)
            if canon:
                g.width(S[2]), g.canon(XR, S[2])
            g.write_w(XR)
        handlers[name] = h

    wbin("W_ADD", lambda g: g.add_chain(XA, XB, XR))
    wbin("W_SUB", lambda g: g.sub_chain(XA, XB, XR))
    for name, op in (("W_AND", "v_and_b32_e32"), ("W_OR", "v_or_b32_e32"), ("W_XOR", "v_xor_b32_e32")):
        wbin(name, lambda g, op=op: [g(f"{op} {v(XR + k)}, {v(XA + k)}, {v(XB + k)}") for k in range(8)])
    wbin("W_MUL", lambda g: mul_full(g, hi=False))

    @handler("W_NOT")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XA)
        for k in range(8):
            g(f"v_not_b32_e32 {v(XR + k)}, {v(XA + k)}")
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    @handler("MOV_W")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XR), g.write_w(XR)

    @handler("W_ITE")
    def _(g):
        g.field("a", S[0]), g.field("b", S[1]), g.field("c", S[2])
        g.fetch_n(S[2], T), g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
        g(f"v_cmp_ne_u32_e32 vcc, 0, {v(T)}")
        g.nop_vcc()
        for k in range(8):
            g(f"v_cndmask_b32_e32 {v(XR + k)}, {v(XB + k)}, {v(XA + k)}, vcc")
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    def shl_into(g, amount, dst):
        """dst..dst+7 = XA << amount (SGPR, < 256): written through a positive
        destination index (limbs past dst+7 land in the next 8 temporaries
        and are dropped); XA has zeros below it"""
        if amount == g.CUR + 3 and g.static_imm() is not None:   # an assembled body: literal limbs
            n = g.static_imm() & 255
            q, b = n >> 5, n & 31
            src = lambda i: v(XA + i) if i >= 0 else "0"   # noqa: E731
            for k in range(8):
                if k - q < 0:
                    g(f"v_mov_b32_e32 {v(dst + k)}, 0")
                elif b == 0:
                    g(f"v_mov_b32_e32 {v(dst + k)}, {v(XA + k - q)}")
                else:
                    g(f"v_alignbit_b32 {v(dst + k)}, {src(k - q)}, {src(k - q - 1)}, {32 - b}")
            return
        q, b = S[4], S[5]
        zb, j = g.L("z0"), g.L("sj")
        for k in range(8):
            g(f"v_mov_b32_e32 {v(dst + k)}, 0")
        g(f"s_lshr_b32 {s(q)}, {s(amount)}, 5", f"s_and_b32 {s(b)}, {s(amount)}, 31",
          f"s_cmp_eq_u32 {s(b)}, 0", f"s_cbranch_scc1 {zb}",
          f"s_sub_u32 {s(b)}, 32, {s(b)}",             # fshl(hi, lo, b) = alignbit(hi, lo, 32 - b)
          f"s_set_gpr_idx_on {s(q)}, gpr_idx(DST)")
        for k in range(8):
            g(f"v_alignbit_b32 {v(dst + k)}, {v(XA + k)}, {v(XA + k - 1)}, {s(b)}")
        g("s_set_gpr_idx_off", f"s_branch {j}")
        g.label(zb)
        g(f"s_set_gpr_idx_on {s(q)}, gpr_idx(DST)")
        for k in range(8):
            g(f"v_mov_b32_e32 {v(dst + k)}, {v(XA + k)}")
        g("s_set_gpr_idx_off")
        g.label(j)

    @handler("W_SHLI")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XA)
        shl_into(g, g.CUR + 3, XR)
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    @handler("W_LSHRI")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XA)
        if g.static_imm() is not None:      # an assembled body: literal limbs
            n = g.static_imm() & 255
            sq, sb = n >> 5, n & 31
            src = lambda i: v(XA + i) if i < 8 else "0"   # noqa: E731
            for k in range(8):
                g(f"v_alignbit_b32 {v(XR + k)}, {src(k + sq + 1)}, {src(k + sq)}, {sb}" if k + sq < 8
                  else f"v_mov_b32_e32 {v(XR + k)}, 0")
        else:
            q, b = S[4], S[5]
            g(f"s_lshr_b32 {s(q)}, {s(g.CUR + 3)}, 5", f"s_and_b32 {s(b)}, {s(g.CUR + 3)}, 31",
              f"s_set_gpr_idx_on {s(q)}, gpr_idx(SRC0,SRC1)")
            for k in range(8):
                g(f"v_alignbit_b32 {v(XR + k)}, {v(XA + k + 1)}, {v(XA + k)}, {s(b)}")
            g("s_set_gpr_idx_off")
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    def var_shift(g, kind):
        """XR = XA shifted by the per-lane amount XB (W_SHL / W_LSHR / W_ASHR;
        mw_alu.h wshl / wlshr / washr): amount >= w gives 0 (shl, lshr) or
        the sign fill (ashr).  A barrel shifter: three limb stages (4, 2, 1
        limbs, lanes select by bits 7..5 of the amount), then one funnel per
        limb by bits 4..0."""
        ge, tmp = SX, MSK2
        fill = None
        if kind == "ashr":
            # sign-extend the w-bit value to 256 bits: (a ^ m) - m, m = 1 << (w - 1)
            g.width(S[2])
            g(f"s_sub_u32 {s(S[3])}, {s(S[2])}, 1", f"s_lshr_b32 {s(S[4])}, {s(S[3])}, 5",
              f"s_and_b32 {s(S[3])}, {s(S[3])}, 31", f"s_lshl_b32 {s(S[3])}, 1, {s(S[3])}")
            for k in range(8):
                g(f"v_mov_b32_e32 {v(XC + k)}, 0")
            g(f"s_set_gpr_idx_on {s(S[4])}, gpr_idx(DST)", f"v_mov_b32_e32 {v(XC)}, {s(S[3])}", "s_set_gpr_idx_off")
            for k in range(8):
                g(f"v_xor_b32_e32 {v(XA + k)}, {v(XA + k)}, {v(XC + k)}")
            g.sub_chain(XA, XC, XA)
            fill = T + 3
            g(f"v_ashrrev_i32_e32 {v(fill)}, 31, {v(XA + 7)}")
        # ge: the amount's limbs 1..7 nonzero, or limb 0 >= w
        g(f"v_or3_b32 {v(T)}, {v(XB + 1)}, {v(XB + 2)}, {v(XB + 3)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 4)}, {v(XB + 5)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 6)}, {v(XB + 7)}")
        g.width(S[2])
        g(f"v_cmp_ne_u32_e64 {sr(ge, 2)}, 0, {v(T)}", f"v_cmp_ge_u32_e64 {sr(tmp, 2)}, {v(XB)}, {s(S[2])}",
          "s_nop 1", f"s_or_b64 {sr(ge, 2)}, {sr(ge, 2)}, {sr(tmp, 2)}")
        if kind == "ashr":   # shift by 255: every bit the sign
            g(f"v_mov_b32_e32 {v(T + 4)}, 0xff", "s_nop 1",
              f"v_cndmask_b32_e64 {v(XB)}, {v(XB)}, {v(T + 4)}, {sr(ge, 2)}")
        for st in range(3):
            n = 1 << st
            g(f"v_and_b32_e32 {v(T)}, {1 << (5 + st)}, {v(XB)}", f"v_cmp_ne_u32_e32 vcc, 0, {v(T)}")
            g.nop_vcc()
            order = range(7, -1, -1) if kind == "shl" else range(8)
            for k in order:
                src = k - n if kind == "shl" else k + n
                if 0 <= src < 8:
                    g(f"v_cndmask_b32_e32 {v(XA + k)}, {v(XA + k)}, {v(XA + src)}, vcc")
                elif fill is not None:
                    g(f"v_cndmask_b32_e32 {v(XA + k)}, {v(XA + k)}, {v(fill)}, vcc")
                else:
                    g(f"v_cndmask_b32_e64 {v(XA + k)}, {v(XA + k)}, 0, vcc")
        g(f"v_and_b32_e32 {v(T + 1)}, 31, {v(XB)}")
        if kind == "shl":
            # fshl(hi, lo, b) = alignbit(hi, lo, 32 - b), and hi itself for b = 0
            g(f"v_sub_u32_e32 {v(T + 2)}, 32, {v(T + 1)}", f"v_cmp_eq_u32_e32 vcc, 0, {v(T + 1)}")
            for k in range(7, 0, -1):
                g(f"v_alignbit_b32 {v(XR + k)}, {v(XA + k)}, {v(XA + k - 1)}, {v(T + 2)}")
            g(f"v_lshlrev_b32_e32 {v(XR)}, {v(T + 1)}, {v(XA)}")
            g.nop_vcc()
            for k in range(1, 8):
                g(f"v_cndmask_b32_e32 {v(XR + k)}, {v(XR + k)}, {v(XA + k)}, vcc")
        else:
            for k in range(7):
                g(f"v_alignbit_b32 {v(XR + k)}, {v(XA + k + 1)}, {v(XA + k)}, {v(T + 1)}")
            if fill is None:
                g(f"v_lshrrev_b32_e32 {v(XR + 7)}, {v(T + 1)}, {v(XA + 7)}")
            else:
                g(f"v_alignbit_b32 {v(XR + 7)}, {v(fill)}, {v(XA + 7)}, {v(T + 1)}")
        if kind != "ashr":
            for k in range(8):
                g(f"v_cndmask_b32_e64 {v(XR + k)}, {v(XR + k)}, 0, {sr(ge, 2)}")

    for _name, _kind in (("W_SHL", "shl"), ("W_LSHR", "lshr"), ("W_ASHR", "ashr")):
        def _h(g, kind=_kind):
            g.field("a", S[0]), g.field("b", S[1])
            g.fetch_w(S[0], XA), g.fetch_w(S[1], XB)
            var_shift(g, kind)
            if kind != "lshr":
                g.width(S[2]), g.canon(XR, S[2])
            g.write_w(XR)
        handlers[_name] = _h

    @handler("W_ZEXTN")
    def _(g):
        g.field("a", S[0]), g.fetch_n(S[0], XR)
        for k in range(1, 8):
            g(f"v_mov_b32_e32 {v(XR + k)}, 0")
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    @handler("W_INSN")
    def _(g):
        # r = a | (zext(N b) << imm)
        g.field("a", S[0]), g.field("b", S[1])
        g.fetch_w(S[0], XR), g.fetch_n(S[1], XA)
        if g.static_imm() is not None:      # an assembled body: the two limbs it reaches
            n = g.static_imm() & 255
            q, b = n >> 5, n & 31
            g(f"v_lshl_or_b32 {v(XR + q)}, {v(XA)}, {b}, {v(XR + q)}")
            if b and q + 1 < 8:
                g(f"v_lshrrev_b32_e32 {v(T)}, {32 - b}, {v(XA)}", f"v_or_b32_e32 {v(XR + q + 1)}, {v(XR + q + 1)}, {v(T)}")
        else:
            for k in range(1, 8):
                g(f"v_mov_b32_e32 {v(XA + k)}, 0")
            shl_imm_into_or(g, g.CUR + 3)
        g.width(S[2]), g.canon(XR, S[2])
        g.write_w(XR)

    def shl_imm_into_or(g, amount):
        """XR |= XA << amount (XA: an N value in limb 0, zeros above)"""
        shl_into(g, amount, XC)
        for k in range(8):
            g(f"v_or_b32_e32 {v(XR + k)}, {v(XR + k)}, {v(XC + k)}")

    def cdins_link(g):
        """one W_CDINS link on the current bank's instruction: XR |= the byte"""
        slow, rng, ins = g.L("cdslow"), g.L("cdrng"), g.L("cdins")
        # predecoded small index (mw_asm_predecode): c = 0x4000 | i, i < 0x4000
        g(f"s_bitcmp1_b32 {s(g.CUR + 2)}, 30", f"s_cbranch_scc0 {slow}",
          f"s_bfe_u32 {s(S[1])}, {s(g.CUR + 2)}, 0xe0010",        # i = bits [29:16]
          f"s_and_b32 {s(S[2])}, {s(g.CUR + 2)}, 0xffff",
          f"s_cmp_eq_u32 {s(S[2])}, {s(S[0])}", f"s_cbranch_scc1 {rng}",
          f"s_mov_b32 {s(S[0])}, {s(S[2])}")
        # size summary in XA: i <s size  <=>  i <u XA, XA = size < 0 ? 0 :
        # (size >= 2^32 ? 2^32 - 1 : size)   (i < 2^14)
        g.field("b", S[2]), g.fetch_w(S[2], XB)
        g(f"v_or3_b32 {v(T)}, {v(XB + 1)}, {v(XB + 2)}, {v(XB + 3)}",
          f"v_and_b32_e32 {v(T + 1)}, 0x7fffffff, {v(XB + 7)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 4)}, {v(XB + 5)}",
          f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 6)}, {v(T + 1)}",
          f"v_cmp_ne_u32_e32 vcc, 0, {v(T)}", "s_nop 1",
          f"v_cndmask_b32_e64 {v(XA)}, {v(XB)}, -1, vcc",
          f"v_cmp_gt_i32_e32 vcc, 0, {v(XB + 7)}", "s_nop 1",
          f"v_cndmask_b32_e64 {v(XA)}, {v(XA)}, 0, vcc")
        g.label(rng)
        g(f"v_cmp_lt_u32_e64 {sr(MSK2, 2)}, {s(S[1])}, {v(XA)}", "s_branch " + ins)
        # any other index: the full signed 256-bit compare
        g.label(slow)
        g(f"s_mov_b32 {s(S[0])}, -1")
        g.field("b", S[1]), g.fetch_w(S[1], XB)
        g.field("c", S[2]), g.fetch_w(S[2], XA)
        g(f"v_xor_b32_e32 {v(XA + 7)}, 0x80000000, {v(XA + 7)}", f"v_xor_b32_e32 {v(XB + 7)}, 0x80000000, {v(XB + 7)}")
        g.sub_chain(XA, XB)
        g(f"s_mov_b64 {sr(MSK2, 2)}, vcc")            # lanes whose byte is in range
        g.label(ins)
        # no lane in range: the inserted byte is 0 in every lane (no leaf draw)
        nos = g.L("cdns")
        g(f"s_cmp_eq_u64 {sr(MSK2, 2)}, 0", f"s_cbranch_scc1 {nos}")
        g(f"s_and_b32 {s(S[3])}, {s(g.CUR + 3)}, 0xffff")
        if g.inline_leaf:   # no call / return jumps on the hottest leaf path (C2: 64 of 86 instructions)
            g(f"s_mov_b32 {s(S67)}, {s(S[3])}")
            g(*leaf_inline(g.L("il")[1:-3], limb0=True))
        else:
            call_leaf(g, S[3])
        # t = in range ? byte : 0, inserted at bit off = imm >> 16 (limb off >> 5)
        g(f"v_cndmask_b32_e64 {v(T)}, 0, {v(XC)}, {sr(MSK2, 2)}",
          f"s_bfe_u32 {s(S[4])}, {s(g.CUR + 3)}, 0x80010",      # off: imm [23:16] (bit 31: the chain flag)
          f"s_lshr_b32 {s(S[5])}, {s(S[4])}, 5", f"s_and_b32 {s(S[4])}, {s(S[4])}, 31",
          f"s_set_gpr_idx_on {s(S[5])}, gpr_idx(SRC2,DST)",
          f"v_lshl_or_b32 {v(XR)}, {v(T)}, {s(S[4])}, {v(XR)}", "s_set_gpr_idx_off")
        # a byte straddling a limb boundary (off & 31 > 24): its high bits go to the next limb
        g(f"s_cmp_le_u32 {s(S[4])}, 24", f"s_cbranch_scc1 {nos}",
          f"s_sub_u32 {s(S[4])}, 32, {s(S[4])}", f"s_add_u32 {s(S[5])}, {s(S[5])}, 1",
          f"v_lshrrev_b32_e32 {v(T)}, {s(S[4])}, {v(T)}",
          f"s_set_gpr_idx_on {s(S[5])}, gpr_idx(SRC1,DST)",
          f"v_or_b32_e32 {v(XR)}, {v(T)}, {v(XR)}", "s_set_gpr_idx_off")
        g.label(nos)

    @handler("W_CDINS")
    def _(g):
        # acc | ((K[c] <s size) ? leaf(imm & 0xffff) : 0) << (imm >> 16), chained
        # links keep the word in XR (mw_interp.h MW_W_CDINS, MW_FLAG_CHAIN).
        # Two links per loop trip, one per bank, each with its own exit: the
        # first exit falls through to this handler's dispatch, the second
        # dispatches from the other bank
        g.field("a", S[0]), g.fetch_w(S[0], XR)
        g(f"s_mov_b32 {s(S[0])}, -1")                 # b operand of the cached size summary: none
        nlinks = 1 if DISPATCH == "single" else 2
        tops, exits = [g.L("cdtop") for _ in range(nlinks)], []
        for j in range(nlinks):
            g.label(tops[j])
            cdins_link(g)
            g.width(S[2]), g.canon(XR, S[2])
            # chained (imm bit 31): consume the next instruction (a W_CDINS whose acc is this word)
            exits.append((g.L("cdlast"), g.CUR))
            g(f"s_bitcmp1_b32 {s(g.CUR + 3)}, {CHAIN_BIT}", f"s_cbranch_scc0 {exits[-1][0]}")
            g.consume()
        g(f"s_branch {tops[0]}")
        for lab, bank in exits[1:]:
            g.label(lab)
            g.CUR = bank
            g.write_w(XR)
            g.next()
        g.label(exits[0][0])
        g.CUR = exits[0][1]
        g.write_w(XR)

    # -------------------------------------------------------- leaves
    def call_leaf(g, li):
        """XC..XC+7 = candidate value of leaf index li (SGPR)"""
        g(f"s_mov_b32 {s(S67)}, {s(li)}")
        g.call_leaf_sub()

    @handler("LEAF_W")
    def _(g):
        g(f"s_mov_b32 {s(S[0])}, {s(g.CUR + 3)}")
        call_leaf(g, S[0])
        g.write_w(XC)

    @handler("LEAF_N")
    def _(g):
        g(f"s_mov_b32 {s(S[0])}, {s(g.CUR + 3)}")
        call_leaf(g, S[0])
        g.write_n(XC)

    # -------------------------------------------------------- spills
    def spill_word(g, wd_sgpr, src, store=True):
        """word wd (SGPR) of this lane's spill area: LDS [wd][lane] below nlds, else the global buffer"""
        glob, j = g.L("sg"), g.L("sj")
        a = S[7]
        g(f"s_cmp_lt_u32 {s(wd_sgpr)}, {s(NLDS)}", f"s_cbranch_scc0 {glob}",
          f"s_lshl_b32 {s(a)}, {s(wd_sgpr)}, 10", f"v_add_u32_e32 {v(T + 7)}, {s(a)}, {v(LDSOFF)}")
        g(f"ds_write_b32 {v(T + 7)}, {v(src)}" if store else f"ds_read_b32 {v(src)}, {v(T + 7)}")
        g(f"s_branch {j}")
        g.label(glob)
        g(f"s_sub_u32 {s(a)}, {s(wd_sgpr)}, {s(NLDS)}", f"s_mul_i32 {s(a)}, {s(a)}, {s(GSTRIDE)}",
          f"v_add_u32_e32 {v(T + 7)}, {s(a)}, {v(GOFF)}")
        g(f"global_store_dword {v(T + 7)}, {v(src)}, {sr(GSP, 2)}" if store
          else f"global_load_dword {v(src)}, {v(T + 7)}, {sr(GSP, 2)}")
        g.label(j)

    @handler("SPILL_W")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XA)
        for k in range(8):
            g(f"s_add_u32 {s(S[1])}, {s(g.CUR + 3)}, {k}")
            spill_word(g, S[1], XA + k)
        g("s_waitcnt vmcnt(0) lgkmcnt(0)")

    @handler("SPILL_N")
    def _(g):
        g.field("a", S[0]), g.fetch_n(S[0], XA)
        g(f"s_mov_b32 {s(S[1])}, {s(g.CUR + 3)}")
        spill_word(g, S[1], XA)
        g("s_waitcnt vmcnt(0) lgkmcnt(0)")

    @handler("FILL_W")
    def _(g):
        for k in range(8):
            g(f"s_add_u32 {s(S[1])}, {s(g.CUR + 3)}, {k}")
            spill_word(g, S[1], XR + k, store=False)
        g("s_waitcnt vmcnt(0) lgkmcnt(0)")
        g.write_w(XR)

    @handler("FILL_N")
    def _(g):
        g(f"s_mov_b32 {s(S[1])}, {s(g.CUR + 3)}")
        spill_word(g, S[1], XR, store=False)
        g("s_waitcnt vmcnt(0) lgkmcnt(0)")
        g.write_n(XR)

    # -------------------------------------------------------- trace rows (mg_eval_generated)
    def store_rows(g, src, n):
        """trace[(imm + k) * ncand + (cand - begin)] = v(src + k), k < n, from
        the chunk's valid lanes only (rows validated against n_trace_rows,
        mw_validate.cpp; the host sizes the buffer rows x ncand); no trace
        buffer (searches): nothing"""
        skip = g.L("ts")
        g(f"s_cmp_eq_u64 {sr(TRACE, 2)}, 0", f"s_cbranch_scc1 {skip}",
          f"s_mul_i32 {s(S[1])}, {s(g.CUR + 3)}, {s(NCAND)}", f"s_lshl_b32 {s(S[2])}, {s(NCAND)}, 2",
          f"v_subrev_u32_e32 {v(T)}, {s(BEGIN)}, {v(CLO)}", f"v_add_u32_e32 {v(T)}, {s(S[1])}, {v(T)}",
          f"v_lshlrev_b32_e32 {v(T)}, 2, {v(T)}",
          f"s_mov_b64 {sr(EXECSV, 2)}, exec", f"s_mov_b64 exec, {sr(VALID, 2)}")
        for k in range(n):
            g(f"global_store_dword {v(T)}, {v(src + k)}, {sr(TRACE, 2)}")
            if k + 1 < n:
                g(f"v_add_u32_e32 {v(T)}, {s(S[2])}, {v(T)}")
        g(f"s_mov_b64 exec, {sr(EXECSV, 2)}", "s_waitcnt vmcnt(0)")
        g.label(skip)

    @handler("STORE_W")
    def _(g):
        g.field("a", S[0]), g.fetch_w(S[0], XR)
        store_rows(g, XR, 8)

    @handler("STORE_N")
    def _(g):
        g.field("a", S[0]), g.fetch_n(S[0], XR)
        store_rows(g, XR, 1)

    # -------------------------------------------------------- multiply
    def mul_full(g, hi):
        """XR = low 256 bits of XA * XB; with hi, XC = the high 256 bits.
        Row by row: acc[i+j] += a_i b_j + carry with one 64-bit mad each
        (mw_alu.h mul8 / mulhi8)."""
        acc = [XR + k for k in range(8)] + ([XC + k for k in range(8)] if hi else [])
        n = len(acc)
        for k in range(n):
            g(f"v_mov_b32_e32 {v(acc[k])}, 0")
        for i in range(8):
            g(f"v_mov_b32_e32 {v(T + 1)}, 0")                 # carry
            for j in range(8):
                if i + j >= n:
                    break
                g(f"v_mov_b32_e32 {v(T + 2)}, {v(acc[i + j])}", f"v_mov_b32_e32 {v(T + 3)}, 0",
                  f"v_mad_u64_u32 {vr(T + 4, 2)}, {sr(SX, 2)}, {v(XA + i)}, {v(XB + j)}, {vr(T + 2, 2)}",
                  f"v_add_co_u32_e32 {v(acc[i + j])}, vcc, {v(T + 4)}, {v(T + 1)}")
                g.nop_vcc()
                g(f"v_addc_co_u32_e32 {v(T + 1)}, vcc, 0, {v(T + 5)}, vcc")
            if i + 8 < n:
                g(f"v_mov_b32_e32 {v(acc[i + 8])}, {v(T + 1)}")

    handlers["_call_leaf"] = call_leaf
    return handlers


HANDLERS = build_handlers()
MARKER = "; MWJIT_BODY"


_NOT_SALU = ("s_cbranch", "s_branch", "s_setpc", "s_set_gpr_idx", "s_call", "s_swappc", "s_endpgm", "s_movrel")


def drop_idx_offs(lines):
    """`s_set_gpr_idx_off` then only scalar instructions (no VALU, no label,
    no branch) then `s_set_gpr_idx_on`: the off is dropped - the on replaces
    the index and the mode, and nothing between reads a VGPR."""
    out = []
    n = len(lines)
    for i, ln in enumerate(lines):
        if ln == "s_set_gpr_idx_off":
            j = i + 1
            while j < n and lines[j].startswith("s_") and not lines[j].startswith(_NOT_SALU) \
                    and not lines[j].endswith(":"):
                j += 1
            if j < n and lines[j].startswith("s_set_gpr_idx_on "):
                continue
        out.append(ln)
    return out


_VCMP_CONSUMERS = ("s_cmp_", "s_and_b64", "s_or_b64", "s_mov_b64", "s_andn2_b64", "v_cndmask")


def tidy_jumps(lines):
    """Branch peepholes over a body: a branch (or conditional branch) to a
    label whose first instruction is `s_branch Y` goes to Y; an `s_branch`
    to the very next instruction is dropped; an `s_nop 1` between a `v_cmp`
    and the scalar instruction or select that reads its mask is dropped (a
    VALU-written SGPR needs no wait states before an SALU or VALU read; only
    lane selects, VMEM and v_div_fmas do, which none of these are)."""
    def first_insn(i):
        while i < len(lines) and lines[i].endswith(":"):
            i += 1
        return i
    at = {ln[:-1]: i for i, ln in enumerate(lines) if ln.endswith(":")}
    out = list(lines)
    for i, ln in enumerate(out):
        if ln.startswith(("s_branch ", "s_cbranch_")):
            op, tgt = ln.split(" ", 1)
            for _ in range(8):
                j = at.get(tgt)
                if j is None:
                    break
                k = first_insn(j + 1)
                if k < len(lines) and lines[k].startswith("s_branch "):
                    tgt = lines[k].split(" ", 1)[1]
                else:
                    break
            out[i] = f"{op} {tgt}"
    res = []
    n = len(out)
    for i, ln in enumerate(out):
        if ln.startswith("s_branch "):
            tgt = ln.split(" ", 1)[1]
            j = i + 1
            labels = set()
            while j < n and out[j].endswith(":"):
                labels.add(out[j][:-1])
                j += 1
            if tgt in labels:
                continue
        if ln == "s_nop 1" and res and res[-1].startswith("v_cmp") and i + 1 < n \
                and out[i + 1].startswith(_VCMP_CONSUMERS):
            continue
        res.append(ln)
    return res


def _hlabel(n, bank):
    """an opcode's handler label in bank 0 (A) or 1 (B); "single" has bank A only"""
    return f"Lh_{n}_%=" if bank == 0 or DISPATCH == "single" else f"Lh_{n}_B_%="


def _flabel(k, bank):
    return f"Lf{k}_%=" if bank == 0 or DISPATCH == "single" else f"Lf{k}_B_%="


def gen(mode="interp"):
    """The inline-asm body, as a list of lines.  mode "interp": the
    threaded-dispatch interpreter; "template": the same kernel with the
    program's place marked by MARKER (an assembled kernel's straight-line body
    goes there and falls through to the chunk's result protocol)."""
    g = Gen()
    handlers = HANDLERS
    body = []
    g.lines = body
    # ---- once per block: launch arguments (AsmArgs) and the program (ProgDev)
    # from memory, per-lane constants from the operands
    g(f"s_mov_b64 {sr(ARGP, 2)}, %[args]", f"s_mov_b64 {sr(PROGP, 2)}, %[prog]",
      f"s_mov_b64 {sr(OUTMIN, 2)}, %[outmin]", f"s_mov_b32 {s(CH)}, %[ch0]",
      f"v_mov_b32_e32 {v(T)}, %[tid]", f"v_mov_b32_e32 {v(GOFF)}, %[goff]",
      f"s_load_dwordx8 {sr(DESC, 8)}, {sr(ARGP, 2)}, 0x0",
      f"s_load_dwordx8 {sr(72, 8)}, {sr(ARGP, 2)}, 0x20",
      "s_waitcnt lgkmcnt(0)",
      # AsmArgs: seed(2) begin(2) end(2) flags nlds | gstride nch gdx pad gsp(2) verdict(2)
      f"s_mov_b64 {sr(SEED, 2)}, {sr(DESC, 2)}", f"s_mov_b64 {sr(BEGIN, 2)}, {sr(DESC + 2, 2)}",
      f"s_mov_b64 {sr(END, 2)}, {sr(DESC + 4, 2)}", f"s_mov_b32 {s(FLAGS)}, {s(DESC + 6)}",
      f"s_mov_b32 {s(NLDS)}, {s(DESC + 7)}", f"s_mov_b32 {s(GSTRIDE)}, {s(72)}", f"s_mov_b32 {s(NCH)}, {s(73)}",
      # the chunk stride: the kernel body's (AsmArgs.gdx, or this program's
      # share of a 1D grid over several, mw_asm_abi.h)
      f"s_mov_b32 {s(GDX)}, %[gdx]", f"s_mov_b64 {sr(GSP, 2)}, {sr(76, 2)}", f"s_mov_b64 {sr(VERD, 2)}, {sr(78, 2)}",
      # AsmArgs (continued): trace(2) ncand pad
      f"s_load_dwordx4 {sr(72, 4)}, {sr(ARGP, 2)}, 0x40", "s_waitcnt lgkmcnt(0)",
      f"s_mov_b64 {sr(TRACE, 2)}, {sr(72, 2)}", f"s_mov_b32 {s(NCAND)}, {s(74)}",
      # ProgDev: code(2) consts(2) leaves(2) pool(2) | n_spill npool n_insn pad
      f"s_load_dwordx8 {sr(DESC, 8)}, {sr(PROGP, 2)}, 0x0", f"s_load_dwordx4 {sr(72, 4)}, {sr(PROGP, 2)}, 0x20",
      "s_waitcnt lgkmcnt(0)",
      f"s_mov_b64 {sr(CODE0, 2)}, {sr(DESC, 2)}", f"s_mov_b64 {sr(CPOOL, 2)}, {sr(DESC + 2, 2)}",
      f"s_mov_b64 {sr(LEAVES, 2)}, {sr(DESC + 4, 2)}",
      f"s_lshl_b32 {s(POOLB)}, {s(NLDS)}, 10",
      f"s_mov_b32 {s(PM0)}, 0xD2511F53", f"s_mov_b32 {s(PM1)}, 0xCD9E8D57",
      f"s_mov_b64 {sr(EVALS, 2)}, 0", f"s_mov_b32 {s(HIT)}, 0", f"s_mov_b32 {s(POLL)}, 0",
      f"v_lshlrev_b32_e32 {v(LDSOFF)}, 2, {v(T)}", f"v_mov_b32_e32 {v(TID)}, {v(T)}")
    if mode == "interp":
        # the handlers' base address (s_getpc_b64 gives the next instruction's)
        g(f"s_getpc_b64 {sr(TABLO, 2) if TABHI == TABLO + 1 else sr(SX, 2)}")
        g.label("Lpc0_%=")
        if TABHI != TABLO + 1:
            g(f"s_mov_b32 {s(TABLO)}, {s(SX)}", f"s_mov_b32 {s(TABHI)}, {s(SX + 1)}")
        # introspection (AsmArgs.flags bit 7): lane 0 writes the word offset of
        # every opcode's handler from Lpc0 to the verdict pointer, bank A's
        # table (opcodes, then the fused sequences) then bank B's, then Lpc0's
        # address (low, high word), and the kernel exits; mg_init reads them
        # once for mw_asm_predecode
        names = {c: n for n, c in isa.OPCODES.items()}
        g(f"s_bitcmp1_b32 {s(FLAGS)}, {INTROSPECT_FLAG}", "s_cbranch_scc0 Lnointro_%=",
          f"s_mov_b64 {sr(EXECSV, 2)}, exec", "s_mov_b64 exec, 1")
        nh = NTAB + len(isa.ASM_FUSED)
        for bank in range(2):
            for code in range(NTAB):
                n = names.get(code)
                tgt = f"{_hlabel(n, bank)}" if n in handlers else "Lh_END_%=" if n == "END" else "Lunsup_%="
                g(f"v_mov_b32_e32 {v(T)}, (({tgt} - Lpc0_%=) >> 2)", f"v_mov_b32_e32 {v(T + 1)}, {4 * (bank * nh + code)}",
                  f"global_store_dword {v(T + 1)}, {v(T)}, {sr(VERD, 2)}")
            for k in range(len(isa.ASM_FUSED)):   # the fused handlers' offsets follow (entries NTAB + k)
                g(f"v_mov_b32_e32 {v(T)}, (({_flabel(k, bank)} - Lpc0_%=) >> 2)",
                  f"v_mov_b32_e32 {v(T + 1)}, {4 * (bank * nh + NTAB + k)}",
                  f"global_store_dword {v(T + 1)}, {v(T)}, {sr(VERD, 2)}")
        for j, reg in enumerate((TABLO, TABHI)):
            g(f"v_mov_b32_e32 {v(T)}, {s(reg)}", f"v_mov_b32_e32 {v(T + 1)}, {4 * (2 * nh + j)}",
              f"global_store_dword {v(T + 1)}, {v(T)}, {sr(VERD, 2)}")
        g(f"s_mov_b64 exec, {sr(EXECSV, 2)}", "s_branch Lexit_%=")
        g.label("Lnointro_%=")
        # the program's narrow constants (mw_asm_predecode: after the predecoded
        # code and the 8 words the dispatch prefetches past END) -> v240..v255
        g(f"s_lshl_b32 {s(74)}, {s(74)}, 4", f"s_add_u32 {s(74)}, {s(74)}, 32",
          f"s_load_dwordx16 {sr(DESC, 16)}, {sr(CODE0, 2)}, {s(74)}", "s_waitcnt lgkmcnt(0)")
        for k in range(NKN):
            g(f"v_mov_b32_e32 {v(NK0 + k)}, {s(DESC + k)}")
        # the dispatch target's high word, for good (after that load: s80..s95)
        g(f"s_mov_b32 {s(JMP + 1)}, {s(TABHI)}")
    else:
        for reg, lab in ((LEAFADDR, "Lleaf_%="), (STOPADDR, "Lstop_%="), (ENDADDR, "Lh_END_%="),
                         (PHILOXADDR, "Lphilox_%=")):
            g.long_addr(reg, lab)
    for k in range(XA - 8, XA, 2):       # the shift padding below and above XA
        g(f"v_mov_b64 {vr(k, 2)}, 0")
    for k in range(XA + 8, XA + 16, 2):
        g(f"v_mov_b64 {vr(k, 2)}, 0")
    # ---- chunk loop: chunk ch covers [begin + 256 ch, +256)
    g.label("Lchunk_%=")
    g(f"s_cmp_lt_u32 {s(CH)}, {s(NCH)}", "s_cbranch_scc0 Lexit_%=",
      f"s_lshl_b32 {s(BASE)}, {s(CH)}, 8", f"s_lshr_b32 {s(BASE + 1)}, {s(CH)}, 24",
      f"s_add_u32 {s(BASE)}, {s(BASE)}, {s(BEGIN)}", f"s_addc_u32 {s(BASE + 1)}, {s(BASE + 1)}, {s(BEGIN + 1)}",
      # stop after hit: a witness below this chunk is known (a stale read only
      # delays the stop).  Polled every POLL_EVERY-th chunk of the wave, not
      # its first: every wave reading the one witness word past the caches
      # queues at one memory channel (a 2^22-candidate miss spent most of its
      # 1.8 ms there, profiles/r5d), and a probe launch covers the lowest
      # indices (engine.search_phased)
      f"s_bitcmp1_b32 {s(FLAGS)}, 1", "s_cbranch_scc0 Lnostop_%=",
      f"s_add_u32 {s(POLL)}, {s(POLL)}, 1", f"s_and_b32 {s(SX)}, {s(POLL)}, {POLL_EVERY - 1}",
      f"s_cmp_lg_u32 {s(SX)}, 0", "s_cbranch_scc1 Lnostop_%=",
      f"s_load_dwordx2 {sr(SX, 2)}, {sr(OUTMIN, 2)}, 0x0 glc", "s_waitcnt lgkmcnt(0)",
      # m <= base  <=>  !(base < m): compare (hi, lo) lexicographically
      f"s_cmp_lt_u32 {s(SX + 1)}, {s(BASE + 1)}", "s_cbranch_scc1 Lexit_%=",
      f"s_cmp_eq_u32 {s(SX + 1)}, {s(BASE + 1)}", "s_cbranch_scc0 Lnostop_%=",
      f"s_cmp_le_u32 {s(SX)}, {s(BASE)}", "s_cbranch_scc1 Lexit_%=")
    g.label("Lnostop_%=")
    g(f"s_mov_b32 {s(DIGKEY)}, -1",
      f"v_mov_b32_e32 {v(T + 7)}, {s(BASE + 1)}",
      f"v_add_co_u32_e32 {v(CLO)}, vcc, {s(BASE)}, {v(TID)}", "s_nop 1",
      f"v_addc_co_u32_e32 {v(CHI)}, vcc, 0, {v(T + 7)}, vcc",
      f"v_cmp_gt_u64_e32 vcc, {sr(END, 2)}, {vr(CLO, 2)}", "s_nop 1",
      f"s_mov_b64 {sr(VALID, 2)}, vcc", f"s_mov_b64 {sr(AM, 2)}, vcc")
    if mode == "interp":
        # the register files start at zero (an assembled body zeroes the
        # registers it reads before writing them: static_body / dead_code)
        for k in range(0, N0 + NFILE, 2):
            g(f"v_mov_b64 {vr(k, 2)}, 0")
    if mode == "template":
        g.long_addr(SX, "Lbody_%=")
        g(f"s_setpc_b64 {sr(SX, 2)}")
    else:
        # ---- the first dispatch: instruction 0 into bank A, 1 into bank B
        if DISPATCH == "single":
            g(f"s_mov_b32 {s(SOFF)}, 0", f"s_load_dwordx4 {sr(NXT, 4)}, {sr(CODE0, 2)}, 0x0")
            g.next()
        else:
            g(f"s_mov_b32 {s(SOFF)}, 16", f"s_load_dwordx4 {sr(CUR, 4)}, {sr(CODE0, 2)}, 0x0",
              f"s_load_dwordx4 {sr(NXT, 4)}, {sr(CODE0, 2)}, 0x10", "s_waitcnt lgkmcnt(0)",
              f"s_mov_b32 {s(JMP)}, {s(CUR)}", f"s_setpc_b64 {sr(JMP, 2)}")
        # handlers, once per bank
        for bank in range(1 if DISPATCH == "single" else 2):
            for n in ASM_OPCODES:
                if n == "END":
                    continue
                g.CUR = (CUR, NXT)[bank]
                g.label(_hlabel(n, bank))
                g.c_in_imm = n in C_IN_IMM
                handlers[n](g)
                g.next()
                g.flush_tail()
            # fused sequences (isa.ASM_FUSED): the handlers back to back, each
            # later one taking its instruction as a W_CDINS chain link does;
            # one dispatch at the end
            for k, seq in enumerate(isa.ASM_FUSED):
                g.CUR = (CUR, NXT)[bank]
                g.label(_flabel(k, bank))
                for j, n in enumerate(seq):
                    if j:
                        g.consume()
                    g.c_in_imm = n in C_IN_IMM
                    handlers[n](g)
                g.next()
                g.flush_tail()
            # every lane dead (a check's all_dead_exit): the chunk ends, or
            # without early exit (traces, verdicts) the next instruction runs
            g.CUR = (CUR, NXT)[bank]
            g.label(f"Ldead{'AB'[bank]}_%=")
            g(f"s_bitcmp1_b32 {s(FLAGS)}, 0", "s_cbranch_scc1 Lstop_%=")
            g.next()
        g.CUR = CUR
    if mode == "interp":
        body[:] = drop_idx_offs(body)
    g.label("Lunsup_%=")
    g.label("Lstop_%=")
    g(f"s_mov_b64 {sr(AM, 2)}, 0")
    g.label("Lh_END_%=")
    # ---- this chunk's result: verdicts, evals, lowest satisfying lane -> atomic min
    g("s_waitcnt vmcnt(0) lgkmcnt(0)",
      f"s_and_b64 {sr(MSK, 2)}, {sr(AM, 2)}, {sr(VALID, 2)}",
      f"s_bcnt1_i32_b64 {s(SX)}, {sr(VALID, 2)}",
      f"s_add_u32 {s(EVALS)}, {s(EVALS)}, {s(SX)}", f"s_addc_u32 {s(EVALS + 1)}, {s(EVALS + 1)}, 0",
      f"s_cmp_eq_u64 {sr(VERD, 2)}, 0", "s_cbranch_scc1 Lnoverd_%=",
      f"v_cndmask_b32_e64 {v(T)}, 0, 1, {sr(MSK, 2)}",
      # verdict[cand - begin]: byte offset (ch * 256 + tid) * 4
      f"s_lshl_b32 {s(SX)}, {s(CH)}, 10", f"v_add_u32_e32 {v(T + 1)}, {s(SX)}, {v(LDSOFF)}",
      f"s_mov_b64 {sr(EXECSV, 2)}, exec", f"s_mov_b64 exec, {sr(VALID, 2)}",
      f"global_store_dword {v(T + 1)}, {v(T)}, {sr(VERD, 2)}",
      f"s_mov_b64 exec, {sr(EXECSV, 2)}")
    g.label("Lnoverd_%=")
    g(f"s_cmp_eq_u64 {sr(MSK, 2)}, 0", "s_cbranch_scc1 Lnohit_%=",
      # a wave that has reported a witness never reports again: its later
      # chunks hold only larger indices (one contended atomic per wave, not
      # one per satisfied chunk: dense programs queued them on one address)
      f"s_cmp_lg_u32 {s(HIT)}, 0", "s_cbranch_scc1 Lnohit_%=",
      # the wave's lowest satisfying lane issues the atomic with its own candidate index
      f"s_ff1_i32_b64 {s(SX)}, {sr(MSK, 2)}", f"s_lshl_b64 {sr(MSK2, 2)}, 1, {s(SX)}",
      f"s_mov_b64 {sr(EXECSV, 2)}, exec", f"s_mov_b64 exec, {sr(MSK2, 2)}",
      f"v_mov_b32_e32 {v(T + 2)}, 0",
      f"global_atomic_umin_x2 {v(T + 2)}, {vr(CLO, 2)}, {sr(OUTMIN, 2)}",
      f"s_mov_b64 exec, {sr(EXECSV, 2)}", f"s_mov_b32 {s(HIT)}, 1")
    g.label("Lnohit_%=")
    g(f"s_add_u32 {s(CH)}, {s(CH)}, {s(GDX)}", "s_branch Lchunk_%=")
    # ------------------------------------------------------ subroutines
    leaf(g)
    philox_sub(g)
    g.label("Lexit_%=")
    g("s_waitcnt vmcnt(0) lgkmcnt(0)", f"s_mov_b64 %[evals], {sr(EVALS, 2)}")
    if mode == "template":
        # the program's straight-line body last (it ends in a jump to Lh_END)
        g.long_addr(SX, "Ldone_%=")
        g(f"s_setpc_b64 {sr(SX, 2)}")
        g.label("Lbody_%=")
        g(MARKER)
        g.label("Ldone_%=")
    if mode == "interp":
        body[:] = tidy_jumps(body)
    return body


def leaf(g, limb0=False):
    """Lleaf: XC = value of leaf S67 for this lane's candidate (mw_leaf.h
    leaf_value with the pool in LDS: kinds 0 random, 1 bit-field digit,
    2 hashed digit, 3 bit-interleaved digit; a pool entry flagged RANDOM draws
    Philox).  limb0: a narrow leaf leaves XC+1..XC+7 as they are (a caller
    that reads XC alone: W_CDINS's byte)."""
    D = DESC   # s80 w, s81 kind, s82 id, s83 shift, s84 bits, s85 poff, s86 inrow, s87 stride
    g.label("Lleaf_%=")
    g(f"s_lshl_b32 {s(S[7])}, {s(S67)}, 5", f"s_load_dwordx8 {sr(D, 8)}, {sr(LEAVES, 2)}, {s(S[7])}",
      "s_waitcnt lgkmcnt(0)",
      # the same digit as the last pooled leaf drawn (the bytes of one calldata
      # word): reuse it (word 6: the digit group; distinct per leaf in the
      # assembled kernels' table, where it is the input row)
      f"s_cmp_eq_u32 {s(D + 6)}, {s(DIGKEY)}", "s_cbranch_scc1 Ldig_hit_%=",
      # kind 3 first: the bit-interleaved digits of every pooled leaf that fits the 40 index bits
      f"s_cmp_eq_u32 {s(D + 1)}, 3", "s_cbranch_scc1 Lk3_%=",
      f"s_cmp_eq_u32 {s(D + 1)}, 1", "s_cbranch_scc1 Lk1_%=",
      f"s_cmp_eq_u32 {s(D + 1)}, 2", "s_cbranch_scc1 Lk2_%=",
      # kind 0 (or anything else: the host never launches other kinds here): Philox
      f"s_call_b64 {sr(PRET, 2)}, Lphilox_%=",
      # w < 32: the draw's low word masked to w bits is the canonical value
      f"s_cmp_lt_u32 {s(D)}, 32", "s_cbranch_scc0 Lk0_wide_%=",
      f"s_bfm_b64 {sr(S[6], 2)}, {s(D)}, 0", f"v_and_b32_e32 {v(XC)}, {s(S[6])}, {v(T)}")
    for k in range(1, 1 if limb0 else 8):
        g(f"v_mov_b32_e32 {v(XC + k)}, 0")
    g(f"s_setpc_b64 {sr(LRET, 2)}")
    g.label("Lk0_wide_%=")
    for k in range(8):
        g(f"v_mov_b32_e32 {v(XC + k)}, {v(T + k)}")
    g("s_branch Lleaf_canon_%=")
    # kind 1: digit = (cand >> shift) & (2^bits - 1)
    g.label("Lk1_%=")
    g(f"v_lshrrev_b64 {vr(T, 2)}, {s(D + 3)}, {vr(CLO, 2)}")
    g(f"s_bfm_b32 {s(S[6])}, {s(D + 4)}, 0", f"s_cmp_ge_u32 {s(D + 4)}, 32", f"s_cselect_b32 {s(S[6])}, -1, {s(S[6])}",
      f"v_and_b32_e32 {v(T + 6)}, {s(S[6])}, {v(T)}", "s_branch Lgather_%=")
    # kind 2: digit = fmix64(cand ^ id * 0x9E3779B97F4A7C15) & (2^bits - 1) (MurmurHash3 finalizer)
    g.label("Lk2_%=")
    lo, hi, t1, t2 = T, T + 1, T + 2, T + 3
    g(f"s_mul_i32 {s(S[6])}, {s(D + 2)}, 0x7F4A7C15", f"s_mul_hi_u32 {s(S[7])}, {s(D + 2)}, 0x7F4A7C15",
      f"s_mul_i32 {s(S[4])}, {s(D + 2)}, 0x9E3779B9", f"s_add_u32 {s(S[7])}, {s(S[7])}, {s(S[4])}",
      f"v_xor_b32_e32 {v(lo)}, {s(S[6])}, {v(CLO)}", f"v_xor_b32_e32 {v(hi)}, {s(S[7])}, {v(CHI)}")

    fmix64(g, lo, hi, t1, t2)
    g(f"s_bfm_b32 {s(S[6])}, {s(D + 4)}, 0", f"s_cmp_ge_u32 {s(D + 4)}, 32", f"s_cselect_b32 {s(S[6])}, -1, {s(S[6])}",
      f"v_and_b32_e32 {v(T + 6)}, {s(S[6])}, {v(lo)}", "s_branch Lgather_%=")
    # kind 3: digit bit b = index bit (shift + b * stride): one 64-bit shift
    # of the index per bit, one loop branch (shift + (bits-1) * stride <= 63,
    # validated)
    g.label("Lk3_%=")
    g(f"v_mov_b32_e32 {v(T + 6)}, 0", f"s_mov_b32 {s(S[4])}, 0", f"s_mov_b32 {s(S[5])}, {s(D + 3)}",
      f"s_cmp_eq_u32 {s(D + 4)}, 0", "s_cbranch_scc1 Lgather_%=")
    g.label("Lm_loop_%=")
    g(f"v_lshrrev_b64 {vr(T + 4, 2)}, {s(S[5])}, {vr(CLO, 2)}", f"v_and_b32_e32 {v(T + 7)}, 1, {v(T + 4)}",
      f"v_lshl_or_b32 {v(T + 6)}, {v(T + 7)}, {s(S[4])}, {v(T + 6)}",
      f"s_add_u32 {s(S[4])}, {s(S[4])}, 1", f"s_add_u32 {s(S[5])}, {s(S[5])}, {s(D + 7)}",
      f"s_cmp_lt_u32 {s(S[4])}, {s(D + 4)}", "s_cbranch_scc1 Lm_loop_%=")
    # pool entry in LDS at poolb + 4 * poff: width >= 32: 9 words (flag, 8 limbs)
    # at + 36 * digit; width < 32: one word (bit 31 RANDOM, else the value) at + 4 * digit
    g.label("Lgather_%=")
    g(f"v_mov_b32_e32 {v(DIGV)}, {v(T + 6)}", f"s_mov_b32 {s(DIGKEY)}, {s(D + 6)}", "s_branch Lgather2_%=")
    g.label("Ldig_hit_%=")
    g(f"v_mov_b32_e32 {v(T + 6)}, {v(DIGV)}")
    g.label("Lgather2_%=")
    g(f"s_lshl_b32 {s(S[6])}, {s(D + 5)}, 2", f"s_add_u32 {s(S[6])}, {s(S[6])}, {s(POOLB)}",
      f"s_cmp_lt_u32 {s(D)}, 32", "s_cbranch_scc1 Lg_narrow_%=",
      f"v_mov_b32_e32 {v(T + 5)}, 36", f"v_mad_u32_u24 {v(T + 5)}, {v(T + 6)}, {v(T + 5)}, {s(S[6])}",
      f"ds_read_b32 {v(T + 4)}, {v(T + 5)}")
    for k in range(4):
        g(f"ds_read2_b32 {vr(XC + 2 * k, 2)}, {v(T + 5)} offset0:{1 + 2 * k} offset1:{2 + 2 * k}")
    g("s_waitcnt lgkmcnt(0)", f"v_and_b32_e32 {v(T + 4)}, 1, {v(T + 4)}", "s_branch Lg_flag_%=")
    # w < 32: pool values are canonical already (masked when the pool is laid
    # out); only RANDOM lanes draw, and their value is the draw's low word
    # masked to w bits (no 8-limb select, no generic canonicalisation)
    g.label("Lg_narrow_%=")
    g(f"v_lshl_add_u32 {v(T + 5)}, {v(T + 6)}, 2, {s(S[6])}", f"ds_read_b32 {v(XC)}, {v(T + 5)}")
    for k in range(1, 1 if limb0 else 8):
        g(f"v_mov_b32_e32 {v(XC + k)}, 0")
    g("s_waitcnt lgkmcnt(0)", f"v_lshrrev_b32_e32 {v(T + 4)}, 31, {v(XC)}",
      f"v_cmp_ne_u32_e32 vcc, 0, {v(T + 4)}", "s_nop 1", "s_cmp_eq_u64 vcc, 0", "s_cbranch_scc1 Lleaf_ret_%=",
      f"s_mov_b64 {sr(MSK, 2)}, vcc", f"s_call_b64 {sr(PRET, 2)}, Lphilox_%=", "s_nop 1",
      f"v_cndmask_b32_e64 {v(XC)}, {v(XC)}, {v(T)}, {sr(MSK, 2)}",
      f"s_bfm_b64 {sr(S[6], 2)}, {s(D)}, 0", f"v_and_b32_e32 {v(XC)}, {s(S[6])}, {v(XC)}")
    g.label("Lleaf_ret_%=")
    g(f"s_setpc_b64 {sr(LRET, 2)}")
    g.label("Lg_flag_%=")
    g(f"v_cmp_ne_u32_e32 vcc, 0, {v(T + 4)}",
      "s_nop 1", "s_cmp_eq_u64 vcc, 0", "s_cbranch_scc1 Lleaf_canon_%=",
      f"s_mov_b64 {sr(MSK, 2)}, vcc", f"s_call_b64 {sr(PRET, 2)}, Lphilox_%=", "s_nop 1")
    for k in range(8):
        g(f"v_cndmask_b32_e64 {v(XC + k)}, {v(XC + k)}, {v(T + k)}, {sr(MSK, 2)}")
    g.label("Lleaf_canon_%=")
    g.canon(XC, D)
    g(f"s_setpc_b64 {sr(LRET, 2)}")


def leaf_inline(tag, limb0=False):
    """The Lleaf subroutine's code for one call site: its labels prefixed with
    tag, its returns a branch to the end (the Philox subroutine is still
    called)"""
    sub = Gen()
    leaf(sub, limb0)
    defined = [ln[:-1] for ln in sub.lines if ln.endswith(":")]
    done = f"L{tag}ret_%="
    out = []
    for ln in sub.lines:
        for lab in defined:   # "_%=" ends every label: no label is a prefix of another's text
            ln = ln.replace(lab, f"L{tag}{lab[1:]}")
        out.append(ln.replace(f"s_setpc_b64 {sr(LRET, 2)}", f"s_branch {done}"))
    return out + [done + ":"]


def fmix64(g, lo, hi, t1, t2):
    """(hi:lo) = MurmurHash3's 64-bit finalizer of (hi:lo) (mw_leaf.h fmix64);
    temporaries t1, t2, T+4..T+5, S[4], S[5] and the carry pair SX"""
    def xs33():   # h ^= h >> 33
        g(f"v_lshrrev_b32_e32 {v(t1)}, 1, {v(hi)}", f"v_xor_b32_e32 {v(lo)}, {v(lo)}, {v(t1)}")

    def mul64(c):  # h *= c (mod 2^64)
        g(f"s_mov_b32 {s(S[4])}, {c & 0xFFFFFFFF:#x}", f"s_mov_b32 {s(S[5])}, {c >> 32:#x}",
          f"v_mul_lo_u32 {v(t1)}, {v(lo)}, {s(S[5])}", f"v_mul_lo_u32 {v(t2)}, {v(hi)}, {s(S[4])}",
          f"v_mad_u64_u32 {vr(T + 4, 2)}, {sr(SX, 2)}, {v(lo)}, {s(S[4])}, 0",
          f"v_mov_b32_e32 {v(lo)}, {v(T + 4)}", f"v_add3_u32 {v(hi)}, {v(T + 5)}, {v(t1)}, {v(t2)}")
    xs33()
    mul64(0xFF51AFD7ED558CCD)
    xs33()
    mul64(0xC4CEB9FE1A85EC53)
    xs33()


def philox_sub(g):
    """Lphilox: T..T+7 = the random leaf value of the candidate index
    (mw_leaf.h random_leaf): w > 32 Philox4x32-10 blocks 0 and (w > 128) 1,
    key (seed_lo ^ id, seed_hi); w <= 32 fmix64(c ^ seed ^ id * 0xC2B2AE3D27D4EB4F)."""
    D = DESC
    g.label("Lphilox_%=")
    narrow = 0xC2B2AE3D27D4EB4F
    g(f"s_cmp_gt_u32 {s(D)}, 32", "s_cbranch_scc1 Lphx_wide_%=",
      # key (PK1:PK0) = seed ^ id * narrow (mod 2^64)
      f"s_mul_i32 {s(PK0)}, {s(D + 2)}, {narrow & 0xFFFFFFFF:#x}",
      f"s_mul_hi_u32 {s(PK1)}, {s(D + 2)}, {narrow & 0xFFFFFFFF:#x}",
      f"s_mul_i32 {s(S[4])}, {s(D + 2)}, {narrow >> 32:#x}", f"s_add_u32 {s(PK1)}, {s(PK1)}, {s(S[4])}",
      f"s_xor_b32 {s(PK0)}, {s(PK0)}, {s(SEED)}", f"s_xor_b32 {s(PK1)}, {s(PK1)}, {s(SEED + 1)}",
      f"v_xor_b32_e32 {v(T)}, {s(PK0)}, {v(CLO)}", f"v_xor_b32_e32 {v(T + 1)}, {s(PK1)}, {v(CHI)}")
    fmix64(g, T, T + 1, T + 2, T + 3)
    for k in range(1, 8):
        g(f"v_mov_b32_e32 {v(T + k)}, 0")
    g(f"s_setpc_b64 {sr(PRET, 2)}")
    g.label("Lphx_wide_%=")
    g(f"v_mov_b32_e32 {v(T + 4)}, 0", f"v_mov_b32_e32 {v(T + 5)}, 0", f"v_mov_b32_e32 {v(T + 6)}, 0",
      f"v_mov_b32_e32 {v(T + 7)}, 0")
    for blk in (0, 1):
        base = T + 4 * blk
        if blk == 1:
            g(f"s_cmp_le_u32 {s(D)}, 128", "s_cbranch_scc1 Lphx_done_%=")
        # counter (c0, c1, c2, c3) = (cand_lo, cand_hi, blk, 0) in base..base+3; temporaries XB..XB+7
        c = [base, base + 1, base + 2, base + 3]
        g(f"v_mov_b32_e32 {v(c[0])}, {v(CLO)}", f"v_mov_b32_e32 {v(c[1])}, {v(CHI)}",
          f"v_mov_b32_e32 {v(c[2])}, {blk}", f"v_mov_b32_e32 {v(c[3])}, 0",
          f"s_xor_b32 {s(PK0)}, {s(SEED)}, {s(D + 2)}", f"s_mov_b32 {s(PK1)}, {s(SEED + 1)}")
        cur = list(c)   # the registers holding c0..c3 this round
        for r in range(10):
            # one v_mad_u64_u32 per product (hi:lo in an aligned pair), not a
            # mul_hi + mul_lo; the products alternate between XB..XB+3 and
            # XB+4..XB+7 so the new c1 / c3 (the products' low words) are
            # renamed instead of moved (two moves per block, not per round)
            pb = XB + 4 * (r & 1)
            lo0, hi0, lo1, hi1 = pb, pb + 1, pb + 2, pb + 3
            g(f"v_mad_u64_u32 {vr(lo0, 2)}, {sr(SX, 2)}, {v(cur[0])}, {s(PM0)}, 0",
              f"v_mad_u64_u32 {vr(lo1, 2)}, {sr(SX, 2)}, {v(cur[2])}, {s(PM1)}, 0",
              # n0 = hi1 ^ c1 ^ k0 ; n2 = hi0 ^ c3 ^ k1 ; c = (n0, lo1, n2, lo0)
              f"v_xor_b32_e32 {v(cur[0])}, {s(PK0)}, {v(hi1)}", f"v_xor_b32_e32 {v(cur[0])}, {v(cur[0])}, {v(cur[1])}",
              f"v_xor_b32_e32 {v(cur[2])}, {s(PK1)}, {v(hi0)}", f"v_xor_b32_e32 {v(cur[2])}, {v(cur[2])}, {v(cur[3])}",
              f"s_add_u32 {s(PK0)}, {s(PK0)}, 0x9E3779B9", f"s_add_u32 {s(PK1)}, {s(PK1)}, 0xBB67AE85")
            cur[1], cur[3] = lo1, lo0
        g(f"v_mov_b32_e32 {v(c[1])}, {v(cur[1])}", f"v_mov_b32_e32 {v(c[3])}, {v(cur[3])}")
    g.label("Lphx_done_%=")
    g(f"s_setpc_b64 {sr(PRET, 2)}")


CLOBBERS = (", ".join(f'"v{i}"' for i in list(range(T + 8)) + list(range(NK0, NVGPR))) + ", "
            + ", ".join(f'"s{i}"' for i in list(range(16, 99)) + [POLL, AM, AM + 1])
            + ', "vcc", "scc", "m0", "memory"')


def _inc(lines, macro):
    out = [f"#define {macro} \\"]
    for ln in lines:
        out.append(f'  "{ln}\\n" \\')
    out.append('  ""')
    return out


def render_interp() -> str:
    """csrc/mw_asm_interp.inc: the interpreter body and the assembled kernels'
    template body (csrc/mw_asmjit_shell.hip)."""
    out = ["// GENERATED by tools/gen_asm_interp.py (mythril_amd/asmgen.py) -- do not edit",
           "// (tests/test_asm_interp.py checks it is current).",
           "// Threaded-dispatch interpreter core for mw_search_asm_kernel (mw_kernels.hip) and the",
           "// template of the assembled kernels (mw_asmjit_shell.hip, mythril_amd/asmjit.py).",
           "#pragma once",
           f"#define MW_ASM_NOPS {len(ASM_OPCODES)}",
           f"#define MW_ASM_MAX_DIV {isa.ASM_MAX_DIV}u",
           "#define MW_ASM_OPCODES " + ", ".join(f"MW_{n}" for n in ASM_OPCODES),
           "#define MW_ASM_LEAF_KINDS " + ", ".join(str(k) for k in ASM_LEAF_KINDS),
           # fused handlers (isa.ASM_FUSED, mw_asm_predecode): opcode sequences
           # padded with 0xff to MW_ASM_FUSED_MAX; their offsets follow the
           # 128 opcodes' in the introspection table
           f"#define MW_ASM_NFUSED {len(isa.ASM_FUSED)}",
           f"#define MW_ASM_FUSED_MAX {isa.ASM_FUSED_MAX}",
           f"#define MW_ASM_NHANDLERS ({NTAB} + MW_ASM_NFUSED)",
           # the introspection table: bank A's handlers, bank B's, Lpc0 (lo, hi)
           "#define MW_ASM_NHTAB (2 * MW_ASM_NHANDLERS + 2)",
           f"// dispatch: {DISPATCH}",
           "#define MW_ASM_FUSED_SEQS " + ", ".join(
               "{" + ", ".join([f"MW_{n}" for n in t] + ["0xffu"] * (isa.ASM_FUSED_MAX - len(t))) + "}"
               for t in isa.ASM_FUSED)]
    out += _inc(gen("interp"), "MW_ASM_BODY")
    out += _inc(gen("template"), "MW_ASMJIT_TEMPLATE_BODY")
    out.append(f"#define MW_ASM_CLOBBERS {CLOBBERS}")
    # the narrow layout's interpreter (mw_search_asm_kernel_n): programs whose N
    # slots all lie below its NFILE; its narrow constants sit at NK_INDEX
    nv = variant("narrow")
    out.append(f"#define MW_ASM_NFILE_N {nv.NFILE}u")
    out.append(f"#define MW_ASM_NK_INDEX_N {nv.NK_INDEX}u")
    out.append(f"#define MW_ASM_NK_N {nv.NKN}u")
    out += _inc(nv.gen("interp"), "MW_ASM_BODY_N")
    out.append(f"#define MW_ASM_CLOBBERS_N {nv.CLOBBERS}")
    # the quarter layout's (mw_search_asm_kernel_q): W slots below WFILE too
    qv = variant("quarter")
    out.append(f"#define MW_ASM_WFILE_Q {qv.WFILE}u")
    out.append(f"#define MW_ASM_NFILE_Q {qv.NFILE}u")
    out.append(f"#define MW_ASM_NK_INDEX_Q {qv.NK_INDEX}u")
    out.append(f"#define MW_ASM_NK_Q {qv.NKN}u")
    out += _inc(qv.gen("interp"), "MW_ASM_BODY_Q")
    out.append(f"#define MW_ASM_CLOBBERS_Q {qv.CLOBBERS}")
    return "\n".join(out) + "\n"


_VARIANTS = {}


def variant(name: str):
    """This module built again with register layout `name` ("wide": this one)."""
    if name == _LAYOUT_NAME:
        return sys.modules[__name__]
    mod = _VARIANTS.get(name)
    if mod is None:
        import types
        mod = types.ModuleType(f"{__name__}_{name}")
        mod.__dict__["_LAYOUT_OVERRIDE"] = name
        mod.__dict__["__file__"] = __file__
        with open(__file__) as f:
            exec(compile(f.read(), __file__, "exec"), mod.__dict__)
        _VARIANTS[name] = mod
    return mod


# ======================================================== assembled kernels
# An assembled kernel is the template (gen("template")) with the program in
# place of MARKER: every instruction is its handler instantiated by StaticGen,
# whose operand access is literal.  Register operands are named directly (no
# s_set_gpr_idx), constants become instruction literals, widths and masks are
# known (canonicalisation emits only the limbs it changes), and there is no
# dispatch.  mythril_amd/asmjit.py assembles and loads the result.

KBIT = isa.KBIT


def _lit(x: int) -> str:
    x &= 0xFFFFFFFF
    return str(x) if x <= 64 else f"{x:#x}"


class StaticGen(Gen):
    """Gen for one program whose fields are known at generation time."""
    inline_leaf = False   # the body calls the template's Lleaf through LEAFADDR
    chains = False

    def __init__(self, consts, leaves=None, pool=None):
        super().__init__()
        self.consts = [int(x) for x in consts]
        self.leaves = [int(x) for x in leaves] if leaves is not None else None
        self.pool = [int(x) for x in pool] if pool is not None else None
        self.cur = {}
        self.sval = {}          # SGPR -> value this instruction set by width() / nmask()
        self.chain_open = False  # XR holds the acc of a W_CDINS chain
        self.summary_b = None    # b field whose size summary XA holds (W_CDINS)
        self.digit_spec = None   # pool digit spec whose digit T+6 holds

    def L(self, base):          # distinct from the template's labels
        self.n += 1
        return f"LS{base}{self.n}_%="

    def set_insn(self, words):
        w0, w1, w2, w3 = (int(x) & 0xFFFFFFFF for x in words)
        self.cur = {"op": w0 & 0xFF, "flags": (w0 >> 8) & 0xFF, "w": w0 >> 16, "dst": w1 & 0xFFFF,
                    "a": w1 >> 16, "b": w2 & 0xFFFF, "c": w2 >> 16, "imm": w3}
        self.sval = {}

    def _field(self, f):
        return self.cur[self.bound[f]]

    def fetch_n(self, f, dst):
        val = self._field(f)
        if val & KBIT:
            self(f"v_mov_b32_e32 {v(dst)}, {_lit(self.consts[val & 0x7FFF])}")
        else:
            self(f"v_mov_b32_e32 {v(dst)}, {v(N0 + val)}")

    def op_n(self, f, fmt, scratch, mode="SRC0"):
        val = self._field(f)
        if val & KBIT:
            self.fetch_n(f, scratch)
            self(fmt.format(a=v(scratch)))
        else:
            self(fmt.format(a=v(N0 + val)))

    def fetch_w(self, f, dst):
        val = self._field(f)
        if val & KBIT:
            o = val & 0x7FFF
            for k in range(8):
                self(f"v_mov_b32_e32 {v(dst + k)}, {_lit(self.consts[o + k])}")
        else:
            for k in range(8):
                self(f"v_mov_b32_e32 {v(dst + k)}, {v(W0 + 8 * val + k)}")

    def w_indexed(self, f, mode, emit, scratch=XA):
        val = self._field(f)
        if val & KBIT:
            self.fetch_w(f, scratch)
            emit(scratch)
        else:
            emit(W0 + 8 * val)

    def _dst(self):
        w, n = isa.decode_dst(self.cur["dst"])
        return w, n

    def write_n(self, src):
        _, n = self._dst()
        self(f"v_mov_b32_e32 {v(N0 + n)}, {v(src)}")

    def write_w(self, src):
        w, _ = self._dst()
        for k in range(8):
            self(f"v_mov_b32_e32 {v(W0 + 8 * w + k)}, {v(src + k)}")

    def width(self, dst):
        self(f"s_mov_b32 {s(dst)}, {self.cur['w']}")
        self.sval[dst] = self.cur["w"]

    def nmask(self, w, dst):
        if w in self.sval:
            m = 0xFFFFFFFF if self.sval[w] >= 32 else (1 << self.sval[w]) - 1
            self(f"s_mov_b32 {s(dst)}, {_lit(m)}")
            self.sval[dst] = m
        else:
            super().nmask(w, dst)

    def insn_mask(self, dst):
        w = self.cur["w"]
        m = 0xFFFFFFFF if w >= 32 else (1 << w) - 1
        self(f"s_mov_b32 {s(dst)}, {_lit(m)}")
        self.sval[dst] = m
        return s(dst)

    def canon(self, base, w):
        if w not in self.sval:
            super().canon(base, w)
            return
        self._canon_static(base, self.sval[w])

    def next(self):
        pass

    def static_imm(self):
        return self.cur["imm"]

    def flip_sign_bits(self, w, t):
        if w not in self.sval:
            super().flip_sign_bits(w, t)
            return
        b = self.sval[w] - 1
        q, m = b >> 5, _lit(1 << (b & 31))
        self(f"v_xor_b32_e32 {v(XA + q)}, {m}, {v(XA + q)}", f"v_xor_b32_e32 {v(XB + q)}, {m}, {v(XB + q)}")

    def bit_at(self, base, w, dst):
        if w not in self.sval:
            super().bit_at(base, w, dst)
            return
        b = self.sval[w]
        self(f"v_bfe_u32 {v(dst)}, {v(base + (b >> 5))}, {b & 31}, 1")

    def extract_limb(self, q, r):
        imm = self.cur["imm"]
        k, sh = imm >> 5, imm & 31
        hi = v(XA + k + 1) if k + 1 < 8 else "0"
        self(f"v_alignbit_b32 {v(XR)}, {hi}, {v(XA + k)}, {sh}")

    # the body sits after the template's code and may be longer than a
    # branch reaches (simm16 words): it leaves through addresses the template
    # computes once per block (gen("template"))
    def stop_if_scc1(self):
        lab = self.L("go")
        self(f"s_cbranch_scc0 {lab}", f"s_setpc_b64 {sr(STOPADDR, 2)}")
        self.label(lab)

    def all_dead_exit(self):
        """straight-line body: no live lane -> Lstop when early exit is on,
        else on with the next instruction"""
        live = self.L("lv")
        self(f"s_cbranch_scc1 {live}", f"s_bitcmp1_b32 {s(FLAGS)}, 0")
        self.stop_if_scc1()
        self.label(live)

    def call_leaf_sub(self):
        self(f"s_swappc_b64 {sr(LRET, 2)}, {sr(LEAFADDR, 2)}")

    # ------------------------------------------------------------ leaves
    def _narrow_random(self, lid, dst):
        """v(dst) = fmix64(cand ^ seed ^ lid * 0xC2B2AE3D27D4EB4F) low word
        (mw_leaf.h random_leaf, w <= 32); temporaries T..T+5, S[4], S[5], SX, PK*"""
        k = (lid * 0xC2B2AE3D27D4EB4F) & ((1 << 64) - 1)
        self(f"s_xor_b32 {s(PK0)}, {s(SEED)}, {_lit(k & 0xFFFFFFFF)}",
             f"s_xor_b32 {s(PK1)}, {s(SEED + 1)}, {_lit(k >> 32)}",
             f"v_xor_b32_e32 {v(T)}, {s(PK0)}, {v(CLO)}", f"v_xor_b32_e32 {v(T + 1)}, {s(PK1)}, {v(CHI)}")
        fmix64(self, T, T + 1, T + 2, T + 3)
        if dst != T:
            self(f"v_mov_b32_e32 {v(dst)}, {v(T)}")

    def _wide_random(self, w, lid):
        """T..T+7 = Philox4x32-10 of the candidate (the Lphilox subroutine)"""
        self(f"s_mov_b32 {s(DESC)}, {w}", f"s_mov_b32 {s(DESC + 2)}, {_lit(lid)}",
             f"s_swappc_b64 {sr(PRET, 2)}, {sr(PHILOXADDR, 2)}")
        self.digit_spec = None   # the subroutine uses T..T+7

    def _bit(self, dst, pos, first):
        src = CLO if pos < 32 else CHI
        if first:
            self(f"v_bfe_u32 {v(dst)}, {v(src)}, {pos & 31}, 1")
        else:
            self(f"v_bfe_u32 {v(T + 7)}, {v(src)}, {pos & 31}, 1")

    def leaf_digit(self, li):
        """T+6 = leaf li's pool digit (kept when the previous leaf's digit
        spec is the same: T+6 survives the gather and the random draw)"""
        w, kind, lid, shift, bits, poff, _, stride = self.leaves[8 * li: 8 * li + 8]
        if kind not in (1, 2, 3):
            return
        dig = T + 6
        spec = (kind, shift, bits, stride, lid if kind == 2 else None)
        if spec == self.digit_spec:
            pass
        elif bits == 0:
            self(f"v_mov_b32_e32 {v(dig)}, 0")
        elif kind == 1:
            if shift + bits <= 32:
                self(f"v_bfe_u32 {v(dig)}, {v(CLO)}, {shift}, {bits}")
            elif shift >= 32:
                self(f"v_bfe_u32 {v(dig)}, {v(CHI)}, {shift - 32}, {bits}")
            else:
                self(f"v_lshrrev_b64 {vr(T + 4, 2)}, {shift}, {vr(CLO, 2)}",
                     f"v_bfe_u32 {v(dig)}, {v(T + 4)}, 0, {bits}")
        elif kind == 2:
            k = (lid * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
            self(f"v_xor_b32_e32 {v(T)}, {_lit(k & 0xFFFFFFFF)}, {v(CLO)}",
                 f"v_xor_b32_e32 {v(T + 1)}, {_lit(k >> 32)}, {v(CHI)}")
            fmix64(self, T, T + 1, T + 2, T + 3)
            self(f"v_bfe_u32 {v(dig)}, {v(T)}, 0, {bits}")
        else:
            for b in range(bits):
                pos = shift + b * stride
                self._bit(dig, pos, b == 0)
                if b:
                    self(f"v_lshl_or_b32 {v(dig)}, {v(T + 7)}, {b}, {v(dig)}")
        self.digit_spec = spec

    def inline_leaf(self, li, limb0_only=False, base=XC):
        """base..base+7 (XC, or a destination slot) = leaf li's candidate value, its descriptor folded in
        (mw_leaf.h leaf_value; the asm interpreter's Lleaf subroutine).
        limb0_only: a narrow leaf whose consumer reads XC alone (the upper
        limbs are left as they are).  The pool digit stays in T+6 for the next
        leaf with the same digit (the bytes of one calldata word share it)."""
        L = self.leaves[8 * li: 8 * li + 8]
        w, kind, lid, shift, bits, poff, _, stride = L
        upper = not (limb0_only and w <= 32)
        if kind not in (1, 2, 3):
            if w <= 32:
                self._narrow_random(lid, base)
                if upper:
                    for k in range(1, 8):
                        self(f"v_mov_b32_e32 {v(base + k)}, 0")
            else:
                self._wide_random(w, lid)
                for k in range(8):
                    self(f"v_mov_b32_e32 {v(base + k)}, {v(T + k)}")
            self._canon_static(base, w)
            return
        if bits == 0 and self.pool is not None:
            # a one-entry pool: the entry is known here (mw_leaf.h leaf_value,
            # digit 0) - a constant, or the random draw on every lane
            e = self.pool[poff:poff + (1 if w < 32 else 9)]
            if w < 32:
                if e[0] & isa.POOL_NARROW_RANDOM:
                    self._narrow_random(lid, base)
                else:
                    self(f"v_mov_b32_e32 {v(base)}, {_lit(e[0])}")
                if upper:
                    for k in range(1, 8):
                        self(f"v_mov_b32_e32 {v(base + k)}, 0")
                    self._canon_static(base, w)
                else:
                    self(f"v_and_b32_e32 {v(base)}, {_lit((1 << w) - 1)}, {v(base)}")
            else:
                if e[0] & 1:
                    self._wide_random(w, lid)
                    for k in range(8):
                        self(f"v_mov_b32_e32 {v(base + k)}, {v(T + k)}")
                else:
                    for k in range(8):
                        self(f"v_mov_b32_e32 {v(base + k)}, {_lit(e[1 + k])}")
                self._canon_static(base, w)
            return
        dig = T + 6
        self.leaf_digit(li)
        # pool entry in LDS at POOLB + 4 * poff
        self(f"s_add_u32 {s(S[6])}, {s(POOLB)}, {_lit(4 * poff)}")
        rnd = self.L("lr")
        done = self.L("ld")
        if w < 32:
            self(f"v_lshl_add_u32 {v(T + 5)}, {v(dig)}, 2, {s(S[6])}", f"ds_read_b32 {v(base)}, {v(T + 5)}")
            if upper:
                for k in range(1, 8):
                    self(f"v_mov_b32_e32 {v(base + k)}, 0")
            # the random draw only when a lane's entry says RANDOM (bit 31): with
            # interleaved digits most waves pick one entry for all their lanes
            self("s_waitcnt lgkmcnt(0)", f"v_cmp_gt_i32_e32 vcc, 0, {v(base)}", "s_nop 1",
                 f"s_cbranch_vccz {done}", f"s_mov_b64 {sr(MSK, 2)}, vcc")
            self._narrow_random(lid, T)
            self(f"v_cndmask_b32_e64 {v(base)}, {v(base)}, {v(T)}, {sr(MSK, 2)}")
        else:
            self(f"v_mov_b32_e32 {v(T + 5)}, 36", f"v_mad_u32_u24 {v(T + 5)}, {v(dig)}, {v(T + 5)}, {s(S[6])}",
                 f"ds_read_b32 {v(T + 4)}, {v(T + 5)}")
            for k in range(4):
                self(f"ds_read2_b32 {vr(base + 2 * k, 2)}, {v(T + 5)} offset0:{1 + 2 * k} offset1:{2 + 2 * k}")
            self("s_waitcnt lgkmcnt(0)", f"v_and_b32_e32 {v(T + 4)}, 1, {v(T + 4)}",
                 f"v_cmp_ne_u32_e32 vcc, 0, {v(T + 4)}", "s_nop 1", f"s_cbranch_vccz {done}",
                 f"s_mov_b64 {sr(MSK, 2)}, vcc")
            self._wide_random(w, lid)
            self("s_nop 1")
            for k in range(8):
                self(f"v_cndmask_b32_e64 {v(base + k)}, {v(base + k)}, {v(T + k)}, {sr(MSK, 2)}")
        self.label(done)
        del rnd
        if upper:
            self._canon_static(base, w)
        elif w < 32:
            self(f"v_and_b32_e32 {v(base)}, {_lit((1 << w) - 1)}, {v(base)}")

    def _canon_static(self, base, wv):
        if wv >= 256:
            return
        q, r = wv >> 5, wv & 31
        for k in range(q + (1 if r else 0), 8):
            self(f"v_mov_b32_e32 {v(base + k)}, 0")
        if r:
            self(f"v_and_b32_e32 {v(base + q)}, {_lit((1 << r) - 1)}, {v(base + q)}")


def _cdins_static(g):
    """W_CDINS with literal operands (mw_interp.h MW_W_CDINS): acc | ((K[c] <s
    size) ? leaf : 0) << off; a chained link leaves the word in XR for the next"""
    cur = g.cur
    if not g.chain_open:
        g.field("a", S[0]), g.fetch_w(S[0], XR)
    o = cur["c"] & 0x7FFF                      # validated: c is a constant
    idx = g.consts[o:o + 8]
    if not any(idx[1:]) and idx[0] < 0x4000:   # i <s size  <=>  i <u summary(size)
        if g.summary_b != cur["b"]:
            g.field("b", S[2]), g.fetch_w(S[2], XB)
            g(f"v_or3_b32 {v(T)}, {v(XB + 1)}, {v(XB + 2)}, {v(XB + 3)}",
              f"v_and_b32_e32 {v(T + 1)}, 0x7fffffff, {v(XB + 7)}",
              f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 4)}, {v(XB + 5)}",
              f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 6)}, {v(T + 1)}",
              f"v_cmp_ne_u32_e32 vcc, 0, {v(T)}", "s_nop 1",
              f"v_cndmask_b32_e64 {v(XA)}, {v(XB)}, -1, vcc",
              f"v_cmp_gt_i32_e32 vcc, 0, {v(XB + 7)}", "s_nop 1",
              f"v_cndmask_b32_e64 {v(XA)}, {v(XA)}, 0, vcc")
            g.summary_b = cur["b"]
        if idx[0] <= 64:
            g(f"v_cmp_lt_u32_e64 {sr(MSK2, 2)}, {idx[0]}, {v(XA)}")
        else:
            g(f"s_mov_b32 {s(S[1])}, {idx[0]:#x}", f"v_cmp_lt_u32_e64 {sr(MSK2, 2)}, {s(S[1])}, {v(XA)}")
    else:
        g.summary_b = None
        g.field("b", S[1]), g.fetch_w(S[1], XB)
        g.field("c", S[2]), g.fetch_w(S[2], XA)
        g(f"v_xor_b32_e32 {v(XA + 7)}, 0x80000000, {v(XA + 7)}", f"v_xor_b32_e32 {v(XB + 7)}, 0x80000000, {v(XB + 7)}")
        g.sub_chain(XA, XB)
        g(f"s_mov_b64 {sr(MSK2, 2)}, vcc")
    skip = g.L("cdns")
    g.leaf_digit(cur["imm"] & 0xFFFF)     # before the skip: T+6 then holds it either way
    g("s_nop 1", f"s_cmp_eq_u64 {sr(MSK2, 2)}, 0", f"s_cbranch_scc1 {skip}")
    g.inline_leaf(cur["imm"] & 0xFFFF, limb0_only=True)
    g(f"v_cndmask_b32_e64 {v(T)}, 0, {v(XC)}, {sr(MSK2, 2)}")
    off = cur["imm"] >> 16
    q, bit = off >> 5, off & 31
    g(f"v_lshl_or_b32 {v(XR + q)}, {v(T)}, {bit}, {v(XR + q)}")
    if bit > 24 and q + 1 < 8:   # a byte straddling a limb boundary
        g(f"v_lshrrev_b32_e32 {v(T)}, {32 - bit}, {v(T)}", f"v_or_b32_e32 {v(XR + q + 1)}, {v(T)}, {v(XR + q + 1)}")
    g.label(skip)
    g.width(S[2]), g.canon(XR, S[2])
    if cur["flags"] & 1:          # MW_FLAG_CHAIN: the next W_CDINS reads XR as its acc
        g.chain_open = True
    else:
        g.chain_open = False
        g.write_w(XR)


_IMM_REG = re.compile(rf"\bs{CUR + 3}\b")


CDINS_BATCH = 8   # gathers in flight per batch (XB..XB+7 addresses, XC..XC+7 values)


def _batchable(g, insn) -> bool:
    """A W_CDINS link the batched emission handles: a small immediate index
    and a pooled narrow leaf."""
    o = (insn[2] >> 16) & 0x7FFF
    idx = g.consts[o:o + 8]
    L = g.leaves[8 * (insn[3] & 0xFFFF): 8 * (insn[3] & 0xFFFF) + 8]
    return (not any(idx[1:]) and idx[0] < 0x4000 and L[0] < 32 and L[1] in (1, 2, 3))


def _cdins_chain_static(g, links):
    """A chain of W_CDINS links (MW_FLAG_CHAIN on all but the last) building one
    word, emitted as batches: every link's pool gather issued before one wait,
    then the random draws (only when some lane's entry says RANDOM), the range
    selects and the inserts.  The per-link form waits for each gather and each
    branch condition in turn (latency-bound)."""
    g.set_insn(links[0])
    g.field("a", S[0]), g.fetch_w(S[0], XR)
    for start in range(0, len(links), CDINS_BATCH):
        batch = links[start:start + CDINS_BATCH]
        for k, insn in enumerate(batch):
            g.set_insn(insn)
            if g.summary_b != g.cur["b"]:     # size summary (mw: i <s size <=> i <u XA)
                g.field("b", S[2]), g.fetch_w(S[2], XB)
                g(f"v_or3_b32 {v(T)}, {v(XB + 1)}, {v(XB + 2)}, {v(XB + 3)}",
                  f"v_and_b32_e32 {v(T + 1)}, 0x7fffffff, {v(XB + 7)}",
                  f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 4)}, {v(XB + 5)}",
                  f"v_or3_b32 {v(T)}, {v(T)}, {v(XB + 6)}, {v(T + 1)}",
                  f"v_cmp_ne_u32_e32 vcc, 0, {v(T)}", "s_nop 1",
                  f"v_cndmask_b32_e64 {v(XA)}, {v(XB)}, -1, vcc",
                  f"v_cmp_gt_i32_e32 vcc, 0, {v(XB + 7)}", "s_nop 1",
                  f"v_cndmask_b32_e64 {v(XA)}, {v(XA)}, 0, vcc")
                g.summary_b = g.cur["b"]
        for k, insn in enumerate(batch):      # addresses and gathers
            li = insn[3] & 0xFFFF
            g.leaf_digit(li)
            poff = g.leaves[8 * li + 5]
            g(f"s_add_u32 {s(S[6])}, {s(POOLB)}, {_lit(4 * poff)}",
              f"v_lshl_add_u32 {v(XB + k)}, {v(T + 6)}, 2, {s(S[6])}", f"ds_read_b32 {v(XC + k)}, {v(XB + k)}")
        g("s_waitcnt lgkmcnt(0)")
        # random draws: only when some lane's entry in the batch says RANDOM (bit 31)
        done = g.L("cbr")
        n = len(batch)
        acc = [XC + k for k in range(n)]
        g(f"v_or_b32_e32 {v(XB)}, {v(acc[0])}, {v(acc[0])}")
        for k in range(1, n):
            g(f"v_or_b32_e32 {v(XB)}, {v(XB)}, {v(acc[k])}")
        g(f"v_cmp_gt_i32_e32 vcc, 0, {v(XB)}", "s_nop 1", f"s_cbranch_vccz {done}")
        for k, insn in enumerate(batch):
            lid = g.leaves[8 * (insn[3] & 0xFFFF) + 2]
            g(f"v_cmp_gt_i32_e64 {sr(MSK, 2)}, 0, {v(XC + k)}")
            g._narrow_random(lid, T)
            g(f"v_cndmask_b32_e64 {v(XC + k)}, {v(XC + k)}, {v(T)}, {sr(MSK, 2)}")
        g.label(done)
        for k, insn in enumerate(batch):      # mask, range select, insert
            g.set_insn(insn)
            li = insn[3] & 0xFFFF
            w = g.leaves[8 * li]
            i = g.consts[(insn[2] >> 16) & 0x7FFF]
            g(f"v_and_b32_e32 {v(XC + k)}, {_lit((1 << w) - 1)}, {v(XC + k)}")
            if i <= 64:
                g(f"v_cmp_lt_u32_e64 {sr(MSK2, 2)}, {i}, {v(XA)}")
            else:
                g(f"s_mov_b32 {s(S[1])}, {i:#x}", f"v_cmp_lt_u32_e64 {sr(MSK2, 2)}, {s(S[1])}, {v(XA)}")
            g("s_nop 1", f"v_cndmask_b32_e64 {v(T)}, 0, {v(XC + k)}, {sr(MSK2, 2)}")
            off = insn[3] >> 16
            q, bit = off >> 5, off & 31
            g(f"v_lshl_or_b32 {v(XR + q)}, {v(T)}, {bit}, {v(XR + q)}")
            if bit > 24 and q + 1 < 8:
                g(f"v_lshrrev_b32_e32 {v(T)}, {32 - bit}, {v(T)}",
                  f"v_or_b32_e32 {v(XR + q + 1)}, {v(T)}, {v(XR + q + 1)}")
            w_word = g.cur["w"]
            if w_word < 256 and g.cur["flags"] & 1:   # a chained link canonicalises its word
                g._canon_static(XR, w_word)
    g.set_insn(links[-1])
    g._canon_static(XR, g.cur["w"])
    g.chain_open = False
    g.write_w(XR)


CHECK_OPS = ("CHECK", "CHECK_IMP", "CHECK_IMPEQ", "CHECK_IMPEQK")
ACC = JMP   # s[92:93]: a check run's lane mask (free in a static body)
CMSK, CMSK2 = S[0], S[2]   # s[72:73], s[74:75]: a check's consequence mask (scratch in a static body)


def _nsrc(g, f):
    """an N operand as a VOPC src0: its register, or its constant as a literal"""
    if f & KBIT:
        return _lit(g.consts[f & 0x7FFF])
    return v(N0 + f)


def _nreg(g, f, tmp):
    """an N operand in a VGPR (constants moved into tmp)"""
    if f & KBIT:
        g(f"v_mov_b32_e32 {v(tmp)}, {_lit(g.consts[f & 0x7FFF])}")
        return v(tmp)
    return v(N0 + f)


def _check_run_static(g, run):
    """A run of CHECK / CHECK_IMP / CHECK_IMPEQ(K) as one lane mask: each check's
    condition is formed in SGPRs (premise false OR consequence), ANDed into
    ACC, and ALIVE and the early-exit test are updated once at the end of the
    run.  The SALU combine of check k is emitted after check k+1's compares,
    so no VALU-written SGPR is read by the next instruction.  Each check
    writes its own pair of mask pairs (premise, consequence), alternating
    between two sets: the consequence must not go through vcc, which the next
    check's compare would overwrite before the deferred combine reads it."""
    g(f"s_mov_b64 {sr(ACC, 2)}, -1")
    pending = None
    for insn in run:
        g.set_insn(insn)
        op = insn[0] & 0xFF
        a, b, c = g.cur["a"], g.cur["b"], g.cur["c"]
        m, mc = (MSK, CMSK) if pending != MSK else (MSK2, CMSK2)   # alternate the mask pairs
        if op == isa.OPCODES["CHECK"]:
            g(f"v_cmp_ne_u32_e64 {sr(m, 2)}, 0, {_nreg(g, a, T)}")
            combine = [f"s_and_b64 {sr(ACC, 2)}, {sr(ACC, 2)}, {sr(m, 2)}"]
        else:
            if op == isa.OPCODES["CHECK_IMPEQK"]:   # premise a = imm (VOP3 takes no literal)
                g(f"v_mov_b32_e32 {v(T + 3)}, {_lit(insn[3])}",
                  f"v_cmp_ne_u32_e64 {sr(m, 2)}, {v(T + 3)}, {_nreg(g, a, T)}")
            else:
                g(f"v_cmp_eq_u32_e64 {sr(m, 2)}, 0, {_nreg(g, a, T)}")
            if op == isa.OPCODES["CHECK_IMP"]:
                g(f"v_cmp_ne_u32_e64 {sr(mc, 2)}, 0, {_nreg(g, b, T + 1)}")
            else:
                g(f"v_cmp_eq_u32_e64 {sr(mc, 2)}, {_nreg(g, b, T + 2)}, {_nreg(g, c, T + 1)}")   # VOP3: no literal
            combine = [f"s_or_b64 {sr(m, 2)}, {sr(mc, 2)}, {sr(m, 2)}",
                       f"s_and_b64 {sr(ACC, 2)}, {sr(ACC, 2)}, {sr(m, 2)}"]
        if pending is not None:
            g(*pending_lines)
        pending, pending_lines = m, combine
    g("s_nop 1")
    g(*pending_lines)
    g(f"s_and_b64 {sr(AM, 2)}, {sr(AM, 2)}, {sr(ACC, 2)}")
    g.all_dead_exit()


LDS_SPILL_WORDS = 80   # mw_kernels.hip kLdsSpillWords


def lds_spill_words(n_spill: int, npool: int) -> int:
    """Spill words an assembled kernel keeps in LDS: mw_kernels.hip
    asm_lds_fit (the pool first, the hottest spill words in what is left)."""
    rows = (npool * 4 + 1023) // 1024
    return max(0, min(n_spill, LDS_SPILL_WORDS - rows))


def _grid_static(g, insn, nlds):
    """A CHECK_GRID row in an assembled body (no exec writes there): the
    lanes out of range read the table's first word instead (j clamped to 0),
    and with the table split between LDS and the global buffer every lane
    reads both places at clamped words and selects (nlds None: the kernel's
    NLDS register; only for text, asmjit passes nlds)."""
    g.set_insn(insn)
    c = g.cur["c"]
    t0, nm1 = c & 1023, (c >> 10) & 31
    key = _nreg(g, g.cur["a"], T + 4)
    skip = g.L("gs")
    g(f"v_sub_u32_e32 {v(T)}, {_lit(insn[3])}, {key}", f"v_cmp_ge_u32_e32 vcc, {nm1}, {v(T)}",
      f"s_and_b64 {sr(CMSK, 2)}, vcc, {sr(AM, 2)}", f"s_cbranch_scc0 {skip}",
      f"v_cndmask_b32_e32 {v(T)}, 0, {v(T)}, vcc")
    if nlds is not None and t0 + nm1 + 1 <= nlds:        # the whole table in LDS
        g(f"v_lshlrev_b32_e32 {v(T + 2)}, 10, {v(T)}", f"v_add_u32_e32 {v(T + 2)}, {v(T + 2)}, {v(LDSOFF)}")
        if t0 * 1024 < 65536:
            g(f"ds_read_b32 {v(T + 3)}, {v(T + 2)} offset:{t0 * 1024}")
        else:
            g(f"v_add_u32_e32 {v(T + 2)}, {_lit(t0 * 1024)}, {v(T + 2)}", f"ds_read_b32 {v(T + 3)}, {v(T + 2)}")
    elif nlds is not None and t0 >= nlds:                 # the whole table in the global buffer
        g(f"v_add_u32_e32 {v(T + 2)}, {_lit(t0 - nlds)}, {v(T)}",
          f"v_mul_lo_u32 {v(T + 2)}, {v(T + 2)}, {s(GSTRIDE)}", f"v_add_u32_e32 {v(T + 2)}, {v(T + 2)}, {v(GOFF)}",
          f"global_load_dword {v(T + 3)}, {v(T + 2)}, {sr(GSP, 2)}")
    else:
        nl = _lit(nlds) if nlds is not None else s(NLDS)
        g(f"v_add_u32_e32 {v(T + 1)}, {_lit(t0)}, {v(T)}",                 # the word
          f"v_cmp_gt_u32_e64 {sr(CMSK2, 2)}, {nl}, {v(T + 1)}",            # lanes whose word is in LDS
          f"v_cndmask_b32_e64 {v(T + 2)}, 0, {v(T + 1)}, {sr(CMSK2, 2)}",
          f"v_lshlrev_b32_e32 {v(T + 2)}, 10, {v(T + 2)}", f"v_add_u32_e32 {v(T + 2)}, {v(T + 2)}, {v(LDSOFF)}",
          f"ds_read_b32 {v(T + 3)}, {v(T + 2)}",
          f"v_subrev_u32_e32 {v(T + 5)}, {nl}, {v(T + 1)}",
          f"v_cndmask_b32_e64 {v(T + 5)}, {v(T + 5)}, 0, {sr(CMSK2, 2)}",
          f"v_mul_lo_u32 {v(T + 5)}, {v(T + 5)}, {s(GSTRIDE)}", f"v_add_u32_e32 {v(T + 5)}, {v(T + 5)}, {v(GOFF)}",
          f"global_load_dword {v(T + 5)}, {v(T + 5)}, {sr(GSP, 2)}",
          "s_waitcnt vmcnt(0) lgkmcnt(0)",
          f"v_cndmask_b32_e64 {v(T + 3)}, {v(T + 5)}, {v(T + 3)}, {sr(CMSK2, 2)}")
    g("s_waitcnt vmcnt(0) lgkmcnt(0)")
    g(f"v_cmp_ne_u32_e64 {sr(CMSK2, 2)}, {_nreg(g, g.cur['b'], T + 5)}, {v(T + 3)}",
      f"s_and_b64 {sr(CMSK2, 2)}, {sr(CMSK2, 2)}, {sr(CMSK, 2)}",
      f"s_andn2_b64 {sr(AM, 2)}, {sr(AM, 2)}, {sr(CMSK2, 2)}")
    g.all_dead_exit()
    g.label(skip)


def _spill_static(g, name, insn, nlds):
    """SPILL/FILL with the word's place known: LDS [word][lane] below nlds,
    else the global buffer [word][thread] (mw_kernels.hip)."""
    wd0 = insn[3]
    n = 8 if name.endswith("_W") else 1
    g.set_insn(insn)

    def addr(word):
        if word < nlds:
            if word * 1024 < 65536:
                return "lds", v(LDSOFF), f" offset:{word * 1024}"
            g(f"v_add_u32_e32 {v(T + 7)}, {_lit(word * 1024)}, {v(LDSOFF)}")
            return "lds", v(T + 7), ""
        g(f"s_mul_i32 {s(S[7])}, {s(GSTRIDE)}, {word - nlds}", f"v_add_u32_e32 {v(T + 7)}, {s(S[7])}, {v(GOFF)}")
        return "glob", v(T + 7), ""

    if name.startswith("SPILL"):
        a = g.cur["a"]
        if a & KBIT:
            o = a & 0x7FFF
            for k in range(n):
                g(f"v_mov_b32_e32 {v(XA + k)}, {_lit(g.consts[o + k])}")
            src = [v(XA + k) for k in range(n)]
        else:
            src = [v(W0 + 8 * a + k) for k in range(n)] if n == 8 else [v(N0 + a)]
        for k in range(n):
            kind, base, off = addr(wd0 + k)
            if kind == "lds":
                g(f"ds_write_b32 {base}, {src[k]}{off}")
            else:
                g(f"global_store_dword {base}, {src[k]}, {sr(GSP, 2)}")
        # no wait: LDS operations of a wave execute in order, and the fill waits
        # for its own loads (the global store is waited for below)
        if any(wd0 + k >= nlds for k in range(n)):
            g("s_waitcnt vmcnt(0)")
    else:
        for k in range(n):
            kind, base, off = addr(wd0 + k)
            if kind == "lds":
                g(f"ds_read_b32 {v(XR + k)}, {base}{off}")
            else:
                g(f"global_load_dword {v(XR + k)}, {base}, {sr(GSP, 2)}")
        g("s_waitcnt vmcnt(0) lgkmcnt(0)")
        (g.write_w if n == 8 else g.write_n)(XR)


def static_body(code, consts, leaves, forward: bool = True, nlds: int = None, pool=None) -> list:
    """The straight-line body of an assembled kernel for a validated,
    asm-eligible program (code: its instruction words, original encoding;
    consts and leaves: its constant pool and leaf table; pool: its candidate
    pool words, which lets one-entry pools fold to constants)."""
    g = StaticGen(consts, leaves, pool)
    names = {c: n for n, c in isa.OPCODES.items()}
    words = [int(x) for x in code]
    out = []
    cdins = isa.OPCODES["W_CDINS"]
    skip_to = 0
    for i in range(0, len(words), 4):
        if i < skip_to:
            continue
        insn = words[i:i + 4]
        name = names[insn[0] & 0xFF]
        if name == "END":
            break
        g.set_insn(insn)
        g.lines = []
        if name in CHECK_OPS:
            run = []
            j = i
            while j + 4 <= len(words) and names[words[j] & 0xFF] in CHECK_OPS:
                run.append(words[j:j + 4])
                j += 4
            g.chain_open = False
            g.summary_b = None
            g.digit_spec = None
            _check_run_static(g, run)
            skip_to = j
            name = f"{name} run x{len(run)}"
        elif name == "W_CDINS" and not g.chain_open:
            # a whole chain, batched, when every link qualifies
            j = i
            links = []
            while True:
                ln_ = words[j:j + 4]
                links.append(ln_)
                if not ((ln_[0] >> 8) & 1) or j + 4 >= len(words) or (words[j + 4] & 0xFF) != cdins:
                    break
                j += 4
            if (len(links) > 1 and all(_batchable(g, x) for x in links) and not ((links[-1][0] >> 8) & 1)
                    and len({x[2] & 0xFFFF for x in links}) == 1):   # one size operand: one summary
                _cdins_chain_static(g, links)
                skip_to = j + 4
                name = f"W_CDINS x{len(links)}"
            else:
                g.set_insn(insn)
                _cdins_static(g)
        elif name == "W_CDINS":
            _cdins_static(g)
        elif name == "CHECK_GRID":
            g.chain_open = False
            g.summary_b = None
            g.digit_spec = None
            _grid_static(g, insn, nlds)
        elif name in ("SPILL_W", "SPILL_N", "FILL_W", "FILL_N") and nlds is not None:
            g.chain_open = False
            g.summary_b = None
            g.digit_spec = None
            _spill_static(g, name, insn, nlds)
        elif name in ("LEAF_W", "LEAF_N"):
            g.chain_open = False
            g.summary_b = None
            if name == "LEAF_W":   # straight into the destination slot: no copy
                g.inline_leaf(insn[3], base=W0 + 8 * g._dst()[0])
            else:
                g.inline_leaf(insn[3], limb0_only=True)
                g.write_n(XC)
        else:
            g.chain_open = False
            g.summary_b = None
            g.digit_spec = None
            HANDLERS[name](g)
        lines = g.lines
        if any(_IMM_REG.search(ln) for ln in lines):   # the handler reads the immediate word
            lines = [f"s_mov_b32 {s(CUR + 3)}, {_lit(insn[3])}"] + lines
        out.append(f"; {i // 4}: {name}")
        out.extend(lines)
    out.append(f"s_setpc_b64 {sr(ENDADDR, 2)}")
    if forward:
        out = forward_copies(const_fold(out))
    out, live_in = dead_code(out)
    # the files start at zero (mw_interp.h): only what the body reads before writing
    zero = sorted(r for r in live_in if r < 128)
    head, k = [], 0
    while k < len(zero):
        r = zero[k]
        if r % 2 == 0 and k + 1 < len(zero) and zero[k + 1] == r + 1:
            head.append(f"v_mov_b64 {vr(r, 2)}, 0")
            k += 2
        else:
            head.append(f"v_mov_b32_e32 {v(r)}, 0")
            k += 1
    return head + out


# ------------------------------------------------ copy forwarding (static bodies)
_VREG = re.compile(r"^v(\d+)$")
_VRANGE = re.compile(r"^v\[(\d+):(\d+)\]$")
TEMP_LO = XA   # v136..v191: operand, result and scratch registers; v0..v127 are the files


def _operands(line: str):
    parts = line.split(None, 1)
    if len(parts) == 1:
        return parts[0], []
    return parts[0], [o.strip() for o in parts[1].split(",")]


def _regs(tok: str):
    """VGPR numbers an operand names (first word of the operand only)"""
    t = tok.split()[0] if tok else ""
    m = _VREG.match(t)
    if m:
        return [int(m.group(1))]
    m = _VRANGE.match(t)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def forward_copies(lines):
    """Peephole over a straight-line body: a read of a register that is a
    plain copy (v_mov_b32 vD, vS) of another reads the source instead, and a
    copy into a scratch register (>= v136) whose value is then overwritten
    before any other read is dropped.  Conservative: labels, branches, calls
    and register-indexing regions end every copy's scope, and multi-register
    operands are never rewritten."""
    out = list(lines)
    dead = set()
    alias = {}     # D -> S
    pending = {}   # D -> index of the copy into scratch register D
    indexed = False

    def clobber(r):
        if r in pending:
            dead.add(pending.pop(r))
        alias.pop(r, None)
        for d in [d for d, src in alias.items() if src == r]:
            del alias[d]
            pending.pop(d, None)   # read later in its own name: keep that copy

    for i, ln in enumerate(out):
        if not ln or ln.startswith(";"):
            continue
        op, ops = _operands(ln)
        if op == "s_set_gpr_idx_on":
            indexed = True
        barrier = (ln.endswith(":") or indexed or op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc",
                                                                    "s_call", "s_set_gpr_idx")))
        if op == "s_set_gpr_idx_off":
            indexed = False
        if barrier:
            alias.clear()
            pending.clear()
            continue
        if not op.startswith(("v_", "ds_", "global_", "buffer_")):
            continue
        if op.startswith(("ds_write", "global_store", "global_atomic", "buffer_store")):
            dst_n, srcs = 0, ops
        elif op.startswith("v_cmp"):
            dst_n, srcs = 0, ops[1:]          # writes vcc / an SGPR pair
        else:
            dst_n, srcs = 1, ops[1:]
        dsts = _regs(ops[0]) if dst_n and ops else []
        new_srcs = []
        for o in srcs:
            rs = _regs(o)
            if len(rs) == 1 and rs[0] in alias and o.split()[0] == f"v{rs[0]}":
                o = o.replace(f"v{rs[0]}", f"v{alias[rs[0]]}", 1)
            else:
                for r in rs:                   # read in its own name: that copy stays
                    pending.pop(r, None)
            new_srcs.append(o)
        if new_srcs != srcs:
            ln = op + " " + ", ".join(([ops[0]] if dst_n or op.startswith("v_cmp") else []) + new_srcs)
            out[i] = ln
        for r in dsts:
            clobber(r)
        if op == "v_mov_b32_e32" and dsts and len(new_srcs) == 1:
            s_regs = _regs(new_srcs[0])
            d = dsts[0]
            if len(s_regs) == 1 and new_srcs[0] == f"v{s_regs[0]}":
                if s_regs[0] == d:
                    dead.add(i)
                else:
                    alias[d] = s_regs[0]
                    if d >= TEMP_LO:
                        pending[d] = i
    return [ln for i, ln in enumerate(out) if i not in dead]


# ------------------------------------------------ constant operands (static bodies)
_INT = re.compile(r"^-?(0x[0-9a-fA-F]+|\d+)$")
_COMMUTE = {"v_xor_b32_e32", "v_or_b32_e32", "v_and_b32_e32", "v_add_u32_e32", "v_add_co_u32_e32",
            "v_addc_co_u32_e32"}
_REVERSE = {"v_sub_co_u32_e32": "v_subrev_co_u32_e32", "v_subb_co_u32_e32": "v_subbrev_co_u32_e32",
            "v_sub_u32_e32": "v_subrev_u32_e32"}
_CMP_SWAP = {"eq": "eq", "ne": "ne", "lt": "gt", "gt": "lt", "le": "ge", "ge": "le"}
_FOLD = {"v_xor_b32_e32": lambda a, b: a ^ b, "v_or_b32_e32": lambda a, b: a | b,
         "v_and_b32_e32": lambda a, b: a & b, "v_add_u32_e32": lambda a, b: a + b}


def _imm(tok):
    t = tok.strip()
    if not _INT.match(t):
        return None
    return int(t, 0) & 0xFFFFFFFF


def _inline(x):
    """gfx9 inline integer constant (VOP3 operands take no literal)"""
    return x <= 64 or x >= 0xFFFFFFF0


def const_fold(lines):
    """Peephole over a straight-line body: a VGPR loaded with a constant
    (v_mov_b32 vX, imm - the static handlers' constant operands) is read as
    that constant where the encoding allows: a VOP2 / VOPC src0 literal
    (operands swapped or the reversed form used when the constant is src1),
    an inline constant anywhere; operations on two constants fold and
    identities (x ^ 0, x | 0, x & -1, x + 0) become copies.  The loads then
    die (dead_code).  Labels, branches and calls end every constant's scope."""
    out = list(lines)
    const = {}
    for i, ln in enumerate(out):
        if not ln or ln.startswith(";"):
            continue
        op, ops = _operands(ln)
        if (ln.endswith(":") or op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_call",
                                               "s_set_gpr_idx")) or "exec" in ln):
            const.clear()
            continue
        if not op.startswith(("v_", "ds_", "global_", "buffer_")):
            continue
        cv = lambda t: const.get(_regs(t)[0]) if (len(_regs(t)) == 1 and t == f"v{_regs(t)[0]}") else None  # noqa
        new = None
        if op == "v_mov_b32_e32" and len(ops) == 2 and cv(ops[1]) is not None:   # a copy of a constant
            new = f"v_mov_b32_e32 {ops[0]}, {_lit(cv(ops[1]))}"
        elif op in _COMMUTE or op in _REVERSE:
            k = 2 if op.endswith("co_u32_e32") else 1          # src0's index (after dst[, vcc])
            s0, s1 = ops[k], ops[k + 1]
            c0, c1 = cv(s0) if _imm(s0) is None else _imm(s0), cv(s1)
            # the constant bus: a carry-in (vcc) leaves no room for a literal, and
            # src1 of a VOP2 must stay a VGPR
            carry_in = op in ("v_addc_co_u32_e32", "v_subb_co_u32_e32")
            if c1 is not None and (not _regs(s0) or (carry_in and not _inline(c1))):
                c1 = None
            if c0 is not None and carry_in and not _inline(c0):
                c0 = None if _imm(s0) is None else c0
            if op in _FOLD and c0 is not None and c1 is not None:
                new = f"v_mov_b32_e32 {ops[0]}, {_lit(_FOLD[op](c0, c1))}"
            elif c1 is not None and c0 is None:
                if op in _FOLD and ((c1 == 0 and op != "v_and_b32_e32") or (c1 == 0xFFFFFFFF and op == "v_and_b32_e32")):
                    new = f"v_mov_b32_e32 {ops[0]}, {s0}"
                elif op == "v_and_b32_e32" and c1 == 0:
                    new = f"v_mov_b32_e32 {ops[0]}, 0"
                elif op in _COMMUTE:
                    rest = ops[k + 2:]
                    new = f"{op} " + ", ".join(ops[:k] + [_lit(c1), s0] + rest)
                elif op in _REVERSE:
                    rest = ops[k + 2:]
                    new = f"{_REVERSE[op]} " + ", ".join(ops[:k] + [_lit(c1), s0] + rest)
            elif c0 is not None and _imm(s0) is None:
                if op in _FOLD and ((c0 == 0 and op != "v_and_b32_e32") or (c0 == 0xFFFFFFFF and op == "v_and_b32_e32")):
                    new = f"v_mov_b32_e32 {ops[0]}, {s1}"
                elif op == "v_and_b32_e32" and c0 == 0:
                    new = f"v_mov_b32_e32 {ops[0]}, 0"
                else:
                    new = f"{op} " + ", ".join(ops[:k] + [_lit(c0)] + ops[k + 1:])
        elif op.startswith("v_cmp_") and op.endswith("_e32") and len(ops) == 3:
            s0, s1 = ops[1], ops[2]
            c0, c1 = (cv(s0) if _imm(s0) is None else None), cv(s1)
            parts = op.split("_")     # v cmp <cc> <type> e32
            if c1 is not None and _imm(s0) is None and c0 is None and parts[2] in _CMP_SWAP and _regs(s0):
                parts[2] = _CMP_SWAP[parts[2]]
                new = "_".join(parts) + f" {ops[0]}, {_lit(c1)}, {s0}"
            elif c0 is not None:
                new = f"{op} {ops[0]}, {_lit(c0)}, {s1}"
        elif op.startswith(("v_cndmask_b32_e64", "v_or3_b32", "v_add3_u32", "v_lshl_or_b32", "v_alignbit_b32",
                            "v_bfe_u32", "v_mad_u32_u24", "v_lshl_add_u32")):
            srcs = []
            changed = False
            for t in ops[1:]:
                c = cv(t)
                if c is not None and _inline(c):
                    srcs.append(_lit(c))
                    changed = True
                else:
                    srcs.append(t)
            if changed:
                new = f"{op} " + ", ".join([ops[0]] + srcs)
        if new is not None:
            out[i] = new
            op, ops = _operands(new)
        defs, _ = _defs_uses(op, ops)
        for d in defs:
            const.pop(d, None)
        if op == "v_mov_b32_e32" and len(ops) == 2 and _imm(ops[1]) is not None and len(defs) == 1:
            const[defs[0]] = _imm(ops[1])
    return out


# ------------------------------------------------ dead-code elimination (static bodies)
# Registers a static body may leave dead: the W and N files and the operand /
# result / scratch registers.  v128..v135 and v144..v151 (zeroed once per
# block) and v160..v167 (candidate, alive, offsets) are the template's and are
# live wherever the body leaves.
DCE_REGS = frozenset(range(0, 128)) | frozenset(range(XA, XA + 8)) | frozenset(range(XB, XB + 8)) \
    | frozenset(range(XR, T + 8))
_ALL_V = frozenset(range(256))
EXIT_LIVE = _ALL_V - DCE_REGS
_PHILOX_DEFS = frozenset(range(T, T + 8))
# VALU forms with no effect besides their VGPR result (no vcc / SGPR write)
_PURE = ("v_mov_b32", "v_mov_b32_e32", "v_mov_b32_e64", "v_mov_b64", "v_cndmask_b32_e32", "v_cndmask_b32_e64",
         "v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32", "v_or3_b32", "v_lshl_or_b32", "v_bfe_u32",
         "v_lshrrev_b32_e32", "v_lshlrev_b32_e32", "v_add_u32_e32", "v_sub_u32_e32", "v_not_b32_e32",
         "v_add3_u32", "v_alignbit_b32", "v_lshl_add_u32", "v_mul_lo_u32", "v_mad_u32_u24")
_LABEL_REF = re.compile(r"\b(L\w+_%=|L\w+_\d+)$")


def _defs_uses(op, ops):
    """(VGPRs written, VGPRs read) of one instruction; None when unknown"""
    regs = [_regs(o) for o in ops]
    if op.startswith(("ds_write", "global_store", "global_atomic", "buffer_store")):
        return [], [r for rs in regs for r in rs]
    if op.startswith("v_cmp"):
        return [], [r for rs in regs[1:] for r in rs]
    if op.startswith(("v_readfirstlane", "v_readlane")):
        return [], [r for rs in regs[1:] for r in rs]
    if op.startswith("v_writelane"):
        return regs[0], [r for rs in regs for r in rs]     # a partial write: the old value stays live
    if op.startswith(("v_", "ds_read", "global_load", "buffer_load")):
        return (regs[0] if ops else []), [r for rs in regs[1:] for r in rs]
    return [], []


def dead_code(lines):
    """Backward liveness over a straight-line body with forward skips: pure
    VALU instructions whose result no later instruction reads are dropped.
    Returns (lines, live_in), live_in being the body registers read before
    any write (the body zeroes those itself).  Exits (s_setpc) leave only the
    template's registers live; calls keep every register from v128 up live;
    an instruction inside an s_set_gpr_idx region reads everything."""
    live = set(EXIT_LIVE)
    at_label = {}
    keep = [True] * len(lines)
    indexed = False
    for i in range(len(lines) - 1, -1, -1):
        ln = lines[i]
        if not ln or ln.startswith(";"):
            continue
        if ln.endswith(":"):
            at_label[ln[:-1]] = set(live)
            continue
        op, ops = _operands(ln)
        if "exec" in ln:
            raise ValueError("dead_code: a body that writes exec")
        if op == "s_set_gpr_idx_off":
            indexed = True            # walking backwards: the region starts here
            live = set(_ALL_V)
            continue
        if op == "s_set_gpr_idx_on":
            indexed = False
            live = set(_ALL_V)
            continue
        if indexed:
            live = set(_ALL_V)
            continue
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = ops[0] if ops else ""
            out = at_label.get(tgt)
            if out is None:
                out = _ALL_V
            live = set(out) if op == "s_branch" else live | out
            continue
        if op == "s_setpc_b64":
            live = set(EXIT_LIVE)
            continue
        if op == "s_swappc_b64" and ops[1:] == [sr(PHILOXADDR, 2)]:
            # Lphilox (philox_sub): writes T..T+7 on every path, reads the
            # candidate index (CLO, CHI) and the template's registers
            live.difference_update(_PHILOX_DEFS)
            live |= EXIT_LIVE
            continue
        if op.startswith(("s_swappc", "s_call")):
            live |= _ALL_V - frozenset(range(0, 128))
            continue
        if not op.startswith(("v_", "ds_", "global_", "buffer_")):
            continue
        defs, uses = _defs_uses(op, ops)
        if op in _PURE and defs and all(d in DCE_REGS and d not in live for d in defs):
            keep[i] = False
            continue
        live.difference_update(defs)
        live.update(uses)
    live_in = sorted(r for r in live if r in DCE_REGS)
    return [ln for ln, k in zip(lines, keep) if k], live_in
