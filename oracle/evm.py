"""ORACLE (test infrastructure only): minimal concrete EVM that builds DAG terms.

Used only to turn the reference's VMTests (``tests/laser/evm_testsuite/VMTests``,
harness ``tests/laser/evm_testsuite/evm_test.py:110-189``) into known-answer
tests for the DAG semantics.  Each EVM opcode is lowered onto SMT terms the way
``mythril/laser/ethereum/instructions.py`` lowers it, e.g.

  ADD/SUB/MUL  ``:457-502``  bvadd/bvsub/bvmul on ``util.pop_bitvec`` (Bool -> If(b,1,0), util.py:67-88)
  DIV          ``:504-517``  concrete-0 divisor -> 0 else UDiv
  SDIV         ``:519-532``  concrete-0 divisor -> 0 else ``/`` (bvsdiv)
  MOD / SMOD   ``:534-545, 572-583`` URem / SRem
  SHL/SHR/SAR  ``:547-570``  bvshl / LShR / ``>>`` (bvashr)
  ADDMOD/MULMOD ``:585-612`` URem(URem(a,n) op URem(b,n), n)
  EXP          ``:622-636``  concrete pow mod 2**256 (exponent_function_manager.py:39-49)
  SIGNEXTEND   ``:638-665``  If(s0 <= 31 (signed), If(bit set, s1 | -bit, s1 & (bit-1)), s1)
  LT/GT/SLT/SGT/EQ/ISZERO ``:668-759``; AND/OR/XOR/NOT/BYTE ``:353-452``
  SHA3         ``:1004-1042`` Concat(memory) -> concrete keccak (keccak_function_manager.py:95-107)
  MLOAD/MSTORE/MSTORE8 ``:1435-1490``; memory words via Concat / Extract (state/memory.py:56-116)

Every term's concrete value is tracked alongside (what Mythril's ``simplify``
folds to), so control flow (JUMP/JUMPI targets, memory offsets) is concrete,
exactly as in the VMTests.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from mythril_amd.ir import Ctx, Node, BOOL
from . import bvsem as S
from .dag_eval import _eval1
from .keccak import keccak256

M256 = (1 << 256) - 1


class Unsupported(Exception):
    pass


class EvmHalt(Exception):
    pass


class MiniEVM:
    def __init__(self, ctx: Ctx, env: dict, model: Optional[dict] = None):
        self.ctx = ctx
        self.env = env
        self.model = dict(model or {})
        self.vals: Dict[int, int] = {}
        self.storage: Dict[int, Node] = {}
        self.mem: Dict[int, Node] = {}
        self.msize = 0

    # -- term helpers with concrete tracking -------------------------------
    def v(self, n: Node) -> int:
        if n.id not in self.vals:
            self.vals[n.id] = _eval1(n, [self.v(a) for a in n.args], self.model)
        return self.vals[n.id]

    def c(self, x: int, w: int = 256) -> Node:
        return self.ctx.const(x, w)

    def app(self, op, *args, params=()):
        return self.ctx.app(op, *args, params=params)

    def bv(self, item) -> Node:
        """util.pop_bitvec: Bool -> If(b, 1, 0)."""
        if isinstance(item, int):
            return self.c(item)
        if item.width == BOOL:
            return self.app("ite", item, self.c(1), self.c(0))
        return item

    def leaf(self, name: str, value: int, w: int = 256) -> Node:
        self.model[name] = value
        return self.ctx.var(name, w)

    # -- memory (state/memory.py) ---------------------------------------------
    def mem_extend(self, off: int, size: int):
        if size:
            end = off + size
            if end > 1 << 20:
                raise Unsupported("memory too large")
            self.msize = max(self.msize, (end + 31) // 32 * 32)

    def mbyte(self, i: int) -> Node:
        return self.mem.get(i) or self.c(0, 8)

    def mload(self, off: int) -> Node:
        self.mem_extend(off, 32)
        return self.app("concat", *[self.mbyte(off + i) for i in range(32)])

    def mstore(self, off: int, val: Node):
        self.mem_extend(off, 32)
        val = self.bv(val)
        for i in range(0, 256, 8):
            self.mem[off + 31 - i // 8] = self.app("extract", val, params=(i + 7, i))

    # -- execution -------------------------------------------------------------
    def run(self, code: bytes, max_steps: int = 100000):
        stack: List = []
        pc = 0
        jumpdests = set()
        i = 0
        while i < len(code):
            op = code[i]
            if op == 0x5B:
                jumpdests.add(i)
            i += (op - 0x5F + 1) if 0x60 <= op <= 0x7F else 1

        def pop():
            if not stack:
                raise EvmHalt("stack underflow")
            return stack.pop()

        def popbv():
            return self.bv(pop())

        def concrete(x) -> int:
            return self.v(self.bv(x))

        steps = 0
        while pc < len(code):
            steps += 1
            if steps > max_steps:
                raise Unsupported("step limit")
            op = code[pc]
            pc += 1
            if op == 0x00:
                return
            elif op == 0x01:
                stack.append(self.app("bvadd", popbv(), popbv()))
            elif op == 0x02:
                stack.append(self.app("bvmul", popbv(), popbv()))
            elif op == 0x03:
                a, b = popbv(), popbv()
                stack.append(self.app("bvsub", a, b))
            elif op == 0x04:
                a, b = popbv(), popbv()
                stack.append(self.c(0) if self.v(b) == 0 else self.app("bvudiv", a, b))
            elif op == 0x05:
                a, b = popbv(), popbv()
                stack.append(self.c(0) if self.v(b) == 0 else self.app("bvsdiv", a, b))
            elif op == 0x06:
                a, b = popbv(), popbv()
                stack.append(self.c(0) if self.v(b) == 0 else self.app("bvurem", a, b))
            elif op == 0x07:
                a, b = popbv(), popbv()
                stack.append(self.c(0) if self.v(b) == 0 else self.app("bvsrem", a, b))
            elif op in (0x08, 0x09):
                a, b, n = popbv(), popbv(), popbv()
                ra, rb = self.app("bvurem", a, n), self.app("bvurem", b, n)
                inner = self.app("bvadd" if op == 0x08 else "bvmul", ra, rb)
                stack.append(self.app("bvurem", inner, n))
            elif op == 0x0A:
                base, e = popbv(), popbv()
                stack.append(self.c(pow(self.v(base), self.v(e), 1 << 256)))
            elif op == 0x0B:
                s0, s1 = self.bv(pop()), self.bv(pop())
                testbit = self.app("bvadd", self.app("bvmul", s0, self.c(8)), self.c(7))
                set_tb = self.app("bvshl", self.c(1), testbit)
                sign_set = self.app("not", self.app("=", self.app("bvand", s1, set_tb), self.c(0)))
                res = self.app(
                    "ite", self.app("bvsle", s0, self.c(31)),
                    self.app("ite", sign_set,
                             self.app("bvor", s1, self.app("bvsub", self.c(0), set_tb)),
                             self.app("bvand", s1, self.app("bvsub", set_tb, self.c(1)))),
                    s1)
                stack.append(res)
            elif op == 0x10:
                stack.append(self.app("bvult", popbv(), popbv()))
            elif op == 0x11:
                stack.append(self.app("bvugt", popbv(), popbv()))
            elif op == 0x12:
                stack.append(self.app("bvslt", popbv(), popbv()))
            elif op == 0x13:
                stack.append(self.app("bvsgt", popbv(), popbv()))
            elif op == 0x14:
                a, b = self.bv(pop()), self.bv(pop())
                stack.append(self.app("=", a, b))
            elif op == 0x15:
                x = pop()
                cond = self.app("not", x) if (not isinstance(x, int) and x.width == BOOL) \
                    else self.app("=", self.bv(x), self.c(0))
                stack.append(self.app("ite", cond, self.c(1), self.c(0)))
            elif op == 0x16:
                stack.append(self.app("bvand", popbv(), popbv()))
            elif op == 0x17:
                stack.append(self.app("bvor", popbv(), popbv()))
            elif op == 0x18:
                stack.append(self.app("bvxor", popbv(), popbv()))
            elif op == 0x19:
                stack.append(self.app("bvsub", self.c(M256), popbv()))
            elif op == 0x1A:
                idx, val = pop(), popbv()
                index = concrete(idx)
                off = (31 - index) * 8
                if off >= 0:
                    stack.append(self.app("concat", self.c(0, 248),
                                          self.app("extract", val, params=(off + 7, off))))
                else:
                    stack.append(self.c(0))
            elif op in (0x1B, 0x1C, 0x1D):
                shift, value = popbv(), popbv()
                name = {0x1B: "bvshl", 0x1C: "bvlshr", 0x1D: "bvashr"}[op]
                stack.append(self.app(name, value, shift))
            elif op == 0x20:
                off, ln = concrete(pop()), concrete(pop())
                self.mem_extend(off, ln)
                data = bytes(self.v(self.mbyte(off + i)) for i in range(ln))
                stack.append(self.c(int.from_bytes(keccak256(data), "big")))
            elif op == 0x30:
                stack.append(self.leaf("address", self.env["address"]))
            elif op == 0x32:
                stack.append(self.leaf("origin", self.env["origin"]))
            elif op == 0x33:
                stack.append(self.leaf("caller", self.env["caller"]))
            elif op == 0x34:
                stack.append(self.leaf("callvalue", self.env["value"]))
            elif op == 0x35:
                off = concrete(pop())
                data = self.env["data"]
                parts = []
                for i in range(32):
                    j = off + i
                    parts.append(self.leaf(f"calldata_{j}", data[j], 8) if j < len(data) else self.c(0, 8))
                stack.append(self.app("concat", *parts))
            elif op == 0x36:
                stack.append(self.leaf("calldatasize", len(self.env["data"])))
            elif op == 0x38:
                stack.append(self.c(len(code)))
            elif op == 0x3A:
                stack.append(self.leaf("gasprice", self.env["gasPrice"]))
            elif op == 0x41:
                stack.append(self.c(self.env["coinbase"]))
            elif op == 0x42:
                stack.append(self.c(self.env["timestamp"]))
            elif op == 0x43:
                stack.append(self.c(self.env["number"]))
            elif op == 0x44:
                stack.append(self.c(self.env["difficulty"]))
            elif op == 0x45:
                stack.append(self.c(self.env["gaslimit"]))
            elif op == 0x50:
                pop()
            elif op == 0x51:
                stack.append(self.mload(concrete(pop())))
            elif op == 0x52:
                off, val = concrete(pop()), pop()
                self.mstore(off, val)
            elif op == 0x53:
                off, val = concrete(pop()), popbv()
                self.mem_extend(off, 1)
                self.mem[off] = self.app("extract", val, params=(7, 0))
            elif op == 0x54:
                k = concrete(pop())
                stack.append(self.storage.get(k, self.c(0)))
            elif op == 0x55:
                k, val = concrete(pop()), pop()
                self.storage[k] = self.bv(val) if isinstance(val, int) else val
            elif op == 0x56:
                dest = concrete(pop())
                if dest not in jumpdests:
                    raise EvmHalt("bad jump")
                pc = dest
            elif op == 0x57:
                dest, cond = concrete(pop()), pop()
                cv = self.v(cond) if (not isinstance(cond, int) and cond.width == BOOL) else concrete(cond)
                if cv:
                    if dest not in jumpdests:
                        raise EvmHalt("bad jump")
                    pc = dest
            elif op == 0x58:
                stack.append(self.c(pc - 1))
            elif op == 0x59:
                stack.append(self.c(self.msize))
            elif op == 0x5B:
                pass
            elif 0x60 <= op <= 0x7F:
                n = op - 0x5F
                stack.append(self.c(int.from_bytes(code[pc:pc + n].ljust(n, b"\x00"), "big")))
                pc += n
            elif 0x80 <= op <= 0x8F:
                d = op - 0x7F
                if len(stack) < d:
                    raise EvmHalt("stack underflow")
                stack.append(stack[-d])
            elif 0x90 <= op <= 0x9F:
                d = op - 0x8F
                if len(stack) < d + 1:
                    raise EvmHalt("stack underflow")
                stack[-d - 1], stack[-1] = stack[-1], stack[-d - 1]
            elif op == 0xF3:
                return
            else:
                raise Unsupported(f"opcode 0x{op:02x}")
            if len(stack) > 1024:
                raise EvmHalt("stack overflow")
