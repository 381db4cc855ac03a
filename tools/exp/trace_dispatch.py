"""Experiment: follow the scalar control flow of the interpreter loop in the
gfx950 disassembly for one bytecode instruction and count what executes.

    python tools/exp/trace_dispatch.py search.s HEAD_LINE w0 w1 w2 w3 [sreg=val ...]

Only SALU state is emulated (exec = all lanes); values the trace cannot know
are None, and a branch on an unknown condition stops the trace.
"""
import re
import sys
from collections import Counter

M32, M64 = (1 << 32) - 1, (1 << 64) - 1


def parse(path):
    insns, addr_of, line_of = [], {}, {}
    start = None
    for l in open(path):
        m = re.match(r"\s+(\S+)\s*(.*?)\s*// ([0-9A-F]{12}):", l)
        if not m:
            continue
        a = int(m.group(3), 16)
        if start is None:
            start = a
        op, rest = m.group(1), m.group(2)
        tgt = re.search(r"<\w+\+0x([0-9a-f]+)>", l)
        rest = re.sub(r"<.*>", "", rest).strip()
        args = [x.strip() for x in rest.split(",")] if rest else []
        insns.append((a - start, op, args, int(tgt.group(1), 16) if tgt else None))
        line_of[a - start] = len(insns) - 1
    return insns, line_of


class St:
    def __init__(self):
        self.s = {}
        self.scc = None
        self.exec = M64
        self.vcc = None

    def get(self, x, wide=False):
        x = x.strip()
        if x == "exec":
            return self.exec
        if x == "vcc":
            return self.vcc
        if x == "scc":
            return self.scc
        m = re.match(r"s\[(\d+):(\d+)\]$", x)
        if m:
            lo = self.s.get(int(m.group(1)))
            hi = self.s.get(int(m.group(2)))
            return None if lo is None or hi is None else lo | (hi << 32)
        m = re.match(r"s(\d+)$", x)
        if m:
            v = self.s.get(int(m.group(1)))
            return v
        try:
            v = int(x, 0)
            return v & (M64 if wide else M32)
        except ValueError:
            return None

    def put(self, x, v):
        x = x.strip()
        if x == "exec":
            self.exec = v
            return
        if x == "vcc":
            self.vcc = v
            return
        m = re.match(r"s\[(\d+):(\d+)\]$", x)
        if m:
            lo, hi = int(m.group(1)), int(m.group(2))
            self.s[lo] = None if v is None else v & M32
            self.s[hi] = None if v is None else (v >> 32) & M32
            return
        m = re.match(r"s(\d+)$", x)
        if m:
            self.s[int(m.group(1))] = None if v is None else v & M32


def sx(v, bits=32):
    return v - (1 << bits) if v is not None and v >> (bits - 1) & 1 else v


def run(insns, line_of, head, st, limit=4000):
    pc = line_of[head]
    cnt = Counter()
    path = []
    for _ in range(limit):
        a, op, args, tgt = insns[pc]
        cls = "branch" if "branch" in op else op.split("_")[0]
        cnt[cls] += 1
        cnt[op] += 0
        path.append((a, op, args))
        nxt = pc + 1
        g = st.get
        w64 = op.endswith("_b64") or op.endswith("_u64")
        try:
            if op == "s_cbranch_execz" or op == "s_cbranch_execnz":
                pass
            if op.startswith("v_") or op.startswith("ds_") or op.startswith("global_") or op.startswith("buffer_"):
                if op.startswith("v_cmp") and args and (args[0] == "vcc" or args[0].startswith("s")):
                    st.put(args[0], None)
                elif op.startswith("v_readfirstlane") or op.startswith("v_readlane"):
                    st.put(args[0], None)
                elif args and args[0].startswith("s[") and op.startswith(("v_add_co", "v_sub_co", "v_addc", "v_subb", "v_mad")):
                    pass
            elif op.startswith("s_load") or op.startswith("s_buffer_load"):
                st.put(args[0], None)
            elif op in ("s_waitcnt", "s_nop", "s_set_gpr_idx_off") or op.startswith("s_set_gpr_idx_on"):
                pass
            elif op in ("s_mov_b32", "s_mov_b64"):
                st.put(args[0], g(args[1], w64))
            elif op in ("s_and_b32", "s_and_b64", "s_or_b32", "s_or_b64", "s_xor_b32", "s_xor_b64",
                        "s_andn2_b32", "s_andn2_b64", "s_orn2_b64", "s_orn2_b32"):
                x, y = g(args[1], w64), g(args[2], w64)
                m = M64 if w64 else M32
                if x is None or y is None:
                    r = None
                    # x & 0 = 0 style shortcuts
                    if op.startswith("s_and_") and (x == 0 or y == 0):
                        r = 0
                else:
                    r = {"s_and": x & y, "s_or": x | y, "s_xor": x ^ y, "s_andn2": x & ~y & m,
                         "s_orn2": (x | ~y) & m}[op.rsplit("_", 1)[0]]
                st.put(args[0], r)
                st.scc = None if r is None else int(r != 0)
            elif op in ("s_not_b32", "s_not_b64"):
                x = g(args[1], w64)
                r = None if x is None else ~x & (M64 if w64 else M32)
                st.put(args[0], r)
                st.scc = None if r is None else int(r != 0)
            elif op in ("s_lshr_b32", "s_lshl_b32", "s_lshr_b64", "s_lshl_b64", "s_ashr_i32"):
                x, y = g(args[1], w64), g(args[2])
                if x is None or y is None:
                    r = None
                else:
                    sh = y & (63 if w64 else 31)
                    r = (x >> sh) if "lshr" in op else (x << sh) if "lshl" in op else (sx(x) >> sh)
                    r &= M64 if w64 else M32
                st.put(args[0], r)
                st.scc = None if r is None else int(r != 0)
            elif op in ("s_add_u32", "s_add_i32", "s_sub_u32", "s_sub_i32", "s_addc_u32", "s_mul_i32",
                        "s_min_u32", "s_max_u32"):
                x, y = g(args[1]), g(args[2])
                if x is None or y is None:
                    r = None
                else:
                    r = {"s_add_u32": x + y, "s_add_i32": x + y, "s_sub_u32": x - y, "s_sub_i32": x - y,
                         "s_addc_u32": x + y + (st.scc or 0), "s_mul_i32": x * y,
                         "s_min_u32": min(x, y), "s_max_u32": max(x, y)}[op] & M32
                st.put(args[0], r)
            elif op.startswith("s_cmp_") or op.startswith("s_cmpk_"):
                kind = op.split("_")[2]
                typ = op.split("_")[3]
                x, y = g(args[0], typ == "u64"), g(args[1], typ == "u64")
                if x is None or y is None:
                    st.scc = None
                else:
                    if typ.startswith("i"):
                        x, y = sx(x), sx(y)
                    st.scc = int({"eq": x == y, "lg": x != y, "lt": x < y, "gt": x > y, "le": x <= y,
                                  "ge": x >= y}[kind])
            elif op.startswith("s_bitcmp"):
                x, b = g(args[0]), g(args[1])
                st.scc = None if x is None or b is None else int(((x >> b) & 1) == (1 if "bitcmp1" in op else 0))
            elif op.startswith("s_cselect"):
                x, y = g(args[1], w64), g(args[2], w64)
                st.put(args[0], None if st.scc is None else (x if st.scc else y))
            elif op == "s_bfe_u32":
                x, c = g(args[1]), g(args[2])
                if x is None or c is None:
                    r = None
                else:
                    off, wd = c & 31, (c >> 16) & 0x7f
                    r = (x >> off) & ((1 << wd) - 1)
                st.put(args[0], r)
                st.scc = None if r is None else int(r != 0)
            elif op == "s_and_saveexec_b64":
                old = st.exec
                y = g(args[1], True)
                st.put(args[0], old)
                st.exec = None if y is None or old is None else old & y
                st.scc = None if st.exec is None else int(st.exec != 0)
            elif op.startswith("s_cbranch") or op == "s_branch":
                cond = {"s_branch": True, "s_cbranch_scc0": None if st.scc is None else st.scc == 0,
                        "s_cbranch_scc1": None if st.scc is None else st.scc == 1,
                        "s_cbranch_vccz": None if st.vcc is None else st.vcc == 0,
                        "s_cbranch_vccnz": None if st.vcc is None else st.vcc != 0,
                        "s_cbranch_execz": None if st.exec is None else st.exec == 0,
                        "s_cbranch_execnz": None if st.exec is None else st.exec != 0}.get(op)
                if cond is None:
                    print(f"unknown branch condition at +{a:#x} {op}; stop")
                    break
                if cond:
                    nxt = line_of[tgt]
            else:
                if op.startswith("s_") and args and (args[0].startswith("s") or args[0] in ("vcc", "exec")):
                    st.put(args[0], None)
        except Exception as e:  # noqa: BLE001
            print("emulation error", op, args, e)
            break
        pc = nxt
        if insns[pc][0] == head:
            break
    return cnt, path


def main():
    path, head = sys.argv[1], int(sys.argv[2], 0)
    words = [int(x, 0) for x in sys.argv[3:7]]
    insns, line_of = parse(path)
    st = St()
    for k, w in zip((36, 37, 38, 39), words):
        st.s[k] = w
    for kv in sys.argv[7:]:
        k, v = kv.split("=")
        st.put(k, int(v, 0))
    cnt, p = run(insns, line_of, head, st)
    tot = sum(v for k, v in cnt.items() if k in ("s", "v", "branch", "ds", "global"))
    print({k: v for k, v in cnt.items() if k in ("s", "v", "branch", "ds", "global")}, "total", tot)
    if "-v" in sys.argv or True:
        for a, op, args in p:
            print(f"  +{a:#06x} {op} {', '.join(args)}")


if __name__ == "__main__":
    main()
