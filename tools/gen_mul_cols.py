#!/usr/bin/env python3
"""Generates the column asm of mw_jit.h's mul8_cols (the Comba multiply of the
specialised kernels): one asm statement per column k = 1..6 over products
(i, k - i), v_mad_u64_u32 into the column's 64-bit pair with its carry-out in
one of three SGPR pairs (rotating), v_addc counting the carries into c.

Hazard rule (gfx950): a VALU that reads an SGPR as carry-in must follow the
VALU that wrote it by two wait states; LLVM does not insert them inside asm.
The list scheduler below issues each product as soon as its SGPR pair is
free and each v_addc once two VALU instructions separate it from its v_mad
(an s_nop only where the column runs out: column 1).

    python tools/gen_mul_cols.py          # prints the column statements
"""
S = ["%[s0]", "%[s1]", "%[s2]"]


def column(k: int, carry: bool):
    """asm lines of column k; carry=False for the column whose carries would
    leave the 256-bit product (k = 6).  List scheduling: a product issues as
    soon as its SGPR pair holds no unread carry, a carry's v_addc as soon as
    two VALU instructions follow its v_mad; an s_nop only when neither can."""
    out, pending = [], []            # pending: (sgpr pair, position of its v_mad)
    pos = 0
    first = True
    prods = [(i, k - i) for i in range(k + 1)]
    n = 0

    def ready(q):
        return pos - q[1] - 1 >= 2

    def addc(q):
        nonlocal pos, first
        gap = pos - q[1] - 1            # VALU instructions since the carry's write
        if gap < 2:
            out.append(f"s_nop {1 - gap}")
        src = "0" if first else "%[c]"
        out.append(f"v_addc_co_u32_e64 %[c], {S[q[0]]}, {src}, 0, {S[q[0]]}")
        first = False
        pending.remove(q)
        pos += 1

    while n < len(prods) or pending:
        s = n % 3
        if n < len(prods) and all(q[0] != s for q in pending):
            i, j = prods[n]
            out.append(f"v_mad_u64_u32 %[p], {S[s]}, %[a{i}], %[b{j}], %[p]")
            # column 1's first product cannot overflow: {hi(a0 b0), 0} + a0 b1 < 2^64
            if carry and not (k == 1 and n == 0):
                pending.append((s, pos))
            pos += 1
            n += 1
            continue
        rdy = [q for q in pending if ready(q)]
        addc(rdy[0] if rdy else pending[0])
    return out


def statements() -> str:
    out = []
    for k in range(1, 7):
        carry = k <= 5
        lines = column(k, carry)
        ins = ", ".join([f'[a{i}] "v"(a[{i}])' for i in range(k + 1)] + [f'[b{j}] "v"(b[{j}])' for j in range(k + 1)])
        outs = '[p] "+v"(p)' + (', [c] "=&v"(c)' if carry else '') + \
            ', [s0] "=&s"(s0), [s1] "=&s"(s1), [s2] "=&s"(s2)'
        out.append(f"  // column {k}")
        out.append("  asm(" + "\n      ".join(f'"{x}\\n"' for x in lines))
        out.append(f"      : {outs}")
        out.append(f"      : {ins});")
        if k < 6:
            out.append(f"  r[{k}] = (u32)p;")
            out.append("  p = (p >> 32) | ((u64)c << 32);")
    return "\n".join(out)


if __name__ == "__main__":
    print(statements())
