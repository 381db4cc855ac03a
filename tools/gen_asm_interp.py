#!/usr/bin/env python3
"""Write mythril_amd/csrc/mw_asm_interp.inc from mythril_amd/asmgen.py (the
threaded-dispatch interpreter body and the assembled kernels' template body).

    python tools/gen_asm_interp.py [--check]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "mythril_amd", "csrc", "mw_asm_interp.inc")
sys.path.insert(0, ROOT)

from mythril_amd.asmgen import render_interp  # noqa: E402


def main():
    txt = render_interp()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != txt:
            print("mw_asm_interp.inc is stale: run python tools/gen_asm_interp.py")
            sys.exit(1)
        return
    open(OUT, "w").write(txt)
    print(f"wrote {OUT}: {txt.count(chr(10))} lines")


if __name__ == "__main__":
    main()
