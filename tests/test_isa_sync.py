"""isa.py's mirrors of the library's constants (the opcode table itself is
checked against mw_isa.h by tests/test_build.py)."""




def test_layout_limits_match_the_library():
    """isa.ASM_LDS_WORDS / ASM_NK_BY_LAYOUT (engine._lands_on) mirror
    mw_kernels.hip kLdsSpillWordsByLayout and the generated MW_ASM_NK_* (ADVICE r5)."""
    import re
    from pathlib import Path

    from mythril_amd import isa
    csrc = Path(__file__).resolve().parent.parent / "mythril_amd" / "csrc"
    k = (csrc / "mw_kernels.hip").read_text()
    m = re.search(r"kLdsSpillWordsByLayout\[kAsmLayouts\] = \{kLdsSpillWords, (\d+), (\d+)\}", k)
    assert m and int(m.group(1)) == isa.ASM_LDS_WORDS["narrow"] and int(m.group(2)) == isa.ASM_LDS_WORDS["quarter"]
    assert f"constexpr u32 kLdsSpillWords = {isa.ASM_LDS_WORDS['wide']};" in k
    inc = (csrc / "mw_asm_interp.inc").read_text()
    assert f"#define MW_ASM_NK_N {isa.ASM_NK_BY_LAYOUT['narrow']}u" in inc
    assert f"#define MW_ASM_NK_Q {isa.ASM_NK_BY_LAYOUT['quarter']}u" in inc
