#!/usr/bin/env python3
"""Generate tests/golden/*.json from the reference's own known-answer data.

Run in the build container (needs /root/reference; never run on the GPU box):
    python tools/make_golden.py

Reads, as data only (nothing from the reference is imported or executed):
  * tests/instructions/{shl,shr,sar}_test.py — EIP-145 vectors: the
    3-string parametrize tuples and the ``BVV(<const-expr>, 256)`` test_data
    rows (constant expressions folded by a tiny AST evaluator); rows with a
    symbolic value and a concrete shift >= 256 become "any value" rows
    (``shl_test.py:32``, ``shr_test.py:33``).
  * tests/laser/evm_testsuite/VMTests/<category>/*.json — exec/env/pre and the
    post-storage values the harness asserts (``evm_test.py:172-189``), for the
    categories the harness runs (``evm_test.py:22-32``) minus its ignore list
    (``:34-61``).
"""
import ast
import json
import operator
import sys
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"

_BIN = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
        ast.FloorDiv: operator.floordiv, ast.LShift: operator.lshift,
        ast.RShift: operator.rshift, ast.Pow: operator.pow}


def _const(node):
    if isinstance(node, ast.Constant) and isinstance(node.value, int):
        return node.value
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        return -_const(node.operand)
    if isinstance(node, ast.BinOp) and type(node.op) in _BIN:
        return _BIN[type(node.op)](_const(node.left), _const(node.right))
    raise ValueError("not a constant expression")


def _bvv(node):
    """BVV(expr, 256) -> int mod 2**256, BV("a",256) -> None, int literal -> int."""
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name):
        if node.func.id == "BVV":
            return _const(node.args[0]) % (1 << _const(node.args[1]))
        if node.func.id == "BV":
            return None
    return _const(node)


def eip145():
    rows = []
    for op in ("shl", "shr", "sar"):
        src = (REF / "tests" / "instructions" / f"{op}_test.py").read_text()
        tree = ast.parse(src)
        for node in ast.walk(tree):
            # parametrize tuples ("0x..", "0x..", "0x..")
            if isinstance(node, ast.Tuple) and len(node.elts) == 3 and all(
                    isinstance(e, ast.Constant) and isinstance(e.value, str) and e.value.startswith("0x")
                    for e in node.elts):
                v, s, e = (int(x.value, 16) for x in node.elts)
                rows.append({"op": op, "value": v, "shift": s, "expected": e,
                             "src": f"tests/instructions/{op}_test.py:{node.lineno}"})
            # test_data rows ([BVV(v), BVV(s)], BVV(e))
            if (isinstance(node, ast.Tuple) and len(node.elts) == 2
                    and isinstance(node.elts[0], ast.List) and len(node.elts[0].elts) == 2):
                try:
                    v, s = (_bvv(x) for x in node.elts[0].elts)
                    e = _bvv(node.elts[1])
                except (ValueError, AttributeError, IndexError):
                    continue
                if s is None or e is None:
                    continue
                rows.append({"op": op, "value": v, "shift": s, "expected": e,
                             "src": f"tests/instructions/{op}_test.py:{node.lineno}"})
    return rows


CATS = ["vmArithmeticTest", "vmBitwiseLogicOperation", "vmEnvironmentalInfo",
        "vmPushDupSwapTest", "vmTests", "vmSha3Test", "vmSystemOperations",
        "vmRandomTest", "vmIOandFlowOperations"]
IGNORED = {"gas0", "gas1", "log1MemExp", "BlockNumberDynamicJumpi0", "BlockNumberDynamicJumpi1",
           "BlockNumberDynamicJump0_jumpdest2", "DynamicJumpPathologicalTest0",
           "BlockNumberDynamicJumpifInsidePushWithJumpDest", "BlockNumberDynamicJumpiAfterStop",
           "BlockNumberDynamicJumpifInsidePushWithoutJumpDest", "BlockNumberDynamicJump0_jumpdest0",
           "BlockNumberDynamicJumpi1_jumpdest", "BlockNumberDynamicJumpiOutsideBoundary",
           "DynamicJumpJD_DependsOnJumps1", "loop_stacklimit_1020", "loop_stacklimit_1021",
           "jumpTo1InstructionafterJump", "sstore_load_2", "jumpi_at_the_end"}


def vmtests():
    out = []
    base = REF / "tests" / "laser" / "evm_testsuite" / "VMTests"
    for cat in CATS:
        d = base / cat
        if not d.is_dir():
            continue
        for f in sorted(d.iterdir()):
            if f.suffix != ".json":
                continue
            top = json.loads(f.read_text())
            for name, t in top.items():
                if name in IGNORED:
                    continue
                ex, env = t["exec"], t.get("env", {})
                post = t.get("post", {})
                addr = ex["address"]
                pre_acct = t["pre"].get(addr, {})
                storage = {}
                if post:
                    acct = post.get(addr) or next(iter(post.values()))
                    storage = acct.get("storage", {})
                out.append({
                    "name": name, "category": cat, "file": f"{cat}/{f.name}",
                    "code": ex["code"], "data": ex["data"], "value": ex["value"],
                    "caller": ex["caller"], "origin": ex["origin"], "address": addr,
                    "gasPrice": ex["gasPrice"],
                    "env": {k: env.get(k, "0x0") for k in ("currentCoinbase", "currentTimestamp",
                                                          "currentNumber", "currentDifficulty",
                                                          "currentGasLimit")},
                    "pre_storage": pre_acct.get("storage", {}),
                    "has_post": bool(post),
                    "post_storage": storage,
                })
    return out


def main():
    if not REF.is_dir():
        sys.exit("needs /root/reference (build container only)")
    OUT.mkdir(parents=True, exist_ok=True)
    e = eip145()
    (OUT / "eip145.json").write_text(json.dumps(e, indent=1))
    v = vmtests()
    (OUT / "vmtests.json").write_text(json.dumps(v, separators=(",", ":")))
    print(f"eip145: {len(e)} rows; vmtests: {len(v)} cases "
          f"({sum(1 for x in v if x['post_storage'])} with post storage)")


if __name__ == "__main__":
    main()
