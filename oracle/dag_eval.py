"""ORACLE (test infrastructure only): evaluate a constraint DAG under a model.

This is what ``z3.ModelRef.eval(expr, model_completion=True)`` computes for a
fully-assigned model, i.e. the ``substitute + simplify + is_true`` reference
path of SURVEY.md §8(d) "CPU baseline" (``mythril/laser/smt/model.py:52-59``
``Model.eval`` -> ``z3.ModelRef.eval``).

A *model* is a dict:
  ``name -> int``                          bitvector / Bool constants
  ``name -> (dict[int,int], default)``     arrays  (``z3.Array``; ``K`` arrays are terms)
  ``name -> (dict[tuple,int], default)``   uninterpreted functions (``z3.Function``,
                                            ``mythril/laser/smt/function.py:7-29``)
Array/UF reads fall back to ``default`` like z3's ``else`` interpretation.
"""
from __future__ import annotations

from typing import Dict, Iterable, List

from . import bvsem as S


class ArrayVal:
    """A concrete array value: finite map + default (z3 ``K``/``Store`` chain)."""

    __slots__ = ("m", "default")

    def __init__(self, m=None, default=0):
        self.m = dict(m or {})
        self.default = default

    def get(self, i):
        return self.m.get(i, self.default)

    def stored(self, i, v):
        out = ArrayVal(self.m, self.default)
        out.m[i] = v
        return out

    def __eq__(self, other):
        if not isinstance(other, ArrayVal):
            return NotImplemented
        keys = set(self.m) | set(other.m)
        return self.default == other.default and all(self.get(k) == other.get(k) for k in keys)


def _topo(roots):
    out, seen = [], set()
    for r in roots:
        stack = [(r, False)]
        while stack:
            n, done = stack.pop()
            if n.id in seen:
                continue
            if done:
                seen.add(n.id)
                out.append(n)
                continue
            stack.append((n, True))
            for a in reversed(n.args):
                if a.id not in seen:
                    stack.append((a, False))
    return out


def eval_nodes(roots: Iterable, model: Dict) -> Dict[int, object]:
    """Return {node.id: value} for every node reachable from roots."""
    vals: Dict[int, object] = {}
    for n in _topo(list(roots)):
        vals[n.id] = _eval1(n, [vals[a.id] for a in n.args], model)
    return vals


def eval_term(root, model: Dict):
    return eval_nodes([root], model)[root.id]


def _eval1(n, av: List, model):
    op, w = n.op, n.width
    if op == "const":
        return n.val
    if op == "var":
        v = model[n.name]
        return v & S.mask(w) if w else (1 if v else 0)
    if op == "array":
        m = model.get(n.name)
        if m is None:
            return ArrayVal({}, 0)
        if isinstance(m, ArrayVal):
            return m
        d, default = m
        return ArrayVal(d, default)
    if op == "const_array":
        return ArrayVal({}, av[0])
    if op == "store":
        return av[0].stored(av[1], av[2])
    if op == "select":
        return av[0].get(av[1])
    if op == "apply":
        d, default = model.get(n.name, ({}, 0))
        return d.get(tuple(av), default) & S.mask(w)
    if op == "ite":
        return av[1] if av[0] else av[2]
    # Bool connectives
    if op == "and":
        return int(all(av))
    if op == "or":
        return int(any(av))
    if op == "not":
        return 1 - av[0]
    if op == "xor":
        r = 0
        for x in av:
            r ^= x
        return r
    if op == "=>":
        return int((not av[0]) or bool(av[1]))
    if op == "=":
        if isinstance(av[0], ArrayVal):
            return int(all(a == av[0] for a in av[1:]))
        return int(all(a == av[0] for a in av[1:]))
    if op == "distinct":
        return int(len(set(av)) == len(av))
    aw = n.args[0].width if n.args else w
    if op in S.BINARY_PRED:
        return S.BINARY_PRED[op](aw, av[0], av[1])
    if op in S.NARY_BV:
        return S.NARY_BV[op](w, *av)
    if op in S.BINARY_BV:
        return S.BINARY_BV[op](w, av[0], av[1])
    if op in S.UNARY_BV:
        return S.UNARY_BV[op](w, av[0])
    if op == "concat":
        return S.concat([a.width for a in n.args], av)
    if op == "extract":
        return S.extract(n.params[0], n.params[1], av[0])
    if op == "zero_extend":
        return av[0]
    if op == "sign_extend":
        return S.sign_extend(aw, n.params[0], av[0])
    if op == "repeat":
        return S.repeat(aw, n.params[0], av[0])
    if op == "rotate_left":
        return S.rotate_left(w, n.params[0], av[0])
    if op == "rotate_right":
        return S.rotate_right(w, n.params[0], av[0])
    if op == "bvcomp":
        return int(av[0] == av[1])
    raise KeyError(f"oracle: unknown op {op}")
