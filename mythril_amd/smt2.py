"""SMT-LIB 2 front end: z3 ``sexpr()`` text -> IR.

Reads exactly what Mythril writes with ``--solver-log`` (``Optimize.sexpr()``,
``mythril/support/model.py:45-56``) and what the drop-in ``get_model`` gets
from a z3 solver holding a constraint set: ``declare-fun`` / ``declare-const``,
``define-fun`` (0-ary), ``assert``, ``minimize`` / ``maximize``, nested
``let`` with z3's ``a!N`` names, ``|quoted|`` symbols, ``#x``/``#b``/``(_ bvN w)``
numerals, indexed ops (``(_ extract i j)``, ``zero_extend``, ``sign_extend``,
``repeat``, ``rotate_*``), arrays (``select``/``store``/``(as const ...)``),
uninterpreted function applications (``keccak256_512`` ...), and z3's internal
spellings (``bvudiv_i`` ..., ``bvumul_noovfl``, ``bvredor``/``bvredand``).

Fails closed: anything else raises :class:`Unsupported` (the caller then uses
z3 unchanged).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

from .compiler import Unsupported
from .ir import BOOL, BOOL_OPS, BV_OPS, ALIASES, Ctx, Node, topo

Sexp = Union[str, list]

# one findall over the whole text; the last alternative catches what no token
# matches (an unterminated |symbol| or "string") so it fails loudly below
_TOKEN = re.compile(r''';[^\n]*|\(|\)|\|[^|]*\||"(?:[^"]|"")*"|[^\s()|";]+|\S''')


def tokenize(text: str) -> List[Union[str, tuple]]:
    out: List[Union[str, tuple]] = []
    emit = out.append
    for t in _TOKEN.findall(text):
        c = t[0]
        if c == ";":
            continue
        if c == "|":
            if len(t) < 2 or t[-1] != "|":
                raise Unsupported(f"smt2: cannot tokenize at {t!r}")
            emit(("Q", t[1:-1]))
        elif c == '"' and (len(t) < 2 or t[-1] != '"'):
            raise Unsupported(f"smt2: cannot tokenize at {t!r}")
        else:
            emit(t)
    return out


def parse_sexps(text: str) -> List[Sexp]:
    """The s-expressions of text, tokenised on the fly (tokenize's rules: no
    intermediate token list)."""
    top: list = []
    stack: List[list] = []
    cur = top
    push, pop = stack.append, stack.pop
    for t in _TOKEN.findall(text):
        c = t[0]
        if c == "(":
            push(cur)
            cur = []
        elif c == ")":
            if not stack:
                raise Unsupported("smt2: unbalanced ')'")
            done = cur
            cur = pop()
            cur.append(done)
        elif c == ";":
            continue
        elif c == "|":
            if len(t) < 2 or t[-1] != "|":
                raise Unsupported(f"smt2: cannot tokenize at {t!r}")
            cur.append(("Q", t[1:-1]))
        elif c == '"' and (len(t) < 2 or t[-1] != '"'):
            raise Unsupported(f"smt2: cannot tokenize at {t!r}")
        else:
            cur.append(t)
    if stack:
        raise Unsupported("smt2: unbalanced '('")
    return top


def _sym(x) -> str:
    if isinstance(x, tuple):
        return x[1]
    if isinstance(x, str):
        return x
    raise Unsupported(f"smt2: expected symbol, got {x!r}")


@dataclass
class Sort:
    kind: str  # "bv" | "bool" | "array"
    width: int = 0
    dom: int = 0


@dataclass
class Decl:
    name: str
    args: List[Sort]
    sort: Sort


@dataclass
class Script:
    ctx: Ctx
    decls: Dict[str, Decl] = field(default_factory=dict)
    asserts: List[Node] = field(default_factory=list)
    minimize: List[Node] = field(default_factory=list)
    maximize: List[Node] = field(default_factory=list)


def _sort(s) -> Sort:
    if s == "Bool":
        return Sort("bool")
    if isinstance(s, list) and len(s) == 3 and s[0] == "_" and s[1] == "BitVec":
        return Sort("bv", int(s[2]))
    if isinstance(s, list) and len(s) == 3 and s[0] == "Array":
        d, r = _sort(s[1]), _sort(s[2])
        if d.kind != "bv" or r.kind != "bv":
            raise Unsupported("smt2: only bitvector arrays")
        return Sort("array", r.width, d.width)
    raise Unsupported(f"smt2: unsupported sort {s!r}")


# applications term() builds straight from their arguments (after ALIASES),
# and the heads with rules of their own
_DIRECT_OPS = frozenset({"select", "store", "ite"}) | frozenset(BOOL_OPS) | frozenset(BV_OPS)
_SPECIAL_HEADS = frozenset({"_", "let", "!", "bvredor", "bvredand"})


class _Builder:
    def __init__(self, script: Script):
        self.s = script
        self.ctx = script.ctx
        self.defs: Dict[str, Node] = {}
        self.lits: Dict[str, Node] = {}   # #x / #b literal -> const node

    def leaf(self, name: str) -> Node:
        if name in self.defs:
            return self.defs[name]
        d = self.s.decls.get(name)
        if d is None:
            raise Unsupported(f"smt2: undeclared symbol {name}")
        if d.args:
            raise Unsupported(f"smt2: function {name} used as constant")
        if d.sort.kind == "bool":
            return self.ctx.var(name, BOOL)
        if d.sort.kind == "bv":
            return self.ctx.var(name, d.sort.width)
        return self.ctx.array(name, d.sort.dom, d.sort.width)

    def term(self, e: Sexp, env: Dict[str, Node]) -> Node:
        # iterative over let-nesting depth is bounded; recursion depth follows term depth,
        # which z3's let-sharing keeps modest.  Raise the limit for deep ad-hoc inputs.
        cls = e.__class__
        if cls is list and e and e[0].__class__ is str:
            # the common application: a plain function symbol (fast path)
            head = e[0]
            if head not in _SPECIAL_HEADS:
                op = ALIASES.get(head, head)
                if op in _DIRECT_OPS:
                    term = self.term
                    return self.ctx.app(op, *[term(a, env) for a in e[1:]])
        elif cls is str:
            v = env.get(e)
            if v is not None:
                return v
        if isinstance(e, tuple):
            name = e[1]
            return env[name] if name in env else self.leaf(name)
        if isinstance(e, str):
            if e in env:
                return env[e]
            if e == "true":
                return self.ctx.true()
            if e == "false":
                return self.ctx.false()
            k = self.lits.get(e)
            if k is not None:
                return k
            if e.startswith("#x"):
                k = self.lits[e] = self.ctx.const(int(e[2:], 16), 4 * (len(e) - 2))
                return k
            if e.startswith("#b"):
                k = self.lits[e] = self.ctx.const(int(e[2:], 2), len(e) - 2)
                return k
            if re.fullmatch(r"\d+", e):
                raise Unsupported("smt2: Int numerals are outside QF_ABV")
            return self.leaf(e)
        if not e:
            raise Unsupported("smt2: empty application")
        head = e[0]
        # (_ bvN w)
        if head == "_" and len(e) == 3 and isinstance(e[1], str) and e[1].startswith("bv"):
            return self.ctx.const(int(e[1][2:]), int(e[2]))
        if head == "let":
            new_env = dict(env)
            for binding in e[1]:
                nm = _sym(binding[0])
                new_env[nm] = self.term(binding[1], env)  # parallel let: bind in the outer env
            return self.term(e[2], new_env)
        if head == "!":  # annotations
            return self.term(e[1], env)
        args = [self.term(a, env) for a in e[1:]]
        if isinstance(head, list):
            if head and head[0] == "_":
                op = head[1]
                params = [int(p) for p in head[2:]]
                if op in ("extract", "zero_extend", "sign_extend", "repeat", "rotate_left", "rotate_right"):
                    return self.ctx.app(op, *args, params=params)
                raise Unsupported(f"smt2: indexed op {op}")
            if head and head[0] == "as" and head[1] == "const":
                srt = _sort(head[2])
                if srt.kind != "array":
                    raise Unsupported("smt2: as-const of non-array")
                return self.ctx.const_array(srt.dom, args[0])
            raise Unsupported(f"smt2: application head {head!r}")
        op = _sym(head)
        op = ALIASES.get(op, op)
        if op == "bvredor":
            (x,) = args
            return self.ctx.app("ite", self.ctx.app("=", x, self.ctx.const(0, x.width)),
                                self.ctx.const(0, 1), self.ctx.const(1, 1))
        if op == "bvredand":
            (x,) = args
            return self.ctx.app("ite", self.ctx.app("=", x, self.ctx.const(-1, x.width)),
                                self.ctx.const(1, 1), self.ctx.const(0, 1))
        if op in ("select", "store", "ite") or op in BOOL_OPS or op in BV_OPS:
            return self.ctx.app(op, *args)
        d = self.s.decls.get(op)
        if d is not None and d.args:
            if len(d.args) != len(args):
                raise Unsupported(f"smt2: arity mismatch for {op}")
            return self.ctx.apply(op, d.sort.width, *args)
        raise Unsupported(f"smt2: unknown function {op}")


def parse_script(text: str, ctx: Optional[Ctx] = None) -> Script:
    import sys
    sys.setrecursionlimit(max(sys.getrecursionlimit(), 20000))
    script = Script(ctx or Ctx())
    b = _Builder(script)
    for cmd in parse_sexps(text):
        if not isinstance(cmd, list) or not cmd:
            raise Unsupported(f"smt2: bad command {cmd!r}")
        c = cmd[0]
        if c == "declare-fun":
            name = _sym(cmd[1])
            args = [_sort(a) for a in cmd[2]]
            script.decls[name] = Decl(name, args, _sort(cmd[3]))
        elif c == "declare-const":
            name = _sym(cmd[1])
            script.decls[name] = Decl(name, [], _sort(cmd[2]))
        elif c == "define-fun":
            name = _sym(cmd[1])
            if cmd[2]:
                raise Unsupported("smt2: define-fun with parameters")
            b.defs[name] = b.term(cmd[4], {})
        elif c == "assert":
            t = b.term(cmd[1], {})
            if t.width != BOOL or t.is_array:
                raise Unsupported("smt2: non-Bool assertion")
            script.asserts.append(t)
        elif c == "minimize":
            script.minimize.append(b.term(cmd[1], {}))
        elif c == "maximize":
            script.maximize.append(b.term(cmd[1], {}))
        elif c in ("check-sat", "get-model", "set-option", "set-info", "set-logic", "push", "pop",
                   "exit", "echo", "get-objectives"):
            continue
        else:
            raise Unsupported(f"smt2: command {c}")
    return script


def parse_file(path: str, ctx: Optional[Ctx] = None) -> Script:
    """Parse a dump; ``.gz`` files (the committed corpora) are read compressed."""
    if path.endswith(".gz"):
        import gzip
        with gzip.open(path, "rt") as f:
            return parse_script(f.read(), ctx)
    with open(path) as f:
        return parse_script(f.read(), ctx)


# --------------------------------------------------------------------------- printer
def _q(name: str) -> str:
    return f"|{name}|"


def _bvsort(w: int) -> str:
    return "Bool" if w == BOOL else f"(_ BitVec {w})"


def to_smt2(asserts: Sequence[Node], minimize: Sequence[Node] = (), maximize: Sequence[Node] = ()) -> str:
    """SMT-LIB2 text in the shape z3's ``Optimize.sexpr()`` gives ``--solver-log``
    (mythril/support/model.py:45-56): declarations, one ``assert`` per
    conjunct with shared subterms ``let``-bound, objectives, ``check-sat``.
    ``parse_script(to_smt2(...))`` rebuilds the same terms."""
    roots = list(asserts) + list(minimize) + list(maximize)
    nodes = topo(roots)
    out: List[str] = []
    seen = set()
    for n in nodes:
        if n.op == "var" and n.name not in seen:
            seen.add(n.name)
            out.append(f"(declare-fun {_q(n.name)} () {_bvsort(n.width)})")
        elif n.op == "array" and n.name not in seen:
            seen.add(n.name)
            out.append(f"(declare-fun {_q(n.name)} () (Array (_ BitVec {n.dom}) (_ BitVec {n.width})))")
        elif n.op == "apply" and n.name not in seen:
            seen.add(n.name)
            doms = " ".join(f"(_ BitVec {w})" for w in n.params)
            out.append(f"(declare-fun {_q(n.name)} ({doms}) (_ BitVec {n.width}))")

    def atom(n: Node, names: Dict[int, str]) -> str:
        if n.id in names:
            return names[n.id]
        if n.op == "const":
            if n.width == BOOL:
                return "true" if n.val else "false"
            if n.width % 4 == 0:
                return "#x" + format(n.val, f"0{n.width // 4}x")
            return "#b" + format(n.val, f"0{n.width}b")
        if n.op in ("var", "array"):
            return _q(n.name)
        args = " ".join(names.get(a.id) or atom(a, names) for a in n.args)
        if n.op in ("extract", "zero_extend", "sign_extend", "repeat", "rotate_left", "rotate_right"):
            return f"((_ {n.op} {' '.join(str(p) for p in n.params)}) {args})"
        if n.op == "const_array":
            return f"((as const (Array (_ BitVec {n.dom}) (_ BitVec {n.width}))) {args})"
        if n.op == "apply":
            return f"({_q(n.name)} {args})"
        return f"({n.op} {args})"

    def term(root: Node) -> str:
        # let-bind every non-leaf subterm used more than once within this root
        sub = topo([root])
        uses: Dict[int, int] = {}
        for m in sub:
            for a in m.args:
                uses[a.id] = uses.get(a.id, 0) + 1
        names: Dict[int, str] = {}
        lets: List[Tuple[str, str]] = []
        for m in sub:
            if m is not root and uses.get(m.id, 0) > 1 and m.args:
                nm = f"a!{len(lets) + 1}"
                lets.append((nm, atom(m, names)))
                names[m.id] = nm
        body = atom(root, names)
        for nm, t in reversed(lets):
            body = f"(let (({nm} {t})) {body})"
        return body

    out += [f"(assert {term(a)})" for a in asserts]
    out += [f"(minimize {term(m)})" for m in minimize]
    out += [f"(maximize {term(m)})" for m in maximize]
    out.append("(check-sat)")
    return "\n".join(out) + "\n"
