"""Names of the leaves that stand for reads at symbolic indices (lower.py
_Rewriter._key_name): a 64-bit structural hash names them, and a collision
must not merge two different reads into one leaf and drop their congruence
pair."""
from mythril_amd import lower
from mythril_amd.ir import Ctx
from mythril_amd.lower import lower_constraints


def _reads():
    c = Ctx()
    a = c.array("A", 256, 256)
    x, y = c.var("x", 256), c.var("y", 256)
    conj = [c.app("=", c.app("select", a, x), c.const(1, 256)),
            c.app("=", c.app("select", a, c.app("bvadd", y, c.const(1, 256))), c.const(2, 256))]
    return c, conj


def test_distinct_reads_keep_distinct_leaves(monkeypatch):
    c, conj = _reads()
    honest = lower_constraints(conj, c)
    c, conj = _reads()
    monkeypatch.setattr(lower, "_shash_args", lambda ctx, args: 0)    # every hash collides
    low = lower_constraints(conj, c)
    assert len(low.ack) == len(honest.ack) == 2
    names = sorted(low.ack)
    assert names[0] != names[1] and names[1].startswith(names[0])
    # the congruence pair (x = y + 1 => both reads agree) is still there
    assert len(low.conjuncts) == len(honest.conjuncts)


def test_one_read_keeps_one_name_across_lowerings():
    """The same read lowered again in the same context gets the same name
    (the long-lived cache dedups leaves by name)."""
    c, conj = _reads()
    first = set(lower_constraints(conj, c).ack)
    again = set(lower_constraints(list(conj), c).ack)
    assert first == again
