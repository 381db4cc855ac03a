"""Builders for the constraint shapes Mythril emits, restated from the reference
(test infrastructure: used to feed the engine the formulas LASER would build).

* keccak UFs and their conditions: ``keccak_function_manager.py:19-21`` (interval
  constants), ``:71-84`` (keccak256_N / keccak256_N-1), ``:95-114`` (create_keccak:
  concrete data -> real hash, symbolic -> UF application), ``:116-130``
  (create_conditions), ``:150-179`` (_create_condition);
* symbolic calldata reads: ``state/calldata.py:214-231`` (``If(item < size,
  calldata[item], 0)`` with the *signed* ``<`` of ``bitvec.py:201-210``).
"""
from mythril_amd.ir import Ctx
from oracle.keccak import keccak256

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30


class KeccakManager:
    def __init__(self, ctx: Ctx):
        self.c = ctx
        self.interval_hook_for_size = {}
        self.index_counter = TOTAL_PARTS - 34534
        self.concrete_hashes = {}   # (width, value) -> hash int
        self.symbolic_inputs = []   # terms

    def func(self, n, x):
        return self.c.apply(f"keccak256_{n}", 256, x)

    def inv(self, n, y):
        return self.c.apply(f"keccak256_{n}-1", n, y)

    def create_keccak(self, data):
        n = data.width
        if data.op == "const":
            h = int.from_bytes(keccak256(data.val.to_bytes(n // 8, "big")), "big")
            self.concrete_hashes[(n, data.val)] = h
            return self.c.const(h, 256)
        self.symbolic_inputs.append(data)
        return self.func(n, data)

    def _create_condition(self, x):
        c = self.c
        n = x.width
        if n not in self.interval_hook_for_size:
            self.interval_hook_for_size[n] = self.index_counter
            self.index_counter -= INTERVAL_DIFFERENCE
        lower = self.interval_hook_for_size[n] * PART
        upper = lower + PART
        fx = self.func(n, x)
        cond = c.app("and", c.app("=", self.inv(n, fx), x),
                     c.app("bvule", c.const(lower, 256), fx),
                     c.app("bvult", fx, c.const(upper, 256)),
                     c.app("=", c.app("bvurem", fx, c.const(64, 256)), c.const(0, 256)))
        concrete = c.false()
        for (kw, kv), h in self.concrete_hashes.items():
            if kw == n:
                concrete = c.app("or", concrete, c.app("and", c.app("=", fx, c.const(h, 256)),
                                                         c.app("=", c.const(kv, kw), x)))
        return c.app("and", c.app("=", self.inv(n, fx), x), c.app("or", cond, concrete))

    def create_conditions(self):
        c = self.c
        cond = c.true()
        for x in self.symbolic_inputs:
            cond = c.app("and", cond, self._create_condition(x))
        for (kw, kv), h in self.concrete_hashes.items():
            k = c.const(kv, kw)
            cond = c.app("and", cond, c.app("=", self.func(kw, k), c.const(h, 256)),
                         c.app("=", self.inv(kw, self.func(kw, k)), k))
        return cond


def calldata_load(ctx: Ctx, tx: str, item):
    """SymbolicCalldata._load: If(item < size (signed), calldata[item], 0)."""
    size = ctx.var(f"{tx}_calldatasize", 256)
    arr = ctx.array(f"{tx}_calldata", 256, 8)
    return ctx.app("ite", ctx.app("bvslt", item, size), ctx.app("select", arr, item), ctx.const(0, 8))


def calldata_word(ctx: Ctx, tx: str, offset: int):
    return ctx.app("concat", *[calldata_load(ctx, tx, ctx.const(offset + i, 256)) for i in range(32)])
