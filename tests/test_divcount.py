"""The division path counts behind the executed-work roofline (VERDICT r2 item
2): the product kernels report per-wave path counts
(mg_stats.lane_div_*), and oracle/c restates udivrem8's documented path rules
independently (odag_div_paths).  Here on CPU: the host build of the product
interpreter (a 'wave' of one candidate) against the oracle with wave = 1, on
divisions whose divisors are full width, one limb, and in between, signed and
unsigned, plus zero divisors.  tests/test_gpu_divcount.py checks the device's
64-lane waves."""
import random

from mythril_amd.compiler import (DIV_PRICE_FULL, DIV_PRICE_GENERAL, DIV_PRICE_SHORT, DIV_PRICE_STEP,
                                  compile_program)
from mythril_amd.hostemu import div_counts
from mythril_amd.ir import Ctx
from oracle import cdag


def _division_dag():
    c = Ctx()
    x, y, z = c.var("x", 256), c.var("y", 256), c.var("z", 256)
    conj = []
    r = random.Random(5)
    for i in range(24):
        # divisors of 1..8 limbs: y >> (32 k) keeps 8 - k limbs; z & mask gives 0 sometimes
        k = r.randrange(0, 8)
        d = c.app("bvlshr", y, c.const(32 * k + r.randrange(0, 32), 256)) if k else y
        if i % 5 == 4:
            d = c.app("bvand", d, c.app("bvlshr", z, c.const(250, 256)))   # zero for most z
        op = r.choice(["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"])
        num = c.app("bvxor", x, c.const(r.getrandbits(256), 256))
        q = c.app(op, num, d)
        conj.append(c.app("bvult", q, c.const(r.getrandbits(256), 256)))
    # a narrow division (N file, not counted) and a 160-bit one (counted: wdiv at w = 160)
    a8 = c.app("extract", x, params=(7, 0))
    conj.append(c.app("bvult", c.app("bvudiv", a8, c.app("extract", y, params=(7, 0))), c.const(9, 8)))
    x160 = c.app("extract", x, params=(159, 0))
    conj.append(c.app("bvult", c.app("bvurem", x160, c.app("extract", z, params=(191, 32))), c.const(7, 160)))
    return conj


def test_host_interpreter_counts_equal_the_oracle_restatement():
    conj = _division_dag()
    p = compile_program(conj)
    assert p.stats["wide_divisions"] == 25
    seed, n = 0x5EED, 600
    host = div_counts(p, seed, 0, n)
    orc = cdag.div_paths(conj, seed, 0, n, wave=1)
    assert host == orc
    # all three paths occur, and every division is counted once per candidate
    assert orc["lane_div_full"] > 0 and orc["lane_div_short"] > 0 and orc["lane_div_general"] > 0
    assert orc["lane_div_full"] + orc["lane_div_short"] + orc["lane_div_general"] == 25 * n
    assert 0 < orc["lane_div_steps"] <= 8 * orc["lane_div_general"]


def test_oracle_waves_take_the_slowest_lane_path():
    """A 64-lane wave goes full/short only when every lane qualifies, so it
    runs the general path at least as often as the lanes do one by one."""
    conj = _division_dag()
    one = cdag.div_paths(conj, 9, 0, 1024, wave=1)
    wv = cdag.div_paths(conj, 9, 0, 1024, wave=64)
    assert wv["lane_div_general"] >= one["lane_div_general"]
    assert wv["lane_div_steps"] >= one["lane_div_steps"]
    tot = lambda d: d["lane_div_full"] + d["lane_div_short"] + d["lane_div_general"]
    assert tot(one) == tot(wv) == 25 * 1024


def test_executed_ops_prices_the_paths():
    conj = _division_dag()
    p = compile_program(conj)
    st = {"lane_div_steps": 7, "lane_div_full": 3, "lane_div_short": 2, "lane_div_general": 1}
    floor = p.executed_ops(10, None)
    assert floor == 10 * (p.ops_per_eval - p.stats["div_nominal_ops"])
    assert p.executed_ops(10, st) == floor + 3 * DIV_PRICE_FULL + 2 * DIV_PRICE_SHORT + DIV_PRICE_GENERAL \
        + 7 * DIV_PRICE_STEP
    # the executed price of any path is below the nominal (SURVEY-derived) division price
    assert max(DIV_PRICE_FULL, DIV_PRICE_SHORT, DIV_PRICE_GENERAL + 8 * DIV_PRICE_STEP) < 664
