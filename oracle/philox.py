"""ORACLE (test infrastructure only): Philox4x32-10 and the candidate-leaf spec.

Philox4x32-10 is restated from its publication (Salmon, Moraes, Dror, Shaw,
"Parallel random numbers: as easy as 1, 2, 3", SC'11), pinned by the
Random123 known-answer vectors in ``tests/test_oracle.py``.

Candidate-leaf specification (DESIGN.md "Candidate space"):
for candidate index ``c`` (u64), leaf ``j`` of width ``w``:

* ``random`` leaf, ``w > 32``: limbs = Philox4x32-10(key=(seed_lo ^ j, seed_hi),
  counter=(c_lo, c_hi, blk, 0)) for blk = 0,1; limb k = block[k//4][k%4]
  (limb 0 least significant), value masked to ``w`` bits.
* ``random`` leaf, ``w <= 32`` (calldata bytes, Bools, small words):
  fmix64(c ^ seed ^ (j * 0xC2B2AE3D27D4EB4F)) masked to ``w`` bits - one
  64-bit finalizer instead of ten Philox rounds (measured: Philox was half of
  the specialised kernels' time on the C2 query).
* ``pool`` leaf with 2**b entries at bit-field ``s``: digit = (c >> s) & (2**b-1);
  entry = pool[digit]; an entry flagged RANDOM yields the random value above,
  otherwise its constant (masked to ``w``).
* ``interleaved`` pool leaf (stride n): digit bit b = index bit (shift + b*n).
* ``hashed`` pool leaf: digit = fmix64(c ^ (salt * 0x9E3779B97F4A7C15)) & (2**b-1).
"""
from __future__ import annotations

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
U32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for r in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> 32, p0 & U32
        hi1, lo1 = p1 >> 32, p1 & U32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & U32, lo1, (hi0 ^ c3 ^ k1) & U32, lo0
        k0 = (k0 + W0) & U32
        k1 = (k1 + W1) & U32
    return c0, c1, c2, c3


NARROW_SALT = 0xC2B2AE3D27D4EB4F
M64 = (1 << 64) - 1


def random_leaf(seed: int, leaf_id: int, c: int, width: int) -> int:
    if width <= 32:
        return fmix64((c ^ seed ^ (leaf_id * NARROW_SALT)) & M64) & ((1 << width) - 1)
    key = ((seed ^ leaf_id) & U32, (seed >> 32) & U32)
    limbs = []
    for blk in range(2):
        limbs.extend(philox4x32_10((c & U32, (c >> 32) & U32, blk, 0), key))
    v = 0
    for k, x in enumerate(limbs):
        v |= x << (32 * k)
    return v & ((1 << width) - 1)


def fmix64(h: int) -> int:
    """MurmurHash3 64-bit finalizer (Appleby, public domain)."""
    M = (1 << 64) - 1
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & M
    h ^= h >> 33
    h = (h * 0xC4CEB9FE1A85EC53) & M
    h ^= h >> 33
    return h


def leaf_value(spec: dict, seed: int, c: int) -> int:
    """spec: {'id','width','shift','bits','pool': [int or None], 'hashed': bool}  (None = RANDOM)."""
    w = spec["width"]
    pool = spec.get("pool")
    if pool:
        if spec.get("hashed"):
            src = fmix64(c ^ ((spec["id"] * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)))
            d = src & ((1 << spec["bits"]) - 1)
        elif spec.get("stride"):
            d = 0
            for b in range(spec["bits"]):
                d |= ((c >> (spec["shift"] + b * spec["stride"])) & 1) << b
        else:
            d = (c >> spec["shift"]) & ((1 << spec["bits"]) - 1)
        e = pool[d]
        if e is not None:
            return e & ((1 << w) - 1)
    return random_leaf(seed, spec["id"], c, w)
