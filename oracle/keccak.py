"""ORACLE (test infrastructure only): Keccak-256, original (pre-NIST) padding.

Restates what ``_pysha3.keccak_256(data).digest()`` computes
(``mythril/support/support_utils.py:50-59`` ``sha3``; ``:31-47`` ``get_code_hash``;
used by ``keccak_function_manager.py:57-69`` ``find_concrete_keccak``).
pysha3 (``requirements.txt:23,36``, unpinned) implements the Keccak team's
reference permutation Keccak-f[1600]; Keccak-256 = rate 1088 bits (136 B),
capacity 512, multi-rate padding with domain byte **0x01** (NIST SHA3-256
uses 0x06 — a different function).  Pinned by ``keccak("")`` =
``keccak_function_manager.py:87-93`` and the ``vmSha3Test`` vectors.
"""
from __future__ import annotations

RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]

# rotation offsets r[x][y]
ROT = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]

M64 = (1 << 64) - 1


def _rol(x, n):
    n %= 64
    return ((x << n) | (x >> (64 - n))) & M64 if n else x


def keccak_f(A):
    """Keccak-f[1600] on a 25-lane state indexed A[x + 5*y]."""
    for rnd in range(24):
        C = [A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20] for x in range(5)]
        D = [C[(x - 1) % 5] ^ _rol(C[(x + 1) % 5], 1) for x in range(5)]
        A = [A[i] ^ D[i % 5] for i in range(25)]
        B = [0] * 25
        for x in range(5):
            for y in range(5):
                B[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(A[x + 5 * y], ROT[x][y])
        A = [B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y])
             for y in range(5) for x in range(5)]
        # the comprehension above is y-major: index = x + 5*y  (x inner)
        A[0] ^= RC[rnd]
    return A


def keccak256(data: bytes) -> bytes:
    rate = 136
    msg = bytearray(data)
    pad = rate - (len(msg) % rate)
    msg += b"\x00" * pad
    msg[len(data)] ^= 0x01
    msg[-1] ^= 0x80
    A = [0] * 25
    for off in range(0, len(msg), rate):
        block = msg[off:off + rate]
        for i in range(rate // 8):
            A[i] ^= int.from_bytes(block[8 * i:8 * i + 8], "little")
        A = keccak_f(A)
    out = b"".join(A[i].to_bytes(8, "little") for i in range(4))
    return out


def keccak256_int(data: bytes) -> int:
    return int.from_bytes(keccak256(data), "big")
