"""Batched Keccak-256 service (mythril_amd/keccak_service.py).

The reference's concrete-hash entry points are ``sha3`` and ``get_code_hash``
(mythril/support/support_utils.py:31-59), ``find_concrete_keccak``
(keccak_function_manager.py:57-69) and ``_replace_with_actual_sha``
(mythril/analysis/solver.py:128-164).  pysha3 is not importable here, so the
reference sha3 is stood in for by the oracle's Keccak-256, itself pinned by the
reference's vmSha3Test vectors (tests/test_oracle.py).  CPU tests drive the
service through the host build of the Keccak kernel source (tests/fakedev.py);
the GPU test drives mg_keccak256 on the device.
"""
import random

import pytest

from mythril_amd.keccak_service import HASH_MATCHER, KeccakService, replace_with_actual_sha
from oracle.keccak import keccak256
from tests.fakedev import FakeDevice

EMPTY = "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"


def _reference_counter():
    calls = {"n": 0}

    def ref(m):
        calls["n"] += 1
        return keccak256(m)
    return ref, calls


def test_sha3_argument_forms_match_reference():
    ref, _ = _reference_counter()
    svc = KeccakService(device=FakeDevice(), reference=ref, min_batch=1)
    assert svc.sha3(b"").hex() == EMPTY
    assert svc.sha3("0x").hex() == EMPTY
    assert svc.sha3("0x0000000000") == keccak256(b"\0" * 5)
    # text is UTF-8 encoded: the selector of transfer(address,uint256)
    assert svc.sha3("transfer(address,uint256)")[:4].hex() == "a9059cbb"
    assert svc.sha3(bytearray(b"abc")) == keccak256(b"abc")


def test_get_code_hash_forms():
    ref, _ = _reference_counter()
    svc = KeccakService(device=FakeDevice(), reference=ref, min_batch=1)
    assert svc.get_code_hash("") == "0x" + EMPTY
    assert svc.get_code_hash("0x6001") == "0x" + keccak256(bytes.fromhex("6001")).hex()
    assert svc.get_code_hash("0xzz") == ""
    t = ("sym", 1)
    assert svc.get_code_hash(t) == str(hash(t))


def test_find_concrete_keccak_empty_constant():
    """keccak_function_manager.py:87-93 pins keccak('') as an integer."""
    svc = KeccakService(device=FakeDevice(), reference=keccak256, min_batch=1)
    assert svc.find_concrete_keccak_int(0, 0) == \
        89477152217924674838424037953991966239322087453347756267410168184682657981552
    # mapping slot: keccak256(pad32(key) ++ pad32(slot)) as a 512-bit preimage
    key, slot = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 1
    assert svc.find_concrete_keccak_int((key << 256) | slot, 512) == int.from_bytes(
        keccak256(key.to_bytes(32, "big") + slot.to_bytes(32, "big")), "big")


def test_batch_goes_to_device_once_and_memoises():
    ref, calls = _reference_counter()
    dev = FakeDevice()
    svc = KeccakService(device=dev, reference=ref, min_batch=8)
    rng = random.Random(3)
    msgs = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 20, 32, 64, 135, 136, 137, 300])))
            for _ in range(100)]
    msgs += msgs[:10]                                  # duplicates inside one batch
    out = svc.hash_many(msgs)
    assert out == [keccak256(m) for m in msgs]
    assert dev.keccak_launches == 1 and calls["n"] == 0
    assert svc.stats["gpu_hashes"] == len(set(msgs))
    # a repeat is answered from the memo, no launch and no reference call
    assert svc.digest(msgs[5]) == keccak256(msgs[5])
    assert dev.keccak_launches == 1 and calls["n"] == 0


def test_small_batches_use_reference_and_no_device_falls_back():
    ref, calls = _reference_counter()
    dev = FakeDevice()
    svc = KeccakService(device=dev, reference=ref, min_batch=64)
    assert svc.hash_many([b"a", b"b"]) == [keccak256(b"a"), keccak256(b"b")]
    assert calls["n"] == 2 and getattr(dev, "keccak_launches", 0) == 0
    svc2 = KeccakService(device=None, reference=ref, min_batch=1)
    assert svc2.hash_many([b"x"] * 3) == [keccak256(b"x")] * 3
    assert calls["n"] == 3
    with pytest.raises(RuntimeError):
        KeccakService(device=None, reference=None).digest(b"y")


def _reference_replace(txs, preimage, code_bytecode=None):
    """solver.py:128-164, one find_concrete_keccak per replaced window."""
    for tx in txs:
        if HASH_MATCHER not in tx["input"]:
            continue
        s_index = len(code_bytecode) + 2 if code_bytecode is not None and code_bytecode in tx["input"] else 10
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i:i + 64]
            if HASH_MATCHER not in data_slice or len(data_slice) != 64:
                continue
            p = preimage(int(data_slice, 16))
            if p is None:
                continue
            size, value = p
            h = keccak256(value.to_bytes(size // 8, "big")).hex()
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i:64 + i], h)


def _placeholder(rng):
    # the shape of a keccak UF value inside its interval: "ffffff..." prefixed, 64-aligned
    return (int("ffffffff" + "".join(rng.choice("0123456789abcdef") for _ in range(56)), 16) >> 6) << 6


@pytest.mark.parametrize("seed", range(6))
def test_replace_with_actual_sha_identical_to_reference(seed):
    rng = random.Random(seed)
    holders = [_placeholder(rng) for _ in range(5)]
    pre = {h: (rng.choice([256, 512, 160]), rng.getrandbits(160)) for h in holders[:4]}   # holders[4]: unknown
    code = "6080604052" * 3

    def make():
        txs = []
        for t in range(4):
            words = []
            for _ in range(rng.randint(0, 5)):
                r = rng.random()
                words.append("%064x" % (rng.choice(holders) if r < 0.6 else rng.getrandbits(256)))
            head = code if t == 0 and seed % 2 else ""
            txs.append({"input": "0x" + head + "a9059cbb" + "".join(words)})
        return txs

    state = rng.getstate()
    a = make()
    rng.setstate(state)
    b = make()
    assert a == b
    evals = {"n": 0}

    def preimage(v):
        evals["n"] += 1
        return pre.get(v)

    dev = FakeDevice()
    svc = KeccakService(device=dev, reference=keccak256, min_batch=1)
    code_bc = code if seed % 2 else None
    replace_with_actual_sha(a, preimage, svc, code_bc)
    _reference_replace(b, lambda v: pre.get(v), code_bc)
    assert a == b
    assert getattr(dev, "keccak_launches", 0) <= 1
