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
    # support_utils.py:53-54 hands "0x..." strings to bytes.fromhex whole: the
    # reference raises ValueError on the "x", and so does the service
    for s in ("0x", "0x0000000000", "0xab"):
        with pytest.raises(ValueError):
            svc.sha3(s)
        with pytest.raises(ValueError):
            bytes.fromhex(s)            # the reference's own operation
    assert svc.sha3("0000000000") == keccak256(b"0000000000")   # no prefix: UTF-8 text, as the reference
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


def test_install_rebinds_reference_sites(monkeypatch):
    """keccak_service.install() against stand-ins for the Mythril modules it
    touches (mythril is not importable here): find_concrete_keccak and
    _replace_with_actual_sha are rebound and give the reference's results."""
    import sys
    import types

    from mythril_amd import keccak_service, model
    from mythril_amd.engine import WitnessEngine

    class BitVecVal:
        def __init__(self, v, size):
            self.value, self._size = v, size
            self.raw = ("val", v)

        def size(self):
            return self._size

    sf = types.SimpleNamespace(BitVecVal=BitVecVal)

    class Inverse:
        def __call__(self, x):
            return types.SimpleNamespace(raw=("inv", x.value))

    class KFM:
        @staticmethod
        def find_concrete_keccak(data):
            raise AssertionError("reference path must not run")

    manager = KFM()
    placeholder = 0xFFFFFFFF00000000000000000000000000000000000000000000000000000040
    preimage = 0xDEADBEEF
    manager.store_function = {256: (None, Inverse())}
    manager.get_concrete_hash_data = lambda m: {256: [placeholder]}

    class Z3Model:
        def eval(self, raw):
            assert raw == ("inv", placeholder)
            return types.SimpleNamespace(as_long=lambda: preimage)

    mods = {
        "mythril": types.ModuleType("mythril"),
        "mythril.analysis": types.ModuleType("mythril.analysis"),
        "mythril.analysis.solver": types.SimpleNamespace(_replace_with_actual_sha=None),
        "mythril.support": types.ModuleType("mythril.support"),
        "mythril.support.support_utils": types.SimpleNamespace(sha3=keccak256),
        "mythril.laser": types.ModuleType("mythril.laser"),
        "mythril.laser.smt": types.SimpleNamespace(symbol_factory=sf),
        "mythril.laser.ethereum": types.ModuleType("mythril.laser.ethereum"),
        "mythril.laser.ethereum.function_managers": types.ModuleType("mythril.laser.ethereum.function_managers"),
        "mythril.laser.ethereum.function_managers.keccak_function_manager":
            types.SimpleNamespace(KeccakFunctionManager=KFM, keccak_function_manager=manager, sha3=None),
    }
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    mods["mythril.laser.ethereum.function_managers"].keccak_function_manager = \
        mods["mythril.laser.ethereum.function_managers.keccak_function_manager"]
    monkeypatch.setattr(keccak_service, "_service", None)
    monkeypatch.setattr(model, "_engine", WitnessEngine(dev=FakeDevice(), budget=1 << 10))
    monkeypatch.setattr(model, "_engine_failed", False)
    assert keccak_service.install()
    svc = keccak_service.service()
    assert svc is not None and svc.device is model._engine.dev
    h = KFM.find_concrete_keccak(BitVecVal(5, 256))
    assert h.value == int.from_bytes(keccak256((5).to_bytes(32, "big")), "big") and h.size() == 256
    kmod = mods["mythril.laser.ethereum.function_managers.keccak_function_manager"]
    assert kmod.sha3(b"").hex() == EMPTY
    with pytest.raises(ValueError):
        kmod.sha3("0x")
    txs = [{"input": "0x" + "a9059cbb" + "%064x" % placeholder + "%064x" % 7}]
    mods["mythril.analysis.solver"]._replace_with_actual_sha(txs, Z3Model())
    assert txs[0]["input"] == "0x" + "a9059cbb" + keccak256(preimage.to_bytes(32, "big")).hex() + "%064x" % 7


def test_transaction_boundary_prefetch_then_memo_hits(monkeypatch):
    """the plugin's stop_sym_trans hook (svm.py:243-245) hashes
    the next transaction's likely storage preimages in ONE mg_keccak256 launch;
    LASER's later one-at-a-time find_concrete_keccak calls for mapping entries
    of the actors are memo hits (no launch, no reference call), with the
    reference's digests.  get_code_hash is rebound at its import sites."""
    import sys
    import types

    from mythril_amd import keccak_service, model, mythril_plugin
    from mythril_amd.engine import WitnessEngine

    class BitVecVal:
        def __init__(self, v, size):
            self.value, self._size = v, size

        def size(self):
            return self._size

    class KFM:
        @staticmethod
        def find_concrete_keccak(data):
            raise AssertionError("reference path must not run")

    ref, calls = _reference_counter()
    instr = types.SimpleNamespace(get_code_hash=None)
    evmc = types.SimpleNamespace(get_code_hash=None)
    mods = {
        "mythril": types.ModuleType("mythril"),
        "mythril.analysis": types.ModuleType("mythril.analysis"),
        "mythril.analysis.solver": types.SimpleNamespace(_replace_with_actual_sha=None),
        "mythril.support": types.ModuleType("mythril.support"),
        "mythril.support.support_utils": types.SimpleNamespace(sha3=ref, get_code_hash=None),
        "mythril.laser": types.ModuleType("mythril.laser"),
        "mythril.laser.smt": types.SimpleNamespace(symbol_factory=types.SimpleNamespace(BitVecVal=BitVecVal)),
        "mythril.laser.ethereum": types.ModuleType("mythril.laser.ethereum"),
        "mythril.laser.ethereum.instructions": instr,
        "mythril.ethereum": types.ModuleType("mythril.ethereum"),
        "mythril.ethereum.evmcontract": evmc,
        "mythril.laser.ethereum.function_managers": types.ModuleType("mythril.laser.ethereum.function_managers"),
        "mythril.laser.ethereum.function_managers.keccak_function_manager":
            types.SimpleNamespace(KeccakFunctionManager=KFM, keccak_function_manager=KFM(), sha3=None),
    }
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    dev = FakeDevice()
    monkeypatch.setattr(keccak_service, "_service", None)
    monkeypatch.setattr(model, "_engine", WitnessEngine(dev=dev, budget=1 << 10))
    monkeypatch.setattr(model, "_engine_failed", False)
    monkeypatch.setattr(model, "install", lambda: True)
    assert keccak_service.install()
    assert instr.get_code_hash("0x6001") == "0x" + keccak256(bytes.fromhex("6001")).hex()
    assert evmc.get_code_hash == instr.get_code_hash

    class VM:
        def __init__(self):
            self.laser, self.post, self.open_states = {}, {}, []

        def register_laser_hooks(self, kind, hook):
            self.laser.setdefault(kind, []).append(hook)

        def register_hooks(self, kind, hooks):
            pass

    vm = VM()
    monkeypatch.setattr(mythril_plugin, "KECCAK_SPECULATION", True)   # opt-in (off by default)
    mythril_plugin.WitnessBatchingLaserPlugin().initialize(vm)
    n_before = getattr(dev, "keccak_launches", 0)
    ref_before = calls["n"]
    vm.laser["stop_sym_trans"][0]()        # transaction boundary
    assert dev.keccak_launches == n_before + 1
    svc = keccak_service.service()
    hashed = svc.stats["gpu_hashes"]
    assert hashed >= 3 * mythril_plugin.SLOTS
    # LASER's SHA3 on balances[msg.sender] (slot 0) and allowance-style slot 3
    for actor in (0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE):
        for slot in (0, 3):
            v = (actor << 256) | slot
            h = KFM.find_concrete_keccak(BitVecVal(v, 512))
            assert h.value == int.from_bytes(keccak256(v.to_bytes(64, "big")), "big")
    assert dev.keccak_launches == n_before + 1 and calls["n"] == ref_before
    assert svc.stats["memo_hits"] >= 4
    # a second boundary re-requests the same preimages: all memo hits, no launch
    vm.laser["stop_sym_trans"][0]()
    assert dev.keccak_launches == n_before + 1
