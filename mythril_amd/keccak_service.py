"""Batched Keccak-256 service (§8a rows A7 and A12).

Mythril hashes concrete data one message at a time with pysha3:

* ``sha3`` (``mythril/support/support_utils.py:50-59``);
* ``get_code_hash`` (``support_utils.py:31-47``, ``lru_cache(2**10)``);
* ``KeccakFunctionManager.find_concrete_keccak``
  (``laser/ethereum/function_managers/keccak_function_manager.py:57-69``), which
  LASER's SHA3 instruction reaches through ``create_keccak`` (``:95-107``);
* ``_replace_with_actual_sha`` (``mythril/analysis/solver.py:128-164``), which
  looks at every 64-hex-digit window of every transaction input of an issue and
  swaps placeholder hashes for the real Keccak of their preimage.

This module keeps those functions' signatures, argument meaning and results,
and answers them from a digest memo that batched launches of the Keccak kernel
(``mg_keccak256``, ``csrc/mw_keccak.h``) fill:

* ``KeccakService.hash_many(msgs)``: the distinct messages that are not yet
  memoised go to the device in ONE launch when there are at least
  ``min_batch`` of them.  Below that the reference's own ``sha3`` answers,
  because one launch costs tens of microseconds and one pysha3 call about one.
* ``sha3`` / ``find_concrete_keccak`` / ``get_code_hash``: memo first, else
  the reference function.  The results are unchanged either way.
* ``prefetch_storage_slots``: at each LaserEVM transaction boundary the
  plugin hashes the likely concrete preimages of the next transaction's SHA3
  instructions (mapping entries and array bases of the actors and the
  contract, low slots) in ONE launch, so LASER's one-at-a-time hashing then
  hits the memo.
* ``replace_with_actual_sha``: a restatement of ``solver.py:128-164``.  It first
  collects the preimage of every window of the unmodified inputs and hashes
  them all in one launch, then runs the reference's loop.  A window that only
  appears after an earlier replacement misses the memo and is hashed on its
  own, so the output is identical.

When the HIP library or a device is unavailable, every call goes to the
reference functions (never to this repository's oracle).
"""
from __future__ import annotations

import logging
import os
from typing import Callable, Dict, Iterable, List, Optional, Sequence

log = logging.getLogger(__name__)

HASH_MATCHER = "fffffff"      # KeccakFunctionManager.hash_matcher (keccak_function_manager.py:37)
MEMO_MAX = 1 << 20            # digests kept (32 B each + the key)


class KeccakService:
    """Digest memo in front of the batched Keccak kernel.

    ``device`` is a ``runtime.Device`` (or anything with its ``keccak256``
    method); ``reference`` is the reference's one-message ``sha3(bytes) ->
    bytes``, used below ``min_batch`` and when no device is available.
    """

    def __init__(self, device=None, reference: Optional[Callable[[bytes], bytes]] = None,
                 min_batch: int = int(os.environ.get("MYTHRIL_AMD_KECCAK_MIN_BATCH", "64"))):
        self.device = device
        self.reference = reference
        self.min_batch = min_batch
        self.memo: Dict[bytes, bytes] = {}
        self.stats = {"requests": 0, "memo_hits": 0, "launches": 0, "gpu_hashes": 0, "reference_hashes": 0}
        # one record per batch of more than one message (a prefetch, a
        # _replace_with_actual_sha): its size, the digests it had to compute,
        # and whether the device computed them (tests/test_keccak_batches.py)
        self.batches: List[Dict[str, object]] = []

    # -- batch entry -------------------------------------------------------
    def hash_many(self, msgs: Iterable[bytes]) -> List[bytes]:
        msgs = [bytes(m) for m in msgs]
        self.stats["requests"] += len(msgs)
        todo = list(dict.fromkeys(m for m in msgs if m not in self.memo))
        self.stats["memo_hits"] += len(msgs) - len(todo)
        if todo:
            if len(self.memo) + len(todo) > MEMO_MAX:
                self.memo.clear()
            on_device = self.device is not None and len(todo) >= self.min_batch
            if on_device:
                digests, _ = self.device.keccak256(todo)
                self.stats["launches"] += 1
                self.stats["gpu_hashes"] += len(todo)
            else:
                digests = [self._reference(m) for m in todo]
            self.memo.update(zip(todo, digests))
        if len(msgs) > 1 and len(self.batches) < 4096:
            self.batches.append({"size": len(msgs), "new": len(todo), "device": bool(todo) and on_device})
        return [self.memo[m] for m in msgs]

    def digest(self, msg: bytes) -> bytes:
        return self.hash_many([msg])[0]

    def _reference(self, m: bytes) -> bytes:
        if self.reference is None:
            raise RuntimeError("keccak service: no device and no reference sha3")
        self.stats["reference_hashes"] += 1
        return self.reference(m)

    # -- the reference's entry points, same arguments and results ----------
    def sha3(self, value) -> bytes:
        """support_utils.py:50-59: strings starting ``0x`` go to ``bytes.fromhex``
        WHOLE (``:53-54``), so they raise ``ValueError`` on the ``x`` exactly
        as the reference does; other strings are UTF-8 encoded, bytes hashed as
        they are."""
        if type(value) == str:
            value = bytes.fromhex(value) if value[:2] == "0x" else value.encode()
        return self.digest(bytes(value))

    def get_code_hash(self, code) -> str:
        """support_utils.py:31-47: tuples (symbolic code) hash to ``str(hash())``,
        undecodable hex to ``""``."""
        if type(code) == tuple:
            return str(hash(code))
        code = code[2:] if code[:2] == "0x" else code
        try:
            data = bytes.fromhex(code)
        except ValueError:
            log.debug("Unable to change the bytecode to bytes. Bytecode: %s", code)
            return ""
        return "0x" + self.digest(data).hex()

    def find_concrete_keccak_int(self, value: int, size_bits: int) -> int:
        """keccak_function_manager.py:57-69 on plain integers: the data is the
        big-endian ``size_bits // 8``-byte encoding of ``value``."""
        return int.from_bytes(self.digest(value.to_bytes(size_bits // 8, "big")), "big")

    def prefetch_values(self, preimages: Iterable[tuple]) -> int:
        """Hash many ``(size_bits, value)`` preimages in one launch (memo fill)."""
        msgs = [v.to_bytes(s // 8, "big") for s, v in preimages]
        self.hash_many(msgs)
        return len(msgs)

    def prefetch_storage_slots(self, keys: Iterable[int], slots: Iterable[int]) -> int:
        """Speculative batch at a LaserEVM transaction boundary: the preimages
        Solidity's storage layout hashes with concrete data — mapping entries
        ``keccak(pad32(key) ++ pad32(slot))`` (``instructions.py:1004-1042``
        reaching ``find_concrete_keccak``) and dynamic-array bases
        ``keccak(pad32(slot))`` — for the keys LASER's transactions use
        (the actor addresses, ``transaction/symbolic.py:29-40``, and the
        contract's address) and the low slots.  One launch fills the memo; the
        SHA3 instructions that follow are memo hits, the results unchanged."""
        keys = list(dict.fromkeys(int(k) for k in keys))
        slots = list(dict.fromkeys(int(sl) for sl in slots))
        pre = [(512, (k << 256) | sl) for k in keys for sl in slots] + [(256, sl) for sl in slots]
        return self.prefetch_values(pre)


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], preimage: Callable[[int], Optional[tuple]],
                            service: KeccakService, code_bytecode: Optional[str] = None) -> None:
    """``_replace_with_actual_sha`` (``mythril/analysis/solver.py:128-164``) with
    its hashes batched.

    ``preimage(window_value)`` returns ``(size_bits, preimage_value)`` for a
    window whose value is a known symbolic hash, else None: in the reference
    the last ``size`` of ``get_concrete_hash_data(model)`` whose list holds the
    value, and ``model.eval(inverse(value))`` (``solver.py:146-155``).  It is
    evaluated at most once per distinct window.  Mutates the transactions' "input"
    strings exactly as the reference does.
    """
    known: Dict[str, Optional[tuple]] = {}

    def lookup(window: str) -> Optional[tuple]:
        if window not in known:
            known[window] = preimage(int(window, 16))
        return known[window]

    def start(tx) -> int:
        if code_bytecode is not None and code_bytecode in tx["input"]:
            return len(code_bytecode) + 2
        return 10

    def windows(tx) -> Iterable[tuple]:
        s = start(tx)
        for i in range(s, len(tx["input"])):
            w = tx["input"][i:i + 64]
            if len(w) == 64 and HASH_MATCHER in w:
                yield s, i, w

    txs = [tx for tx in concrete_transactions if HASH_MATCHER in tx["input"]]
    # one launch for every preimage visible in the unmodified inputs
    service.prefetch_values({p for tx in txs for _, _, w in windows(tx) for p in [lookup(w)] if p is not None})
    for tx in txs:
        s = start(tx)
        for i in range(s, len(tx["input"])):
            w = tx["input"][i:i + 64]
            if len(w) != 64 or HASH_MATCHER not in w:
                continue
            p = lookup(w)
            if p is None:
                continue
            size, value = p
            digest = service.find_concrete_keccak_int(value, size)
            tx["input"] = tx["input"][:s] + tx["input"][s:].replace(w, "%064x" % digest)


# -- installation into a Mythril process ------------------------------------
_service: Optional[KeccakService] = None


def service() -> Optional[KeccakService]:
    return _service


def install(device=None) -> bool:
    """Rebind Mythril's concrete-keccak sites to the service (used by the
    plugin next to ``model.install``).  ``device`` defaults to the witness
    engine's device; without one the service still memoises but every miss
    goes to the reference ``sha3``."""
    global _service
    try:
        import mythril.analysis.solver as a_solver
        import mythril.support.support_utils as su
        from mythril.laser.ethereum.function_managers import keccak_function_manager as kfm_mod
        from mythril.laser.smt import symbol_factory
    except ImportError:
        return False
    if _service is not None:
        return True
    if device is None:
        from . import model
        eng = model.engine()
        device = eng.dev if eng is not None else None
    ref_sha3 = su.sha3
    svc = KeccakService(device=device, reference=lambda m: ref_sha3(m))
    _service = svc

    def find_concrete_keccak(data):
        return symbol_factory.BitVecVal(svc.find_concrete_keccak_int(data.value, data.size()), 256)

    kfm_mod.KeccakFunctionManager.find_concrete_keccak = staticmethod(find_concrete_keccak)
    kfm_mod.sha3 = svc.sha3
    # get_code_hash (support_utils.py:31-47) at its import sites: EXTCODEHASH and
    # CREATE2 (instructions.py:62,1292-1300,1775-1788), EVMContract (evmcontract.py:9)
    su.get_code_hash = svc.get_code_hash
    for site in ("mythril.laser.ethereum.instructions", "mythril.ethereum.evmcontract"):
        try:
            mod = __import__(site, fromlist=["get_code_hash"])
            if hasattr(mod, "get_code_hash"):
                mod.get_code_hash = svc.get_code_hash
        except ImportError:
            pass
    manager = kfm_mod.keccak_function_manager

    def _replace(concrete_transactions, model, code=None):
        concrete = manager.get_concrete_hash_data(model)

        def preimage(v):
            hit = None
            for size in concrete:
                if v in concrete[size]:
                    _, inverse = manager.store_function[size]
                    hit = (size, model.eval(inverse(symbol_factory.BitVecVal(v, 256)).raw).as_long())
            return hit

        replace_with_actual_sha(concrete_transactions, preimage, svc,
                                code.bytecode if code is not None else None)

    a_solver._replace_with_actual_sha = _replace
    log.info("MI355X keccak service installed (device: %s)", device is not None)
    return True
