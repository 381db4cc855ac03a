"""Mythril plugin: installs the witness engine behind ``get_model`` and batches
LaserEVM's reachability queries.

Discovered through the ``mythril.plugins`` entry point
(``mythril/plugin/discovery.py:17-21,44-57``) and, being
``plugin_default_enabled``, loaded when the CLI is imported
(``mythril/interfaces/cli.py:37``, ``mythril/plugin/loader.py:71-78``).
``__call__`` builds the LASER plugin (``mythril/laser/plugin/builder.py``) whose
``initialize(vm)`` (``laser/plugin/interface.py:18``) rebinds ``get_model`` and
registers two batching hooks:

* ``stop_sym_trans`` (``svm.py:243-245``): right before the next
  transaction's reachability prune over ``open_states`` (``svm.py:216-223``)
  every open state's constraint set is searched in ONE launch (and, opt-in,
  likely concrete Keccak preimages of the next transaction are hashed in one
  launch: see KECCAK_SPECULATION);
* a JUMPI post hook (``svm.py:_execute_post_hook``, run on each successor):
  the successors are queued, and the first per-step ``is_possible``
  (``svm.py:287-292``) searches the pair in one launch.

``is_possible`` then finds the confirmed witness in the memo.  Exploration
order is untouched.  It also installs the batched Keccak-256 service
(``keccak_service.install``) behind ``find_concrete_keccak`` and
``_replace_with_actual_sha``.
"""
from __future__ import annotations

import logging
import os

log = logging.getLogger(__name__)

try:  # Mythril is present in a real deployment; absent in this repo's CI
    from mythril.laser.plugin.interface import LaserPlugin as _LaserPlugin
    from mythril.plugin.interface import MythrilLaserPlugin as _MythrilLaserPlugin
    HAVE_MYTHRIL = True
except Exception:  # pragma: no cover - exercised only where mythril is installed
    _LaserPlugin = object
    _MythrilLaserPlugin = object
    HAVE_MYTHRIL = False


SLOTS = 16   # storage slots whose mapping entries / array bases are prefetched
# Speculative mapping-slot hashing at each transaction boundary, OFF by default:
# replayed in LASER's order over the corpus (tests/laser_replay.py), LASER made
# no concrete SHA3 request at all (sender_N is symbolic, so keccak(sender .
# slot) is the keccak256_512 UF, keccak_function_manager.py:104-114), so every
# speculated digest was wasted.  The memo still serves repeated concrete hashes.
KECCAK_SPECULATION = os.environ.get("MYTHRIL_AMD_KECCAK_SPECULATION", "0") == "1"


def storage_keys(symbolic_vm) -> list:
    """Concrete keys the next transaction's mapping lookups use: LASER's three
    actors (transaction/symbolic.py:29-40) and the open states' concrete
    account addresses."""
    keys = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
            0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]
    for ws in getattr(symbolic_vm, "open_states", []):
        for addr in getattr(ws, "accounts", {}) or {}:
            try:
                keys.append(int(getattr(addr, "value", addr)))
            except (TypeError, ValueError):
                pass
    return keys


class WitnessBatchingLaserPlugin(_LaserPlugin):
    """LASER plugin: rebinding + transaction-boundary batching."""

    def initialize(self, symbolic_vm) -> None:
        from . import keccak_service, model
        model.install()
        keccak_service.install()

        def prefetch_open_states():
            try:
                n = model.prefetch([s.constraints for s in symbolic_vm.open_states])
                log.info("witness engine: %d/%d open states witnessed in one launch", n,
                         len(symbolic_vm.open_states))
            except Exception as e:  # never disturb the analysis
                log.warning("witness engine prefetch skipped: %s", e)
            if KECCAK_SPECULATION:
                try:
                    svc = keccak_service.service()
                    if svc is not None:
                        svc.prefetch_storage_slots(storage_keys(symbolic_vm), range(SLOTS))
                except Exception as e:  # never disturb the analysis
                    log.debug("keccak prefetch skipped: %s", e)

        symbolic_vm.register_laser_hooks("stop_sym_trans", prefetch_open_states)

        def defer_successor(global_state):
            # svm.py:_execute_post_hook runs this on each JUMPI successor before
            # the per-step prune (svm.py:287-292) calls is_possible on them
            try:
                model.defer(global_state.world_state.constraints)
            except Exception as e:  # never disturb the analysis
                log.debug("witness engine: successor not deferred: %s", e)

        symbolic_vm.register_hooks("post", {"JUMPI": [defer_successor]})

        def report():
            log.info("witness engine stats: %s", model.STATS)
            if keccak_service.service() is not None:
                log.info("keccak service stats: %s", keccak_service.service().stats)

        symbolic_vm.register_laser_hooks("stop_sym_exec", report)


class MI355XWitnessEngine(_MythrilLaserPlugin):
    """``mythril.plugins`` entry point (see setup.py / INTEGRATION.md)."""

    author = "mythril-amd"
    name = "mi355x-witness-engine"
    plugin_license = "MIT"
    plugin_type = "Laser Plugin"
    plugin_version = "0.1.0"
    plugin_description = ("GPU witness search on AMD MI355X in front of z3 for feasibility-only "
                          "get_model queries; z3 re-checks every witness and answers every miss.")
    plugin_default_enabled = True

    def __init__(self, **kwargs):
        if HAVE_MYTHRIL:
            super().__init__(**kwargs)
        self.enabled = True
        # rebind as early as possible (before any state is explored)
        from . import model
        model.install()

    def __call__(self, *args, **kwargs):
        return WitnessBatchingLaserPlugin()
