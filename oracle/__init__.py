"""ORACLE — test infrastructure only.

CPU restatement of the reference's hot-path arithmetic, used exclusively as the
*checker* by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg.  Nothing under ``mythril_amd/`` may import it; the
product path (HIP kernels behind the C-ABI) must fail loudly rather than fall
back to anything in here.

What it restates (the reference is pure Python over z3 — SURVEY.md §0, §8c):

* ``bvsem``   — SMT-LIB 2.6 / z3 semantics of every bitvector/Bool op that
  Mythril's ``mythril/laser/smt`` wrappers emit (z3-solver is a third-party
  dependency, ``requirements.txt:35`` ``z3-solver>=4.8.8.0``, unpinned and
  absent here; we restate its published semantics, the SMT-LIB 2.6
  FixedSizeBitVectors theory).
* ``dag_eval`` — model evaluation of a constraint DAG under an assignment
  (what ``z3.ModelRef.eval`` / ``substitute+simplify`` compute).
* ``keccak``  — Keccak-256 with the original 0x01 padding (what
  ``_pysha3.keccak_256`` computes, ``mythril/support/support_utils.py:50-59``;
  pysha3 is unpinned, ``requirements.txt:23``).
* ``philox``  — Philox4x32-10 (Salmon et al., SC'11), the candidate generator.
* ``evm``     — a minimal concrete EVM that lowers opcodes onto ``bvsem`` the
  way ``mythril/laser/ethereum/instructions.py`` does, so the reference's
  VMTests post-storage values pin ``bvsem``.
* ``c/``      — the same DAG semantics in plain C (+OpenMP) for large parity
  sweeps and the CPU baseline.

Parity is pinned by the reference's own known-answer data:
EIP-145 shift vectors (``tests/instructions/{shl,shr,sar}_test.py``), the
VMTests post-storage values (``tests/laser/evm_testsuite/VMTests``), the
``vmSha3Test`` Keccak vectors, the empty-keccak constant
(``keccak_function_manager.py:87-93``) and the keccak/calldata sat/unsat
expectations (``tests/laser/keccak_tests.py``, ``tests/laser/state/calldata_test.py``),
committed as fixtures under ``tests/golden/``.  z3-level parity (``model.eval``
on arbitrary DAGs) is unpinned here: z3 is not installed in this image.
"""
