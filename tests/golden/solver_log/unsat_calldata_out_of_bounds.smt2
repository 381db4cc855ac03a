; expect: unsat
; synthetic --solver-log dump (tests/make_solver_log_corpus.py)
(declare-fun |0_calldatasize| () (_ BitVec 256))
(declare-fun |0_calldata| () (Array (_ BitVec 256) (_ BitVec 8)))
(assert (= (ite (bvslt #x0000000000000000000000000000000000000000000000000000000000000033 |0_calldatasize|) (select |0_calldata| #x0000000000000000000000000000000000000000000000000000000000000033) #x00) #x01))
(assert (= |0_calldatasize| #x0000000000000000000000000000000000000000000000000000000000000032))
(check-sat)
