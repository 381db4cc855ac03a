; expect: unsat
; synthetic --solver-log dump (tests/make_solver_log_corpus.py)
(declare-fun |a| () (_ BitVec 160))
(declare-fun |keccak256_160| ((_ BitVec 160)) (_ BitVec 256))
(declare-fun |keccak256_160-1| ((_ BitVec 256)) (_ BitVec 160))
(assert (let ((a!1 (|keccak256_160| |a|))) (let ((a!2 (= (|keccak256_160-1| a!1) |a|))) (and true (and a!2 (or (and a!2 (bvule #xfffffffffffffffffffffffffffffb5f425e64931f886225fdab9e36684d9d1a a!1) (bvult a!1 #xfffffffffffffffffffffffffffffb5f4b1477a6db3430525fddd8fb1c01771b) (= (bvurem a!1 #x0000000000000000000000000000000000000000000000000000000000000040) #x0000000000000000000000000000000000000000000000000000000000000000)) false))))))
(assert (= #x000000000000000000000000000000000000000000000000000000000000000a (|keccak256_160| |a|)))
(check-sat)
