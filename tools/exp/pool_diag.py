import sys, collections
from mythril_amd.smt2 import parse_file, to_smt2
from mythril_amd.engine import prepare
from tests.helpers import oracle_models
from oracle.dag_eval import eval_nodes
N=int(sys.argv[1]) if len(sys.argv)>1 else 2048
for f in sys.argv[2:] or ["c2_token_transfer_ok","c2_token_transfer_underflow","c4_wallet_onlyowner"]:
    s=parse_file(f"tests/golden/solver_log/{f}.smt2")
    q=prepare(s.asserts, s.ctx)
    conj=q.lowered.conjuncts
    ms=oracle_models(q.program, 0x5EED0002, 0, N)
    fails=collections.Counter(); first=None
    for j,m in enumerate(ms):
        vals=eval_nodes(conj, m)
        bad=[i for i,c in enumerate(conj) if not vals[c.id]]
        for i in bad: fails[i]+=1
        if not bad and first is None: first=j
    print("==",f,"first witness",first, "conj", len(conj))
    for i,c in fails.most_common(6):
        print(i, c, to_smt2([conj[i]])[-260:].replace("\n"," "))
