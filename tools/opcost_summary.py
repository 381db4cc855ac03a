#!/usr/bin/env python3
"""Per-bytecode-instruction counters from tools/interp_opcost.py's PMC pass: python tools/opcost_summary.py TAG (reads gpurun_out/TAG/opcost_pmc)."""
import csv, collections, sys
tag=sys.argv[1]
rows=collections.defaultdict(dict)
for row in csv.DictReader(open(f'gpurun_out/{tag}/opcost_pmc/run_counter_collection.csv')):
    if 'mw_search' in row['Kernel_Name']:
        rows[int(row['Dispatch_Id'])][row['Counter_Name']]=float(row['Counter_Value'])
names=["CHECK","CHECK_IMPEQ_regs","CHECK_IMPEQ_const","N_ADD","N_EQN","MOV_N","N_EQ_wide","W_ADD","W_AND","LEAF_N","LEAF_W"]
ids=sorted(rows)
for k,name in enumerate(names):
    if 2*k+1>=len(ids): break
    r=rows[ids[2*k+1]]
    rep=500 if name.startswith('LEAF') else 2000
    w=r['SQ_WAVES']; chunks=(1<<18)//64/w
    per=lambda c: r[c]/w/chunks/rep
    print(f"{name:18s} VALU {per('SQ_INSTS_VALU'):6.1f} SALU {per('SQ_INSTS_SALU'):6.1f} SMEM {per('SQ_INSTS_SMEM'):5.2f} BR {per('SQ_INSTS_BRANCH'):5.1f} cyc {per('SQ_WAVE_CYCLES'):7.1f}")
