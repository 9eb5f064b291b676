import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from karma_amd import engine
from oracle import oracle
def orc(rec, n):
    r = rec.astype(np.int64); st = np.flatnonzero(np.r_[True, r[1:,0] != r[:-1,0]])
    return oracle.graph_groups(np.r_[st, len(r)], r[:,1], None, None, n, dedup=True)
for (seed, n, lo, hi) in [(23, 1400, 0, 60000), (23, 1400, 60000, 120000), (5, 300, 0, 20000), (2, 20000, 0, 400000)]:
    genes = engine.synth_genes(seed, n)
    rec = engine.synth_records(seed, n, lo, hi, True, genes=genes)
    e = engine.graph_from_records(rec, n)
    o = orc(rec, n)
    ka = set(zip(e.a.tolist(), e.b.tolist())); ko = set(zip(o['a'].tolist(), o['b'].tolist()))
    tot_ok = np.array_equal(e.totals, o['totals'])
    print(seed, n, lo, len(rec), 'E', len(e.a), len(o['a']), 'extra', sorted(ka-ko)[:8], 'missing', sorted(ko-ka)[:8], 'tot_ok', tot_ok)
    if not tot_ok:
        d = np.flatnonzero(e.totals != o['totals']); print('  tot diff', d[:10], e.totals[d[:10]], o['totals'][d[:10]])
