"""Per-kernel timing of the records -> pairs pipeline on config3's records.

Each argument sets KARMA_DBG for one timed group of 3 runs (0 = production; a
debug build may read other values).  Only kernel times are printed.
Usage (GPU box): python tools/ablate.py [values...]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from karma_amd import _lib, engine  # noqa: E402

seed, n, f = 3, 200_000, 100_000_000
genes = engine.synth_genes(seed, n)
rec = engine.synth_records(seed, n, 0, f, True, genes=genes)
ctx = _lib.Context(0)
dev = _lib.DevBuf.from_numpy(ctx, rec.view(np.int64).reshape(-1))
out = {}
for d in (sys.argv[1:] or ["0"]):
    os.environ["KARMA_DBG"] = d
    p = engine.Pairs.from_records(ctx, None, n, device_ptr=dev.ptr, n_records=len(rec))
    p.close()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(3):
        p = engine.Pairs.from_records(ctx, None, n, device_ptr=dev.ptr, n_records=len(rec))
        p.close()
    ctx.sync()
    k = {name: round(v[0] / 3, 4) for name, v in ctx.timing_read().items()}
    ctx.timing(False)
    out[d] = k
    print(d, json.dumps(k), flush=True)
