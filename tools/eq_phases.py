#!/usr/bin/env python3
"""Where the eq path's time goes (GPU box): config 3's eq classes through
karma_graph_eq, phase by phase (H2D + kernels, edges, D2H), next to plain
pageable H2D / D2H copies of the same byte counts through torch.  Prints one
JSON line.  Diagnostic only.

  python tools/eq_phases.py [--config config3] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def best(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    from karma_amd import _lib, engine

    seed, n, f, paired, _ = bench.CONFIGS[a.config]
    genes = engine.synth_genes(seed, n)
    cls_off, members, counts = engine.synth_eq_classes(seed, n, 0, f, paired, genes=genes)
    skip = (np.diff(cls_off) == 1).astype(np.uint8)
    ctx = _lib.Context(0)
    out = {"classes": int(len(counts)), "members": int(len(members))}
    ins = [np.ascontiguousarray(x) for x in (cls_off, members, counts, skip)]
    out["h2d_bytes"] = int(sum(x.nbytes for x in ins))

    def whole():
        return engine.graph_from_eq(cls_off, members, counts, skip, n, ctx=ctx)

    e = whole()
    E = len(e.a)
    out["edges"] = E
    out["d2h_bytes"] = int(E * 32 + n * 8)
    out["whole_ms"] = best(whole, a.reps)
    out["whole_ordered_ms"] = best(lambda: engine.graph_from_eq_ordered(cls_off, members, counts, skip, n, ctx=ctx),
                                   a.reps)
    cq = engine.eq_compact(cls_off, counts, skip)
    c_sz, c_mem, c_cnt = (_lib.pinned_empty(len(x), x.dtype) for x in (cq[0], members, cq[1]))
    c_sz[:], c_mem[:], c_cnt[:] = cq[0], members, cq[1]
    out["compact_h2d_bytes"] = int(c_sz.nbytes + c_mem.nbytes + c_cnt.nbytes)
    out["whole_compact_pinned_ms"] = best(
        lambda: engine.graph_from_eq_compact_ordered(c_sz, c_mem, c_cnt, n, ctx=ctx), a.reps)
    out["whole_compact_pageable_ms"] = best(
        lambda: engine.graph_from_eq_compact_ordered(cq[0], members, cq[1], n, ctx=ctx), a.reps)

    def from_eq():
        p = engine.Pairs.from_eq(ctx, cls_off, members, counts, skip, n)
        p.close()

    out["from_eq_ms"] = best(from_eq, a.reps)

    def upto_edges():
        p = engine.Pairs.from_eq(ctx, cls_off, members, counts, skip, n)
        ed = p.edges(_lib.KARMA_MODE_EQ, n)
        ed.close()
        p.close()

    out["upto_edges_ms"] = best(upto_edges, a.reps)
    # plain copies of the same bytes (pageable host memory, torch's path)
    dev = torch.empty(out["h2d_bytes"], dtype=torch.uint8, device="cuda")
    host = [torch.from_numpy(x.view(np.uint8).reshape(-1)) for x in ins]

    def h2d():
        o = 0
        for h in host:
            dev[o:o + h.numel()].copy_(h, non_blocking=False)
            o += h.numel()
        torch.cuda.synchronize()

    out["h2d_pageable_ms"] = best(h2d, a.reps)
    outs = [np.zeros(E * 4, np.uint8), np.zeros(E * 4, np.uint8), np.zeros(E * 8, np.uint8),
            np.zeros(E * 8, np.uint8), np.zeros(E * 8, np.uint8), np.zeros(n * 8, np.uint8)]
    dsrc = torch.empty(out["d2h_bytes"], dtype=torch.uint8, device="cuda")

    def d2h():
        o = 0
        for h in outs:
            torch.from_numpy(h).copy_(dsrc[o:o + h.size])
            o += h.size

    out["d2h_pageable_ms"] = best(d2h, a.reps)
    pin = torch.empty(out["d2h_bytes"], dtype=torch.uint8).pin_memory()

    def d2h_pinned():
        pin.copy_(dsrc, non_blocking=True)
        torch.cuda.synchronize()

    out["d2h_pinned_ms"] = best(d2h_pinned, a.reps)
    ctx.timing(True)
    ctx.timing_reset()
    engine.graph_from_eq_compact_ordered(c_sz, c_mem, c_cnt, n, ctx=ctx)
    out["kernels_ms"] = {k: round(ms, 4) for k, (ms, nl) in sorted(ctx.timing_read().items())}
    ctx.timing(False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
