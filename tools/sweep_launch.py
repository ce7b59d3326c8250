#!/usr/bin/env python3
"""Interleaved in-process sweep of the streaming kernel's launch variants (blocks/CU, unroll, variant)
on the bench workload.  Every configuration is timed with HIP events in each of R rounds; the rounds
interleave all configurations (one process, one device) so drift hits them alike.  Outputs of every
configuration are compared bit-for-bit on a sample against the default configuration."""

import argparse
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=float, default=1e9)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--bpc", default="2,4,8,16")
    ap.add_argument("--unroll", default="4,8,16")
    ap.add_argument("--variant", default="0,1,2,3")
    ap.add_argument("--mode", default="torch")
    ap.add_argument("--layout", choices=["rows", "tiled"], default="rows")
    ap.add_argument("--tile", default="1024,2048,4096", help="tiled layout: tile widths (elements)")
    ap.add_argument("--seg-pad", default="0", help="tiled layout: padding after each client segment (elements)")
    ap.add_argument("--tile-pad", default="0", help="tiled layout: padding after each tile (elements)")
    ap.add_argument("--row-skew", default="0", help="rows layout: byte skew added per client row (k * skew)")
    args = ap.parse_args()
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    K, P = args.clients, int(args.params)
    if args.layout == "tiled":
        return sweep_tiled(args, ctx, K, P)
    skews = [int(x) for x in args.row_skew.split(",")]
    smax = max(skews)
    rows = [ctx.alloc(P * 4 + K * smax + 256) for _ in range(K)]
    out = ctx.alloc(P * 4)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    op, fin = (1, 2) if args.mode == "torch" else (0, 1)
    idx = np.unique(np.random.default_rng(0).integers(0, P, 20000)).astype(np.uint64)
    configs = list(itertools.product([int(x) for x in args.bpc.split(",")], [int(x) for x in args.unroll.split(",")],
                                     [int(x) for x in args.variant.split(",")], skews))
    times = {c: [] for c in configs}
    ref = None
    alg = 4.0 * K * P + 4.0 * P
    filled = None
    for r in range(args.rounds):
        for c in configs:
            if filled != c[3]:
                ptrs = [b.ptr + k * c[3] for k, b in enumerate(rows)]
                for k, p in enumerate(ptrs):
                    ctx.fill_synthetic_f32(p, P, 1000, k, 0)
                ctx.sync()
                filled = c[3]
            ctx.set_launch(c[0], c[1])
            ctx.set_variant(c[2])
            ctx.accumulate(ptrs, ws, P, out.ptr, 0, 0, op, fin, cnt)  # warm
            ctx.timing_begin()
            for _ in range(args.reps):
                ctx.accumulate(ptrs, ws, P, out.ptr, 0, 0, op, fin, cnt)
            ms = ctx.timing_end() / args.reps
            times[c].append(ms)
            if r == 0:
                sample = ctx.gather_f32(out.ptr, idx)
                if ref is None:
                    ref = sample
                assert np.array_equal(sample.view(np.uint32), ref.view(np.uint32)), f"bits differ for {c}"
        print(f"round {r} done", file=sys.stderr, flush=True)
    res = []
    for c, t in times.items():
        med = float(np.median(t))
        res.append({"bpc": c[0], "unroll": c[1], "variant": c[2], "row_skew": c[3], "ms_median": round(med, 4), "ms_min": round(min(t), 4),
                    "GBps_median": round(alg / med / 1e6, 1), "frac_peak": round(alg / med / 1e6 / 8000, 4)})
    res.sort(key=lambda x: x["ms_median"])
    for x in res:
        print(json.dumps(x))


def sweep_tiled(args, ctx, K, P):
    from nvflare_amd.device import TiledLayout

    geoms = list(itertools.product([int(x) for x in args.tile.split(",")], [int(x) for x in args.seg_pad.split(",")],
                                   [int(x) for x in args.tile_pad.split(",")]))
    layouts = {g: TiledLayout(g[0], K, g[1], g[2]) for g in geoms}
    slab = ctx.alloc(max(l.slab_elems(P) for l in layouts.values()) * 4)
    out = ctx.alloc(P * 4)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    op, fin = (1, 2) if args.mode == "torch" else (0, 1)
    configs = list(itertools.product(geoms, [int(x) for x in args.bpc.split(",")], [int(x) for x in args.variant.split(",")],
                                     [int(x) for x in args.unroll.split(",")]))
    times = {c: [] for c in configs}
    alg = 4.0 * K * P + 4.0 * P
    filled = None
    for r in range(args.rounds):
        for c in configs:
            geom, bpc, var, unr = c
            lay = layouts[geom]
            if filled != geom:
                ctx.fill_synthetic_tiled_f32(slab.ptr, lay, P, 1000, 0)
                ctx.sync()
                filled = geom
            ctx.set_launch(bpc, unr)
            ctx.set_variant(var)
            ctx.accumulate_tiled(slab.ptr, lay, list(range(K)), ws, P, out.ptr, op, fin, cnt)
            ctx.timing_begin()
            for _ in range(args.reps):
                ctx.accumulate_tiled(slab.ptr, lay, list(range(K)), ws, P, out.ptr, op, fin, cnt)
            times[c].append(ctx.timing_end() / args.reps)
        print(f"round {r} done", file=sys.stderr, flush=True)
    res = []
    for c, t in times.items():
        med = float(np.median(t))
        res.append({"layout": "tiled", "tile": c[0][0], "seg_pad": c[0][1], "tile_pad": c[0][2], "bpc": c[1],
                    "variant": c[2], "unroll": c[3], "ms_median": round(med, 4), "ms_min": round(min(t), 4),
                    "GBps_median": round(alg / med / 1e6, 1), "frac_peak": round(alg / med / 1e6 / 8000, 4)})
    res.sort(key=lambda x: x["ms_median"])
    for x in res:
        print(json.dumps(x))


if __name__ == "__main__":
    main()
