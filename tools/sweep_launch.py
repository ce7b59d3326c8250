#!/usr/bin/env python3
"""Interleaved in-process sweep of the streaming kernel's launch parameters on the bench workload
(tiled slab of K slots): tile width x blocks/CU x unroll x cache-policy variant.  Every configuration is
timed with HIP events in each of R rounds; rounds interleave all configurations (one process, one
device), per cdna_hip_programming.md section 5.4 rule 24.  Outputs are compared bit-for-bit on a sample
across configurations of the same tile width."""

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
    ap.add_argument("--tile", default="2048,4096")
    ap.add_argument("--bpc", default="1,2,4")
    ap.add_argument("--unroll", default="4,8")
    ap.add_argument("--variant", default="0,1,2,3")
    ap.add_argument("--mode", default="torch")
    args = ap.parse_args()
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(0)
    K, P = args.clients, int(args.params)
    P -= P % 4
    tiles = [int(x) for x in args.tile.split(",")]
    layouts = {t: TiledLayout(t, K) for t in tiles}
    slab = ctx.alloc(max(l.slab_elems(P) for l in layouts.values()) * 4)
    out = ctx.alloc(P * 4)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    op, fin = (1, 2) if args.mode == "torch" else (0, 1)
    idx = np.unique(np.random.default_rng(0).integers(0, P, 20000)).astype(np.uint64)
    configs = list(itertools.product(tiles, [int(x) for x in args.bpc.split(",")], [int(x) for x in args.unroll.split(",")],
                                     [int(x) for x in args.variant.split(",")]))
    times = {c: [] for c in configs}
    ref = {}
    alg = 4.0 * K * P + 4.0 * P
    filled = None
    for r in range(args.rounds):
        for c in configs:
            tile, bpc, unroll, var = c
            lay = layouts[tile]
            bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
            if filled != tile:
                for k, b in enumerate(bases):
                    ctx.fill_synthetic_f32(b, P, 1000, k, 0, lay.tile, lay.tile_stride)
                ctx.sync()
                filled = tile
            ctx.set_launch(bpc, unroll)
            ctx.set_variant(var)
            run = lambda: ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, P, out.ptr, op, fin, cnt)  # noqa: E731
            run()
            ctx.timing_begin()
            for _ in range(args.reps):
                run()
            times[c].append(ctx.timing_end() / args.reps)
            if r == 0:
                sample = ctx.gather_f32(out.ptr, idx)
                ref.setdefault(tile, sample)
                assert np.array_equal(sample.view(np.uint32), ref[tile].view(np.uint32)), f"bits differ for {c}"
        print(f"round {r} done", file=sys.stderr, flush=True)
    ctx.set_launch(0, 0)
    ctx.set_variant(0)
    res = []
    for c, t in times.items():
        med = float(np.median(t))
        res.append({"tile": c[0], "bpc": c[1], "unroll": c[2], "variant": c[3], "ms_median": round(med, 4),
                    "ms_min": round(min(t), 4), "GBps_median": round(alg / med / 1e6, 1),
                    "frac_peak": round(alg / med / 1e6 / 8000, 4)})
    res.sort(key=lambda x: x["ms_median"])
    for x in res:
        print(json.dumps(x))


if __name__ == "__main__":
    main()
