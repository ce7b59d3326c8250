"""Same-process A/B of the fused-epilogue kernel variants vs the plain aggregation kernel (one box,
one slab, so cross-box HBM variance cancels).  Prints one JSON line per (epilogue, variant).

  python tools/sweep_epilogue.py --clients 64 --params 1e9 --reps 5
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(0)
    K, P = a.clients, int(a.params)
    lay = TiledLayout(4096, K)
    end = (P + 3) // 4 * 4
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
    for k in range(K):
        ctx.fill_synthetic_f32(bases[k], P, 1234, k, 0, lay.tile, lay.tile_stride)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    bufs = [ctx.alloc(end * 4) for _ in range(3)]
    for b in bufs:
        ctx.memset(b.ptr, 0, end * 4)
    out = ctx.alloc(end * 4)
    ctx.sync()

    def timed(fn):
        fn()
        ctx.timing_begin()
        for _ in range(a.reps):
            fn()
        return ctx.timing_end() / a.reps

    rows = []
    ms = timed(lambda: ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, end, out.ptr, 1, 2, cnt))
    rows.append(("none", 0, 2, ms, 4.0 * K * P + 4.0 * P))
    for epi_name, kind, extra in (("add_base", N.FEDAVG_EPI_ADD_BASE, 8.0), ("sgd", N.FEDAVG_EPI_SGD, 16.0),
                                  ("adam", N.FEDAVG_EPI_ADAM, 24.0)):
        for variant, bpc in ((0, 2), (4, 2), (0, 3), (0, 4), (4, 3)):
            ctx.set_variant(variant)
            ctx.set_launch(bpc, 0)
            e = N.Epilogue()
            e.kind = kind
            e.lr, e.momentum, e.beta1, e.beta2, e.eps, e.step = 1e-3, 0.9, 0.9, 0.999, 1e-8, 1.0
            if kind == N.FEDAVG_EPI_ADD_BASE:
                e.base = bufs[0].ptr
                o = out.ptr
            else:
                e.param, e.state1, e.state2 = bufs[0].ptr, bufs[1].ptr, bufs[2].ptr
                o = None
            ms = timed(lambda: ctx.accumulate_tiled_epi(bases, ws, lay.tile, lay.tile_stride, 0, end, o, 1, 2, cnt, e))
            rows.append((epi_name, variant, bpc, ms, 4.0 * K * P + extra * P))
    ctx.set_variant(0)
    ctx.set_launch(0, 0)
    for name, variant, bpc, ms, b in rows:
        print(json.dumps({"epilogue": name, "variant": variant, "blocks_per_cu": bpc, "ms": round(ms, 3), "GBps": round(b / ms / 1e6, 1),
                          "frac_8TBps": round(b / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
