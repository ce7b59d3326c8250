#!/usr/bin/env python3
"""Throughput of the contiguous-rows entry point (fedavg_accumulate) for fp64 and fp32 values: K separate
device-resident client rows of P values -> P values, numpy-mode arithmetic.  fp64 (numpy's default dtype)
and the integer types run the generic kernel; fp32 rows run the streaming kernel.  Algorithmic bytes per
launch: (K + 1) * P * itemsize.

  python tools/bench_generic.py [--clients 8 --params 125e6 --dtype float64 --steps 10]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=float, default=125e6)
    ap.add_argument("--dtype", choices=["float64", "float32"], default="float64")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--variants", default="0", help="comma list of fedavg_set_variant values, interleaved rounds")
    ap.add_argument("--blocks-per-cu", default="0", help="comma list, swept with every variant (0 = library default)")
    ap.add_argument("--mode", choices=["numpy", "torch"], default="numpy",
                    help="numpy: v*w then add, T * (1.0/count); torch: fma, T / count")
    ap.add_argument("--check", action="store_true", help="every configuration's output bit-equal to the first's")
    ap.add_argument("--layout", choices=["rows", "tiled"], default="rows",
                    help="rows: K separate client buffers (fedavg_accumulate); tiled: the engine's fp64 slab "
                         "(fedavg_accumulate_tiled64, float64 only)")
    args = ap.parse_args()
    import torch

    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext

    K, P = args.clients, int(args.params)
    ctx = DeviceContext.get(0)
    tdt = torch.float64 if args.dtype == "float64" else torch.float32
    code = N.FEDAVG_F64 if args.dtype == "float64" else N.FEDAVG_F32
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    op = N.FEDAVG_OP_TORCH if args.mode == "torch" else N.FEDAVG_OP_NUMPY
    fin = N.FEDAVG_FIN_DIV if args.mode == "torch" else N.FEDAVG_FIN_SCALE
    if args.layout == "tiled":
        from nvflare_amd.device import TiledLayout

        assert args.dtype == "float64", "the tiled layout here is the fp64 arena's"
        lay = TiledLayout(4096, K)
        slab = torch.randn(lay.slab_elems(P), dtype=tdt, device="cuda:0", generator=g)
        rows = [slab]
        bases = [slab.data_ptr() + lay.slot_offset_elems(k) * 8 for k in range(K)]
        end = (P + 1) // 2 * 2
        out = torch.empty(end, dtype=tdt, device="cuda:0")

        def launch():
            ctx.accumulate_tiled64(bases, ws, 4096, lay.tile_stride, 0, end, out.data_ptr(), op, fin, sum(ws))
    else:
        rows = [torch.randn(P, dtype=tdt, device="cuda:0", generator=g) for _ in range(K)]
        out = torch.empty(P, dtype=tdt, device="cuda:0")

        def launch():
            ctx.accumulate([r.data_ptr() for r in rows], ws, P, out.data_ptr(), code, code, op, fin, sum(ws))
    torch.cuda.synchronize()

    variants = [(int(v), int(b)) for v in args.variants.split(",") for b in args.blocks_per_cu.split(",")]
    res = {v: [] for v in variants}
    first = None
    for rep in range(3):
        for v in variants:
            ctx.set_variant(v[0])
            ctx.set_launch(v[1], 0)
            if args.check and rep == 0:
                out.fill_(float("nan"))
                torch.cuda.synchronize()  # torch's stream is not the library's: the fill must land before the launch
            launch()
            ctx.sync()
            if args.check and rep == 0:
                if first is None:
                    first = out.clone()
                elif not torch.equal(out.view(torch.int64 if out.element_size() == 8 else torch.int32),
                                     first.view(torch.int64 if out.element_size() == 8 else torch.int32)):
                    raise SystemExit(f"variant {v[0]} blocks/CU {v[1]}: output differs from variant {variants[0][0]}'s")
            ctx.timing_begin()
            for _ in range(args.steps):
                launch()
            res[v].append(ctx.timing_end() / args.steps)
    ctx.set_variant(0)
    ctx.set_launch(0, 0)
    nbytes = (K + 1) * P * out.element_size()
    for v in variants:
        ms = sorted(res[v])[len(res[v]) // 2]
        print(json.dumps({"tool": "bench_generic", "dtype": args.dtype, "mode": args.mode, "layout": args.layout,
                          "clients": K, "params": P,
                          "variant": v[0], "blocks_per_cu": v[1], "kernel_ms": round(ms, 3), "alg_GBs": round(nbytes / ms / 1e6, 1),
                          "frac_of_8TBs": round(nbytes / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
