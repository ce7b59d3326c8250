#!/usr/bin/env python3
"""Throughput of the 16-bit (float16 / bfloat16) aggregation kernel: K device-resident client rows of P
values -> P values, torch-mode arithmetic (fedavg_narrow.hip).  Algorithmic bytes per launch 2*K*P + 2*P.

  python tools/bench_narrow.py [--clients 64 --params 1e9 --fmt bfloat16 --steps 10]
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
    ap.add_argument("--fmt", choices=["bfloat16", "float16"], default="bfloat16")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", choices=["torch", "numpy", "copy"], default="torch",
                    help="copy: unweighted, no finalisation -- the 1-client launch moves bytes only")
    ap.add_argument("--blocks-per-cu", default="0", help="comma list: interleaved same-process sweep (0 = default)")
    ap.add_argument("--variants", default="0", help="comma list of fedavg_set_variant values (0 = burst kernel, "
                                                      "8 = per-tile stores), swept with every blocks-per-cu value")
    ap.add_argument("--layout", choices=["rows", "tiled"], default="tiled",
                    help="rows: K separate client buffers (fedavg_accumulate); tiled: the engine's slab "
                         "(fedavg_accumulate_tiled16)")
    ap.add_argument("--check", action="store_true", help="every configuration's output bit-equal to the first's")
    args = ap.parse_args()
    import torch

    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext

    K, P = args.clients, int(args.params)
    ctx = DeviceContext.get(0)
    tdt = torch.bfloat16 if args.fmt == "bfloat16" else torch.float16
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    from nvflare_amd.device import TiledLayout

    lay = TiledLayout(4096, K)
    if args.layout == "tiled":
        slab = torch.randn(lay.slab_elems(P), dtype=tdt, device="cuda:0", generator=g)
        rows = [slab]
        bases = [slab.data_ptr() + lay.slot_offset_elems(k) * 2 for k in range(K)]
    else:
        rows = [torch.randn(P, dtype=tdt, device="cuda:0", generator=g) for _ in range(K)]
        bases = [r.data_ptr() for r in rows]
    out = torch.empty((P + 7) // 8 * 8, dtype=tdt, device="cuda:0")
    torch.cuda.synchronize()
    code = N.FEDAVG_BF16 if args.fmt == "bfloat16" else N.FEDAVG_F16
    op = {"torch": N.FEDAVG_OP_TORCH, "numpy": N.FEDAVG_OP_NUMPY, "copy": N.FEDAVG_OP_UNWEIGHTED}[args.mode]
    fin = {"torch": N.FEDAVG_FIN_DIV, "numpy": N.FEDAVG_FIN_SCALE, "copy": N.FEDAVG_FIN_NONE}[args.mode]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    end = (P + 7) // 8 * 8

    def launch():
        if args.layout == "tiled":
            ctx.accumulate_tiled16(code, bases, ws, 4096, lay.tile_stride, 0, end, out.data_ptr(), op, fin, sum(ws))
        else:
            ctx.accumulate(bases, ws, P, out.data_ptr(), code, code, op, fin, sum(ws))
    alg = 2.0 * K * P + 2.0 * P
    cfgs = [(int(v), int(b)) for v in args.variants.split(",") for b in args.blocks_per_cu.split(",")]
    res = {c: [] for c in cfgs}
    first = None
    for rep in range(3):
        for c in cfgs:
            ctx.set_variant(c[0])
            ctx.set_launch(c[1], 0)
            if args.check and rep == 0:
                out.fill_(float("nan"))
                torch.cuda.synchronize()  # torch's stream is not the library's: the fill must land before the launch
            launch()
            ctx.sync()
            if args.check and rep == 0:
                if first is None:
                    first = out.clone()
                elif not torch.equal(out.view(torch.int16), first.view(torch.int16)):
                    raise SystemExit(f"variant {c[0]} blocks/CU {c[1]}: output differs from variant {cfgs[0][0]}'s")
            ctx.timing_begin()
            for _ in range(args.steps):
                launch()
            res[c].append(ctx.timing_end() / args.steps)
    ctx.set_variant(0)
    ctx.set_launch(0, 0)
    for c in cfgs:
        ms = sorted(res[c])[len(res[c]) // 2]
        print(json.dumps({"tool": "bench_narrow", "fmt": args.fmt, "mode": args.mode, "clients": K, "params": P,
                          "variant": c[0], "blocks_per_cu": c[1], "layout": args.layout, "kernel_ms": round(ms, 3),
                          "alg_GBs": round(alg / ms / 1e6, 1),
                          "frac_of_8TBs": round(alg / ms / 1e6 / 8000.0, 4),
                          "GiBs_aggregated": round(2.0 * K * P / (ms / 1e3) / 2 ** 30, 1)}), flush=True)


if __name__ == "__main__":
    main()
