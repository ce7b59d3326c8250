"""Interleaved same-process A/B of launch variant bits (fedavg_set_variant) on the plain aggregation kernel
and the fused-epilogue kernel: one slab, rounds of (epilogue x variant) so drift and box-to-box HBM variance
cancel.  Prints one JSON line per measurement and a median summary line per (epilogue, variant).

  python tools/ab_variants.py --clients 64 --params 1e9 --variants 0,4 --epilogues none,adam --rounds 3
"""

import argparse
import json

import numpy as np
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EXTRA = {"none": 4.0, "add_base": 8.0, "sgd": 16.0, "adam": 24.0, "adagrad": 16.0, "adamax": 24.0, "nadam": 24.0,
         "radam": 24.0, "rprop": 24.0, "asgd": 16.0, "rmsprop": 24.0, "adam_ams": 32.0, "rmsprop_c": 32.0}
FOUR = ("adam_ams", "rmsprop_c")  # amsgrad's max_exp_avg_sq / centered RMSprop's grad_avg in state3
TWO_STATES = ("adam", "adamax", "nadam", "radam", "rprop", "rmsprop")  # rmsprop: square_avg, momentum buffer  # algorithmic bytes per param beyond 4K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,4", help="variant bits, or variant:unroll:blocks_per_cu triples")
    ap.add_argument("--epilogues", default="none,adam")
    ap.add_argument("--pads", default="0", help="tile-stride pads in elements (multiples of 64): one slab each, "
                                                "interleaved -- DRAM channel mapping of power-of-two strides")
    ap.add_argument("--op-shifts", default="0",
                    help="byte offsets (multiples of 256) of the fused epilogues' operand buffers (p, m, v / base): one "
                         "set of configs each, interleaved -- where the write streams fall in HBM relative to the reads")
    ap.add_argument("--mode", choices=["torch", "numpy"], default="torch",
                    help="torch: fma steps, IEEE division at the end; numpy: mul + add, multiply by 1/count")
    ap.add_argument("--check", action="store_true",
                    help="every config's output (the fused epilogues: p and the last state, from zeroed state) must "
                         "equal the first config's bit for bit")
    ap.add_argument("--frozen-frac", type=float, default=0.0,
                    help="this leading fraction of the parameters gets exactly-zero updates from every client (frozen "
                         "layers): Adam's exp_avg_sq stays 0 there, the restated sqrt's and quotients' rare inputs")
    ap.add_argument("--prewarm-s", type=float, default=0.0,
                    help="seconds of the first config run back to back before the first round (the GPU's power state "
                         "ramps over the first seconds of load: VERDICT r05 item 3)")
    ap.add_argument("--sqrt", choices=["ieee", "torch_cpu", "torch_cpu_amd"], default="ieee",
                    help="the fused epilogues' sqrt (EpiParams.torch_sqrt)")
    a = ap.parse_args()
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(0)
    from tools.gpu_state import GpuMonitor

    mon = GpuMonitor(0)  # clocks, power, temperatures per measurement
    print(json.dumps({"gpu_state": mon.snapshot()}), flush=True)
    K, P = a.clients, int(a.params)
    lay = TiledLayout(4096, K)
    end = (P + 3) // 4 * 4
    pads = [int(x) for x in a.pads.split(",")]
    slabs = {}
    for pad in pads:
        assert pad % 64 == 0
        stride = lay.tile_stride + pad
        n_tiles = (P + lay.tile - 1) // lay.tile
        slab = ctx.alloc(n_tiles * stride * 4)
        bases = [slab.ptr + k * lay.tile * 4 for k in range(K)]
        for k in range(K):
            ctx.fill_synthetic_f32(bases[k], P, 1234, k, 0, lay.tile, stride)
        frozen = int(a.frozen_frac * P) // 4 * 4
        if frozen:
            zeros = np.zeros(min(frozen, 1 << 24), dtype=np.float32)
            for k in range(K):
                for off in range(0, frozen, zeros.size):
                    n = min(zeros.size, frozen - off)
                    ctx.h2d_tiled(bases[k], lay.tile * 4, stride * 4, off * 4, zeros.ctypes.data, n * 4)
        slabs[pad] = (slab, bases, stride)
    op, fin = (1, 2) if a.mode == "torch" else (0, 1)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    shifts = [int(x) for x in a.op_shifts.split(",")]
    assert all(x % 256 == 0 and x >= 0 for x in shifts)
    bufs = [ctx.alloc(end * 4 + max(shifts)) for _ in range(4)]
    for b in bufs:
        ctx.memset(b.ptr, 0, end * 4 + max(shifts))
    out = ctx.alloc(end * 4)
    ctx.sync()
    kinds = {"add_base": N.FEDAVG_EPI_ADD_BASE, "sgd": N.FEDAVG_EPI_SGD, "adam": N.FEDAVG_EPI_ADAM,
             "adagrad": N.FEDAVG_EPI_ADAGRAD, "adamax": N.FEDAVG_EPI_ADAMAX, "nadam": N.FEDAVG_EPI_NADAM,
             "radam": N.FEDAVG_EPI_RADAM, "rprop": N.FEDAVG_EPI_RPROP, "asgd": N.FEDAVG_EPI_ASGD,
             "rmsprop": N.FEDAVG_EPI_RMSPROP, "adam_ams": N.FEDAVG_EPI_ADAM, "rmsprop_c": N.FEDAVG_EPI_RMSPROP}

    def launcher(epi, pad, sh=0):
        _, bases, stride = slabs[pad]
        if epi == "none":
            return lambda: ctx.accumulate_tiled(bases, ws, lay.tile, stride, 0, end, out.ptr, op, fin, cnt)
        e = N.Epilogue()
        e.kind = kinds[epi]
        e.lr, e.momentum, e.beta1, e.beta2, e.eps, e.step = 1e-3, 0.9, 0.9, 0.999, 1e-8, 1.0
        e.etaminus, e.etaplus, e.step_size_min, e.step_size_max = 0.5, 1.2, 1e-6, 50.0
        e.lambd, e.eta, e.mu = 1e-4, 1e-2, 0.5
        e.alpha = 0.99  # RMSprop (with momentum 0.9: not centered, three operand streams)
        e.torch_sqrt = {"ieee": N.FEDAVG_SQRT_IEEE, "torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512,
                        "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD}[a.sqrt]
        if epi == "add_base":
            e.base, o = bufs[0].ptr + sh, out.ptr
        else:
            e.param, e.state1 = bufs[0].ptr + sh, bufs[1].ptr + sh
            if epi in TWO_STATES or epi in FOUR or epi == "sgd":
                e.state2 = bufs[2].ptr + sh
            if epi in FOUR:
                e.state3 = bufs[3].ptr + sh
                e.amsgrad, e.centered = int(epi == "adam_ams"), int(epi == "rmsprop_c")
            o = None
        return lambda: ctx.accumulate_tiled_epi(bases, ws, lay.tile, stride, 0, end, o, op, fin, cnt, e)

    variants = [tuple(int(x) for x in (v.split(":") + ["0", "0"])[:3]) for v in a.variants.split(",")]
    epis = a.epilogues.split(",")
    res = {}
    ref_out = {}
    if a.prewarm_s > 0:
        import time

        v = variants[0]
        ctx.set_variant(v[0])
        ctx.set_launch(v[2], v[1])
        fn = launcher(epis[0], pads[0])
        t_end = time.perf_counter() + a.prewarm_s
        n = 0
        while time.perf_counter() < t_end:
            for _ in range(10):
                fn()
            ctx.sync()
            n += 10
        print(json.dumps({"prewarm_s": a.prewarm_s, "calls": n, "gpu_state": mon.snapshot()}), flush=True)
    for rnd in range(a.rounds):
        for epi, pad, sh in [(e_, p_, s_) for e_ in epis for p_ in pads for s_ in shifts]:
            fn = launcher(epi, pad, sh)
            for b in bufs:  # every epilogue from zeroed states: not another kind's (an RMSprop square_avg holding Adam's
                ctx.memset(b.ptr, 0, end * 4 + max(shifts))  # exp_avg goes negative and takes the sqrt's rare path)
            for v in variants:
                ctx.set_variant(v[0])
                ctx.set_launch(v[2], v[1])
                if a.check and epi != "none" and rnd == 0 and pad == pads[0] and sh == shifts[0]:
                    for b in bufs:  # the same state in for every config
                        ctx.memset(b.ptr, 0, end * 4)
                fn()
                if a.check and rnd == 0 and pad == pads[0] and sh == shifts[0]:
                    host = np.empty(end, dtype=np.float32)
                    ctx.sync()
                    ctx.d2h(host, out.ptr if epi in ("none", "add_base") else bufs[0].ptr + shifts[0])
                    if epi not in ("none", "add_base"):
                        last = np.empty(end, dtype=np.float32)
                        ctx.d2h(last, bufs[3 if epi in FOUR else 2 if epi in TWO_STATES else 1].ptr + shifts[0])
                        host = np.concatenate([host, last])
                    if epi not in ref_out:
                        ref_out[epi] = host
                    else:
                        bad = int(np.count_nonzero(host.view(np.uint32) != ref_out[epi].view(np.uint32)))
                        print(json.dumps({"check": ":".join(map(str, v)), "epilogue": epi, "mismatches": bad}), flush=True)
                        if bad:
                            raise SystemExit(f"config {v}: {bad} outputs differ from config {variants[0]}")
                    ctx.memset(out.ptr, 0xFF, end * 4)
                with mon.sample(0.02) as smp:
                    ctx.timing_begin()
                    for _ in range(a.reps):
                        fn()
                    ms = ctx.timing_end() / a.reps
                st = smp.summary()
                state = {k: (st[k]["median"] if isinstance(st.get(k), dict) else st.get(k))
                         for k in ("current_gfxclk", "current_uclk", "current_socket_power", "temperature_hotspot",
                                   "temperature_mem", "throttle_status", "samples") if k in st}
                gbs = (4.0 * K * P + EXTRA[epi] * P) / ms / 1e6
                res.setdefault((epi, pad, sh, v), []).append(ms)
                print(json.dumps({"round": rnd, "epilogue": epi, "pad": pad, "op_shift": sh, "mode": a.mode,
                                  "variant": ":".join(map(str, v)), "clients": K, "params": P,
                                  "ms": round(ms, 4), "GBps": round(gbs, 1), "frac_8TBps": round(gbs / 8000, 4),
                                  "gpu": state}),
                      flush=True)
    ctx.set_variant(0)
    ctx.set_launch(0, 0)
    for (epi, pad, sh, v), xs in res.items():
        ms = statistics.median(xs)
        gbs = (4.0 * K * P + EXTRA[epi] * P) / ms / 1e6
        print(json.dumps({"summary": True, "epilogue": epi, "pad": pad, "op_shift": sh, "mode": a.mode,
                          "variant": ":".join(map(str, v)), "clients": K, "params": P,
                          "median_ms": round(ms, 4), "GBps": round(gbs, 1), "frac_8TBps": round(gbs / 8000, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
