#!/usr/bin/env python3
"""Same-box, same-process A/B of the FedAvg kernel layouts against the HBM read ceiling.

Rounds interleave: the read probe (tools/hbm_probe.hip, nontemporal float4 grid-stride read), the
rows-layout kernel and the tiled-slab kernel in a few launch configurations.  Device-to-device spread is
as large as the layout effect, so only numbers from one process on one device are compared."""

import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=float, default=0.45e9)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    from nvflare_amd.device import DeviceContext, TiledLayout

    lib_path = os.path.join(HERE, "build", "libhbm_probe.so")
    if not os.path.exists(lib_path):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        os.path.join(HERE, "hbm_probe.hip"), "-o", lib_path], check=True)
    probe = ctypes.CDLL(lib_path)
    probe.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_float)]
    ctx = DeviceContext.get(0)
    K, P = args.clients, int(args.params)
    P -= P % 4096
    rows = [ctx.alloc(P * 4) for _ in range(K)]
    for k, b in enumerate(rows):
        ctx.fill_synthetic_f32(b.ptr, P, 1000, k, 0)
    lay = TiledLayout(4096, K)
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    for k in range(K):
        ctx.fill_synthetic_f32(slab.ptr + lay.slot_offset_elems(k) * 4, P, 1000, k, 0, lay.tile, lay.tile_stride)
    out = ctx.alloc(P * 4)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    cnt = sum(ws)
    alg = 4.0 * K * P + 4.0 * P
    row_ptrs = [b.ptr for b in rows]
    slab_bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]

    def run(bases, tstride, bpc, unroll, variant):
        ctx.set_launch(bpc, unroll)
        ctx.set_variant(variant)
        ctx.accumulate_tiled(bases, ws, 4096, tstride, 0, P, out.ptr, 1, 2, cnt)
        ctx.timing_begin()
        for _ in range(3):
            ctx.accumulate_tiled(bases, ws, 4096, tstride, 0, P, out.ptr, 1, 2, cnt)
        return ctx.timing_end() / 3

    def probe_run(mode, bpc):
        ms = ctypes.c_float(0)
        rc = probe.probe_run(mode, ctypes.c_void_p(slab.ptr), lay.slab_elems(P) * 4, 256 * bpc, 3, ctypes.byref(ms))
        assert rc == 0
        return ms.value

    cases = {
        "probe_read_nt_bpc1": (lambda: probe_run(0, 1), lay.slab_elems(P) * 4.0),
        "probe_read_bpc1": (lambda: probe_run(1, 1), lay.slab_elems(P) * 4.0),
        "rows_b2_u4_nt": (lambda: run(row_ptrs, 4096, 2, 4, 0), alg),
        "rows_b2_u4_temporal": (lambda: run(row_ptrs, 4096, 2, 4, 3), alg),
        "slab_b2_u4_nt": (lambda: run(slab_bases, lay.tile_stride, 2, 4, 0), alg),
        "slab_b2_u4_nt_loads_temporal_stores": (lambda: run(slab_bases, lay.tile_stride, 2, 4, 2), alg),
        "slab_b2_u8_nt": (lambda: run(slab_bases, lay.tile_stride, 2, 8, 0), alg),
        "slab_b1_u8_nt": (lambda: run(slab_bases, lay.tile_stride, 1, 8, 0), alg),
        "slab_b3_u4_nt": (lambda: run(slab_bases, lay.tile_stride, 3, 4, 0), alg),
    }
    t = {k: [] for k in cases}
    for r in range(args.rounds):
        for name, (fn, _) in cases.items():
            t[name].append(fn())
        print(f"round {r}", file=sys.stderr, flush=True)
    ctx.set_launch(0, 0)
    ctx.set_variant(0)
    for name, (_, nbytes) in cases.items():
        med = float(np.median(t[name]))
        print(json.dumps({"case": name, "ms_median": round(med, 4), "ms_min": round(min(t[name]), 4),
                          "GBps": round(nbytes / med / 1e6, 1), "frac_spec": round(nbytes / med / 1e6 / 8000, 4),
                          "K": K, "P": P}))


if __name__ == "__main__":
    main()
