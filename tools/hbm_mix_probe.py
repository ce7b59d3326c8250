#!/usr/bin/env python3
"""R:1 read/write mix probe (diagnostic; tools/hbm_pattern_probe.hip ``mix_run``): the chip's ceiling for the
traffic shape of a K-client aggregation (K reads per result write; config 2 = 8 clients: 8:1), next to the
real burst kernel on the same footprint, interleaved rounds in one process, medians.  Prints JSON lines.

  python tools/hbm_mix_probe.py [--ratio 8] [--params 1.25e8] [--rounds 5]
"""

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def lib_path():
    path = os.path.join(HERE, "build", "libhbm_pattern_probe.so")
    src = os.path.join(HERE, "hbm_pattern_probe.hip")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", path],
                       check=True)
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ratio", type=int, default=8)
    ap.add_argument("--params", type=float, default=1.25e8, help="results (fp32) per pass: footprint (R+1) x 4 x this")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--preset", choices=["default", "few", "epi"], default="default",
                    help="epi: the fused server step's shape at R = 1..3 clients (R + 3 reads, 3 in-place writes per "
                         "chunk; epi_run) next to the library's fused Adam kernel")
    a = ap.parse_args()
    lp = lib_path()
    if a.build_only:
        return
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(0)
    lib = ctypes.CDLL(lp)
    lib.mix_set_dyn.argtypes = [ctypes.c_int]
    lib.epi_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                            ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_int)]
    lib.mix_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                            ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_int)]
    R = a.ratio
    P = int(a.params)
    n_tiles = (P + 4095) // 4096
    nbytes = n_tiles * ((R + 6) if a.preset == "epi" else (R + 1)) * 16384
    buf = ctx.alloc(nbytes)
    ctx.fill_synthetic_f32(buf.ptr, nbytes // 4, 1, 0)
    # the real kernel on a slab of R clients x P params (torch mode, library defaults)
    lay = TiledLayout(4096, R)
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(R)]
    for k, b in enumerate(bases):
        ctx.fill_synthetic_f32(b, P, 1000, k, 0, lay.tile, lay.tile_stride)
    end = (P + 3) // 4 * 4
    out = ctx.alloc(end * 4)
    ops = []
    if a.preset == "epi":  # p, m, v of the library's fused Adam step
        ops = [ctx.alloc(end * 4) for _ in range(3)]
        for j, b in enumerate(ops):
            ctx.fill_synthetic_f32(b.ptr, end, 77, j, 0)
    ws = [float(1 + (37 * k) % 100) for k in range(R)]
    cnt = sum(ws)
    ctx.sync()
    ncu = ctx.num_cus
    cases = [("grid", 0, 0, 0, 4), ("grid", 0, 0, 0, 8), ("read", 1, 0, 0, 1), ("read", 1, 0, 0, 2),
             ("tile", 2, 0, 0, 1), ("tile", 2, 0, 0, 2),
             ("burst_r8_l4", 3, 8, 4, 2), ("burst_r8_l5", 3, 8, 5, 2), ("burst_r8_l0", 3, 8, 0, 2),
             ("burst_r4_l4", 3, 4, 4, 2), ("burst_r8_l10", 3, 8, 10, 1), ("burst_r0_l8", 3, 0, 8, 1),
             ("write", 4, 0, 0, 1), ("write", 4, 0, 0, 2), ("write_grid", 5, 0, 0, 2),
             ("write_aux0", 7, 0, 0, 1), ("write_aux2", 7, 2, 0, 1), ("write_aux16", 7, 16, 0, 1),
             ("write_aux17", 7, 17, 0, 1), ("write_aux0", 7, 0, 0, 2),
             ("dyn_r8_l9_avg12", 6, 8, 9, 1, 12), ("dyn_r8_l9_avg15", 6, 8, 9, 1, 15),
             ("dyn_r8_l4_avg11", 6, 8, 4, 2, 11), ("dyn_r8_l4_avg12", 6, 8, 4, 2, 12),
             ("kernel", -1, 0, 0, 0)]
    if a.preset == "few":  # few-client shapes (R = 1..4): the additive bound's halves, the per-chunk store forms at
        # several occupancies, and the multi forms (G chunks' loads in flight per lane, stores immediate / deferred)
        cases = [("read", 1, 0, 0, 1), ("read", 1, 0, 0, 2), ("read", 1, 0, 0, 4),
                 ("write", 4, 0, 0, 1), ("write", 4, 0, 0, 2), ("write", 4, 0, 0, 4),
                 ("grid", 0, 0, 0, 2), ("grid", 0, 0, 0, 4), ("grid", 0, 0, 0, 8),
                 ("tile", 2, 0, 0, 1), ("tile", 2, 0, 0, 2), ("tile", 2, 0, 0, 4),
                 ("burst_r8_l4", 3, 8, 4, 2)]
        for g in (1, 2, 4):
            for bpc in (1, 2, 4):
                cases.append((f"multi_g{g}", 8, g, 0, bpc))
                cases.append((f"multi_defer_g{g}", 9, g, 0, bpc))
        cases.append(("kernel", -1, 0, 0, 0))
    if a.preset == "epi":  # (name, -10 - epi mode, reg, lds, bpc)
        cases = [("read", 1, 0, 0, 1), ("read", 1, 0, 0, 2), ("write", 4, 0, 0, 1),
                 ("e_tile2", -10, 0, 0, 1), ("e_tile2", -10, 0, 0, 2), ("e_tile2", -10, 0, 0, 4),
                 ("e_tile1", -11, 0, 0, 1), ("e_tile1", -11, 0, 0, 2), ("e_tile1", -11, 0, 0, 4),
                 ("e_burst_r4", -12, 4, 0, 1), ("e_burst_r4_l3", -12, 4, 3, 1), ("e_burst_r2_l1", -12, 2, 1, 2),
                 ("e_burst_r3", -12, 3, 0, 2), ("e_burst_d_r8_l4", -13, 8, 4, 2), ("e_burst_d_r8_l9", -13, 8, 9, 1),
                 ("kernel_adam", -2, 0, 0, 0)]
    if os.environ.get("MIX_CASES"):  # comma list of probe names to run
        keep = set(os.environ["MIX_CASES"].split(","))
        cases = [c for c in cases if c[0] in keep]
    res = {c: [] for c in cases}
    info = {}
    for _ in range(a.rounds):
        for c in cases:
            name, mode, reg, lds, bpc = c[:5]
            lib.mix_set_dyn(c[5] if len(c) > 5 else 12)
            if mode <= -10:
                ms = ctypes.c_float(0)
                moved = ctypes.c_double(0)
                nl = ctypes.c_int(0)
                rc = lib.epi_run(-10 - mode, R, reg, lds, ctypes.c_void_p(buf.ptr), nbytes, ncu * bpc, a.reps,
                                 ctypes.byref(ms), ctypes.byref(moved), ctypes.byref(nl))
                if rc != 0:
                    raise SystemExit(f"epi probe {c} rc={rc}")
                info[c] = (moved.value, nl.value)
                res[c].append(ms.value)
                continue
            if mode == -2:  # the library's fused Adam step over R clients (default routing)
                e = N.Epilogue()
                e.kind = N.FEDAVG_EPI_ADAM
                e.lr, e.beta1, e.beta2, e.eps, e.step = 1e-3, 0.9, 0.999, 1e-8, 1.0
                e.param, e.state1, e.state2 = (ops[j].ptr for j in range(3))
                ctx.timing_begin()
                n0 = ctx.launch_count()
                for _ in range(a.reps):
                    ctx.accumulate_tiled_epi(bases, ws, lay.tile, lay.tile_stride, 0, end, None, N.FEDAVG_OP_TORCH,
                                             N.FEDAVG_FIN_DIV, cnt, e)
                ctx.sync()
                ms = ctx.timing_end() / a.reps
                info[c] = (4.0 * R * P + 24.0 * P, (ctx.launch_count() - n0) / a.reps)
                res[c].append(ms)
                continue
            if mode < 0:
                ctx.timing_begin()
                n0 = ctx.launch_count()
                for _ in range(a.reps):
                    ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, end, out.ptr, N.FEDAVG_OP_TORCH,
                                         N.FEDAVG_FIN_DIV, cnt)
                ctx.sync()
                ms = ctx.timing_end() / a.reps
                info[c] = (4.0 * R * P + 4.0 * P, (ctx.launch_count() - n0) / a.reps)
                res[c].append(ms)
                continue
            ms = ctypes.c_float(0)
            moved = ctypes.c_double(0)
            nl = ctypes.c_int(0)
            rc = lib.mix_run(mode, R, reg, lds, ctypes.c_void_p(buf.ptr), nbytes, ncu * bpc, a.reps, ctypes.byref(ms),
                             ctypes.byref(moved), ctypes.byref(nl))
            if rc != 0:
                raise SystemExit(f"mix probe {c} rc={rc}")
            info[c] = (moved.value, nl.value)
            res[c].append(ms.value)
    for c, v in res.items():
        name, mode, reg, lds, bpc = c[:5]
        med = statistics.median(v)
        moved, nl = info[c]
        print(json.dumps({"probe": name, "ratio": R, "params": P, "blocks_per_cu": bpc, "reg_tiles": reg,
                          "lds_tiles": lds, "launches": nl, "ms_median": round(med, 4),
                          "ms_all": [round(x, 4) for x in v], "bytes": moved,
                          "GBps": round(moved / (med / 1e3) / 1e9, 1), "frac_spec": round(moved / (med / 1e3) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
