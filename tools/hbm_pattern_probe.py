#!/usr/bin/env python3
"""HBM read-pattern probe (diagnostic, tools/hbm_pattern_probe.hip): grid-stride sweep vs per-block chunk
streams (the slab kernel's pattern) vs LDS-DMA chunk streams vs two interleaved chunk streams per block, at
several chunk sizes and blocks per CU, on one buffer, interleaved rounds, medians.  Prints JSON lines."""

import ctypes
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    lib_path = os.path.join(HERE, "build", "libhbm_pattern_probe.so")
    src = os.path.join(HERE, "hbm_pattern_probe.hip")
    if not os.path.exists(lib_path) or os.path.getmtime(lib_path) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", lib_path],
                       check=True)
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    lib = ctypes.CDLL(lib_path)
    lib.pattern_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 32.0
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    nbytes = int(gib * 2**30) // (8 << 20) * (8 << 20)
    buf = ctx.alloc(nbytes)
    ctx.fill_synthetic_f32(buf.ptr, nbytes // 4, 1, 0)
    ctx.sync()
    ncu = ctx.num_cus
    cases = []
    if os.environ.get("PROBE_SET") == "footprint":
        for bpc in (1, 2):
            cases.append(("grid", 0, 8, 0, bpc))
            cases.append(("chunk", 1, 16, 1 << 20, bpc))
            cases.append(("chunk_w", 4, 16, 1 << 20, bpc))
            cases.append(("chunk_wd", 5, 16, 1 << 20, bpc))
            cases.append(("chunk_w_sc1", 6, 16, 1 << 20, bpc))
            cases.append(("chunk_w_sc0sc1", 7, 16, 1 << 20, bpc))
            cases.append(("chunk_w_plain", 8, 16, 1 << 20, bpc))
            if bpc == 1:
                cases.append(("chunk_w_lds_burst", 9, 16, 1 << 20, bpc))
                cases.append(("chunk_w_lds_burst_sliced", 10, 16, 1 << 20, bpc))
    for bpc in (1, 2) if not cases else ():
        for u in (8, 16):
            cases.append(("grid", 0, u, 0, bpc))
    for ch in (64 << 10, 256 << 10, 1 << 20, 4 << 20) if os.environ.get("PROBE_SET") != "footprint" else ():
        for bpc in (1, 2, 4):
            cases.append(("chunk", 1, 16, ch, bpc))
    for ch in (256 << 10, 1 << 20) if os.environ.get("PROBE_SET") != "footprint" else ():
        for bpc in (1, 2):
            cases.append(("chunk_lds", 2, 8, ch, bpc))
            cases.append(("chunk_pair", 3, 16, ch, bpc))
    res = {c: [] for c in cases}
    for _ in range(rounds):
        for c in cases:
            name, mode, u, ch, bpc = c
            ms = ctypes.c_float(0)
            rc = lib.pattern_run(mode, u, ctypes.c_void_p(buf.ptr), nbytes, ch or (1 << 20), ncu * bpc, 4, ctypes.byref(ms))
            if rc != 0:
                raise SystemExit(f"probe {c} rc={rc}")
            res[c].append(ms.value)
    for c, v in res.items():
        name, mode, u, ch, bpc = c
        med = statistics.median(v)
        moved = nbytes * 63 // 64 * 65 // 64 if mode >= 4 else nbytes  # chunk_w: reads + 1/64 writes
        print(json.dumps({"probe": name, "unroll": u, "chunk_KiB": ch >> 10, "blocks_per_cu": bpc, "GiB": gib,
                          "ms_median": round(med, 3), "GBps": round(moved / (med / 1e3) / 1e9, 1),
                          "frac_spec": round(moved / (med / 1e3) / 8e12, 4), "bytes": moved}), flush=True)


if __name__ == "__main__":
    main()
