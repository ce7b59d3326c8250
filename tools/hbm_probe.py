#!/usr/bin/env python3
"""HBM ceiling probe (diagnostic): read-only and copy bandwidth on the device, for reading the FedAvg
kernel's roofline fraction against what this chip actually sustains (cdna_hip_programming.md rule 10)."""

import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    lib_path = os.path.join(HERE, "build", "libhbm_probe.so")
    if not os.path.exists(lib_path):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        os.path.join(HERE, "hbm_probe.hip"), "-o", lib_path], check=True)
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    lib = ctypes.CDLL(lib_path)
    lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                              ctypes.POINTER(ctypes.c_float)]
    nbytes = int(float(sys.argv[1]) if len(sys.argv) > 1 else 64e9)
    buf = ctx.alloc(nbytes)
    ctx.fill_synthetic_f32(buf.ptr, nbytes // 4, 1, 0)
    ctx.sync()
    names = {0: "read_nt", 1: "read", 2: "copy_kernel", 3: "hipMemcpy_d2d"}
    for mode in (0, 1, 2, 3):
        for bpc in ((1, 2, 4, 8) if mode < 3 else (1,)):
            ms = ctypes.c_float(0)
            rc = lib.probe_run(mode, ctypes.c_void_p(buf.ptr), nbytes, 256 * bpc, 5, ctypes.byref(ms))
            moved = nbytes if mode < 2 else nbytes  # copy: half read + half written = nbytes moved
            print(json.dumps({"probe": names[mode], "blocks_per_cu": bpc, "rc": rc, "ms": round(ms.value, 3),
                              "GBps": round(moved / (ms.value / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
