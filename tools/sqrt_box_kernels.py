#!/usr/bin/env python3
"""Which MKL vsSqrt kernel does this host's torch.sqrt run?  (diagnostic, CPU only; for the GPU box's AMD host)

Calls every single-precision vsSqrt kernel the libtorch_cpu of this torch exports (mkl_vml_kernel_sSqrt_{E2,EX,H8,
L9,Z0}{HA,LA,EP}) on tools/sqrt_probe.py's 59.8 M inputs ON THIS HOST, and counts where each differs from this host's
torch.sqrt; also the oracle's restatements (AVX-512: oracle_sqrt_torch_cpu, AMD: oracle_sqrt_mkl_rsqrtps with the
captured table, SSE2: oracle_sqrt_mkl_sse2) by input class.
Kernels built on approximate instructions (rcpps / rsqrtps) can give other bits on another CPU vendor, so this must
run where the question is asked.

  python tools/sqrt_box_kernels.py OUT_DIR     writes OUT_DIR/sqrt_box_kernels.json and, for [1, 4), the inputs
                                               where torch differs from the SSE2 restatement (sse2_misses_1_4.npz)
                                               and from the AMD one (amd_misses_1_4.npz)
"""

import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def differ(a, b):
    return ~((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b)))


def main():
    import torch

    import sqrt_probe
    from oracle import fedavg_oracle as orc

    out_dir = sys.argv[1]
    os.makedirs(out_dir, exist_ok=True)
    x = sqrt_probe.probe_set().view(np.float32)
    with np.errstate(invalid="ignore"):
        t = torch.from_numpy(x.copy()).sqrt().numpy()
        cr = np.sqrt(x)
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
    rec = {"host_cpu": sqrt_probe_cpu(), "torch": torch.__version__, "inputs": int(x.size),
           "torch_vs_correctly_rounded": int(differ(t, cr).sum()), "kernels": {}}
    for isa in ("E2", "EX", "H8", "L9", "Z0"):
        for acc in ("HA", "LA", "EP"):
            name = f"mkl_vml_kernel_sSqrt_{isa}{acc}{'nnn' if acc == 'EP' else 'ynn'}"
            try:
                fn = getattr(lib, name)
            except AttributeError:
                continue
            fn.restype = None
            fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
            try:
                got = np.empty_like(x)
                for i in range(0, x.size, 1 << 24):
                    n = min(1 << 24, x.size - i)
                    fn(n, x[i:].ctypes.data, got[i:].ctypes.data)
            except Exception as e:  # noqa: BLE001 -- an ISA this CPU lacks
                rec["kernels"][name] = f"{type(e).__name__}: {e}"
                continue
            rec["kernels"][name] = {"vs_torch": int(differ(got, t).sum()), "vs_correctly_rounded": int(differ(got, cr).sum())}
            print(name, rec["kernels"][name], flush=True)
    b = x.view(np.uint32)
    classes = {"subnormal": (b > 0) & (b < 0x00800000), "normal_lt_2m96": (b >= 0x00800000) & (x < 2.0 ** -96),
               "normal_ge_2m96": (x >= 2.0 ** -96) & (b < 0x7F800000), "one_to_four": (x >= 1) & (x < 4)}
    for label, fn in (("sse2_restated", orc.sqrt_torch_cpu_sse2), ("amd_restated", orc.sqrt_torch_cpu_amd),
                      ("avx512_restated", orc.sqrt_torch_cpu)):
        with np.errstate(invalid="ignore"):
            r = fn(x)
        d = differ(r, t)
        rec[label] = {"vs_torch": int(d.sum()), **{k: int((d & m).sum()) for k, m in classes.items()}}
        print(label, rec[label], flush=True)
        if label in ("sse2_restated", "amd_restated"):
            sel = d & classes["one_to_four"]
            np.savez_compressed(os.path.join(out_dir, f"{label[:-9]}_misses_1_4.npz"), x=b[sel],
                                torch=t.view(np.uint32)[sel], restated=r.view(np.uint32)[sel])
    with open(os.path.join(out_dir, "sqrt_box_kernels.json"), "w") as f:
        json.dump(rec, f, indent=1)


def sqrt_probe_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            lines = f.read().splitlines()
        model = next((ln.split(":", 1)[1].strip() for ln in lines if ln.startswith("model name")), "?")
        flags = next((ln.split(":", 1)[1].split() for ln in lines if ln.startswith("flags")), [])
        return {"model": model, "avx512f": "avx512f" in flags, "avx2": "avx2" in flags}
    except OSError:
        return {}


if __name__ == "__main__":
    main()
