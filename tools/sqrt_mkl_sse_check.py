#!/usr/bin/env python3
"""Check the oracle's restatements of MKL's SSE vsSqrt kernels exhaustively -- diagnostic, not part of the product.

  python tools/sqrt_mkl_sse2_check.py kernel [--stride S]   oracle_sqrt_mkl_sse2 against mkl_vml_kernel_sSqrt_E2HAynn
                                                            itself, called from the libtorch_cpu this torch ships
  python tools/sqrt_mkl_sse2_check.py ex --rsqrtps DUMP     oracle_sqrt_mkl_rsqrtps with THIS CPU's RSQRTPS table
                                                            (a tools/rsqrtps_dump.c dump made here) against
                                                            mkl_vml_kernel_sSqrt_EXHAynn run here
  python tools/sqrt_mkl_sse2_check.py torch [--stride S]    oracle_sqrt_mkl_rsqrtps with the AMD host's table
                                                            (nvflare_amd/data/rsqrtps_amd.bin) against this host's
                                                            torch.sqrt (run it on the AMD box)

Every fp32 bit pattern (or every S-th) in chunks of 2^24; NaN results compare as NaN.  Prints one JSON line per
input class and a summary.
"""

import argparse
import ctypes
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
CHUNK = 1 << 24


def mkl_kernel(name):
    import torch

    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
    fn = getattr(lib, name)
    fn.restype = None
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return fn


def classify(bits):
    cls = np.full(bits.shape, 3, np.int8)  # 3: negative / NaN / inf (callout)
    cls[bits < 0x00800000] = 0  # +0 and subnormals (callout)
    cls[(bits >= 0x00800000) & (bits <= 0x7F7FF000)] = 1  # the vector path
    cls[(bits > 0x7F7FF000) & (bits < 0x7F800000)] = 2  # top finite values (callout)
    return cls


def work(job):
    i, stride, against, dump = job
    import torch

    from oracle import fedavg_oracle as orc

    torch.set_num_threads(1)
    bits = ((np.uint64(i) * CHUNK + np.arange(0, CHUNK, stride, dtype=np.uint64)) & 0xFFFFFFFF).astype(np.uint32)
    x = bits.view(np.float32)
    if against in ("kernel", "ex"):
        got = np.empty_like(x)
        mkl_kernel("mkl_vml_kernel_sSqrt_E2HAynn" if against == "kernel" else "mkl_vml_kernel_sSqrt_EXHAynn")(
            x.size, x.ctypes.data, got.ctypes.data)
    else:
        got = torch.from_numpy(x.copy()).sqrt().numpy()
    if against == "kernel":
        want = orc.sqrt_torch_cpu_sse2(x)
    else:
        import make_rsqrtps_table

        want = orc.sqrt_torch_cpu_amd(x, make_rsqrtps_table.table_from_dump(dump) if dump else None)
    with np.errstate(invalid="ignore"):
        cr = np.sqrt(x)
    both_nan = np.isnan(got) & np.isnan(want)
    bad = (got.view(np.uint32) != want.view(np.uint32)) & ~both_nan
    off_cr = (got.view(np.uint32) != cr.view(np.uint32)) & ~(np.isnan(got) & np.isnan(cr))
    cls = classify(bits)
    out = []
    for c in range(4):
        sel = cls == c
        out.append((int(sel.sum()), int((bad & sel).sum()), int((off_cr & sel).sum())))
    ex = [(hex(int(b)), hex(int(g)), hex(int(w))) for b, g, w in
          zip(bits[bad][:3], got.view(np.uint32)[bad][:3], want.view(np.uint32)[bad][:3])]
    return i, out, ex


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("against", choices=["kernel", "ex", "torch"])
    ap.add_argument("--rsqrtps", default=None, help="tools/rsqrtps_dump.c dump of this CPU (for 'ex')")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--workers", type=int, default=8)
    args = ap.parse_args()
    names = ["zero_subnormal", "vector_path", "top_finite", "neg_inf_nan"]
    tot = np.zeros((4, 3), np.int64)
    examples = []
    with Pool(args.workers) as pool:
        for i, out, ex in pool.imap_unordered(work, [(i, args.stride, args.against, args.rsqrtps) for i in range(256)]):
            tot += np.array(out)
            examples += ex
    for c, name in enumerate(names):
        print(json.dumps({"class": name, "inputs": int(tot[c, 0]), "mismatches_vs_restatement": int(tot[c, 1]),
                          "differ_from_correctly_rounded": int(tot[c, 2])}))
    what = {"kernel": "oracle_sqrt_mkl_sse2 vs MKL's E2HA kernel",
            "ex": "oracle_sqrt_mkl_rsqrtps (this CPU's table) vs MKL's EXHA kernel",
            "torch": "oracle_sqrt_mkl_rsqrtps (AMD table) vs torch.sqrt"}[args.against]
    print(json.dumps({"summary": what,
                      "inputs": int(tot[:, 0].sum()), "mismatches": int(tot[:, 1].sum()), "stride": args.stride,
                      "examples": examples[:10]}), flush=True)
    return 1 if tot[:, 1].sum() else 0


if __name__ == "__main__":
    sys.exit(main())
