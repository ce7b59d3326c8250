#!/usr/bin/env python3
"""The device's restated torch-CPU sqrts against the oracle on ALL 2^32 fp32 bit patterns (diagnostic; GPU box).

For each mode (FEDAVG_SQRT_TORCH_AVX512 = sqrt_torch_cpu, FEDAVG_SQRT_TORCH_AMD = sqrt_mkl_rsqrtps) the test entry
fedavg_sqrt_f32 runs over chunks of 2^26 inputs and each chunk is compared bit for bit (NaN payloads aside) with
oracle_sqrt_torch_cpu / oracle_sqrt_mkl_rsqrtps, the oracle side spread over a process pool.  Prints one JSON line.

  python tools/sqrt_device_exhaustive.py [--log2-chunk 26] [--workers 12]
"""

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def oracle_chunk(args):
    lo, n, mode = args
    from oracle import fedavg_oracle as orc

    x = (np.uint64(lo) + np.arange(n, dtype=np.uint64)).astype(np.uint32).view(np.float32)
    return (orc.sqrt_torch_cpu(x) if mode == 1 else orc.sqrt_torch_cpu_amd(x)).view(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2-chunk", type=int, default=26)
    ap.add_argument("--workers", type=int, default=12)
    args = ap.parse_args()
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    n = 1 << args.log2_chunk
    buf, out = ctx.alloc(4 * n), ctx.alloc(4 * n)
    res = {}
    t0 = time.time()
    with ProcessPoolExecutor(args.workers) as pool:
        for mode, name in ((1, "torch_cpu (Intel hosts)"), (2, "torch_cpu_amd (AMD hosts)")):
            mism, examples = 0, []
            starts = list(range(0, 1 << 32, n))
            want_it = pool.map(oracle_chunk, [(lo, n, mode) for lo in starts])
            for lo, want in zip(starts, want_it):
                x = (np.uint64(lo) + np.arange(n, dtype=np.uint64)).astype(np.uint32)
                ctx.h2d_ptr(buf.ptr, x.ctypes.data, x.nbytes)
                ctx.sqrt_f32(buf.ptr, out.ptr, n, mode)
                got = np.empty(n, np.uint32)
                ctx.d2h(got, out.ptr)
                gf, wf = got.view(np.float32), want.view(np.float32)
                bad = (got != want) & ~(np.isnan(gf) & np.isnan(wf))
                k = int(bad.sum())
                if k:
                    mism += k
                    examples += [(hex(int(a)), hex(int(b)), hex(int(c))) for a, b, c in
                                 zip(x[bad][:3], got[bad][:3], want[bad][:3])]
                if lo // n % 16 == 15:
                    print(json.dumps({"mode": name, "done": (lo + n) / 2 ** 32, "mismatches": mism}), flush=True)
            res[name] = {"inputs": 1 << 32, "mismatches": mism, "examples": examples[:10]}
    buf.close()
    out.close()
    print(json.dumps({"summary": "device sqrt (fedavg_sqrt_f32) vs oracle over all 2^32 fp32 bit patterns",
                      "seconds": round(time.time() - t0, 1), **res}), flush=True)
    return 1 if any(r["mismatches"] for r in res.values()) else 0


if __name__ == "__main__":
    sys.exit(main())
