#!/usr/bin/env python3
"""Exhaustive check of the constant-divisor quotient (tools/div_const_probe.hip) over every fp32 dividend, for a list
of divisors: integer counts 1..N (weights are NUM_STEPS integers in most jobs), powers of two and their neighbours,
all-ones significands, and seeded random divisors in [2^-60, 2^60].  Prints one JSON line per divisor with a mismatch
and a summary line.

  python tools/div_const_probe.py [--ints 4096] [--random 2000]
"""

import argparse
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ints", type=int, default=4096)
    ap.add_argument("--random", type=int, default=20000)
    ap.add_argument("--all", action="store_true", help="every divisor significand of [1, 2) (2^23 x 2^23 pairs)")
    a = ap.parse_args()
    lib_path = os.path.join(HERE, "build", "libdiv_const_probe.so")
    src = os.path.join(HERE, "div_const_probe.hip")
    if not os.path.exists(lib_path) or os.path.getmtime(lib_path) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", lib_path],
                       check=True)
    lib = ctypes.CDLL(lib_path)
    rng = np.random.default_rng(1)
    ints = np.arange(1, a.ints + 1, dtype=np.float32)  # integer weight sums (NUM_STEPS counts)
    fracs = (rng.integers(1, 100000, 2000) / 10.0).astype(np.float32)  # sums of fractional weights
    rnd = rng.uniform(1.0, 2.0, a.random).astype(np.float32)
    edges = np.array([1.0, 1.0 + 2.0 ** -23, 2.0 - 2.0 ** -23, 1.5, 1.5 - 2.0 ** -23, 1.5 + 2.0 ** -23], np.float32)
    raw = np.concatenate([ints, fracs, rnd, edges])
    m = raw.view(np.uint32) & np.uint32(0x7FFFFF)  # the significand in [1, 2): exponents do not matter (header)
    bs = np.ascontiguousarray(np.unique((m | np.uint32(0x3F800000)).view(np.float32)), dtype=np.float32)
    if a.all:
        bs = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(np.float32)
    bad = np.zeros(bs.size, np.uint64)
    first = np.zeros(bs.size, np.uint32)
    rc = lib.div_probe_run(ctypes.c_void_p(bs.ctypes.data), ctypes.c_int(bs.size), ctypes.c_void_p(bad.ctypes.data),
                           ctypes.c_void_p(first.ctypes.data))
    if rc:
        raise SystemExit(f"div_probe_run rc={rc}")
    shown = 0
    for b, n, f in zip(bs, bad, first):
        if n and shown < 50:
            shown += 1
            print(json.dumps({"divisor": float(b), "divisor_bits": hex(int(np.float32(b).view(np.uint32))),
                              "mismatches": int(n), "first_dividend_bits": hex(int(f))}), flush=True)
    print(json.dumps({"summary": True, "divisor_significands": int(bs.size),
                      "dividends_per_divisor": "every significand of [1, 2) (2^23)",
                      "divisors_with_mismatches": int(np.count_nonzero(bad)),
                      "mismatches": int(bad.sum())}), flush=True)


if __name__ == "__main__":
    main()
