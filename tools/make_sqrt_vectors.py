#!/usr/bin/env python3
"""Writes nvflare_amd/data/sqrt_vectors.npz: the probe nvflare_amd/torch_sqrt.py uses to tell which fp32 sqrt
this host's torch CPU computes.  Inputs: 6144 fp32 values where torch CPU's AVX-512 vsSqrt (restated by the oracle,
oracle_sqrt_torch_cpu, pinned against torch in tests/test_torch_sqrt.py) and the correctly rounded sqrt DIFFER
(spread over 48 binades, subnormals included), plus 2048 where they agree, then 3072 where the AMD hosts' vsSqrt
(oracle_sqrt_mkl_rsqrtps with the captured RSQRTPS table, tests/test_torch_sqrt_amd.py) differs from both; outputs:
the three results.

  python tools/make_sqrt_vectors.py          (test infrastructure: run where the oracle is built)
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from oracle import fedavg_oracle as orc

    rng = np.random.default_rng(20261017)
    picked_diff, picked_same = [], []
    exps = list(range(-40, 8)) + [-126, -127]  # 127 + e in the biased field; -127 = subnormals
    for e in exps:
        if e == -127:
            bits = rng.integers(1, 1 << 23, 200_000, dtype=np.uint32)
        else:
            bits = (np.uint32((e + 127) << 23) | rng.integers(0, 1 << 23, 200_000, dtype=np.uint32)).astype(np.uint32)
        x = bits.view(np.float32)
        a = orc.sqrt_torch_cpu(x)
        b = np.sqrt(x)
        d = a.view(np.uint32) != b.view(np.uint32)
        picked_diff.append(x[d][:128])
        picked_same.append(x[~d][:40])
    x = np.concatenate(picked_diff + picked_same + [np.array([0.0, 1.0, 4.0, 0.25, 2.0, 3.4e38, 1e-45], np.float32)])
    rng2 = np.random.default_rng(20261018)
    picked_amd = []
    for e in range(-40, 8):
        bits = (np.uint32((e + 127) << 23) | rng2.integers(0, 1 << 23, 20_000, dtype=np.uint32)).astype(np.uint32)
        y = bits.view(np.float32)
        c = orc.sqrt_torch_cpu_amd(y).view(np.uint32)
        d = (c != np.sqrt(y).view(np.uint32)) & (c != orc.sqrt_torch_cpu(y).view(np.uint32))
        picked_amd.append(y[d][:64])
    x = np.concatenate([x] + picked_amd)
    out = os.path.join(ROOT, "nvflare_amd", "data", "sqrt_vectors.npz")
    np.savez(out, x=x, torch_cpu=orc.sqrt_torch_cpu(x), torch_cpu_amd=orc.sqrt_torch_cpu_amd(x), ieee=np.sqrt(x))
    print(out, x.size, int(np.count_nonzero(orc.sqrt_torch_cpu(x).view(np.uint32) != np.sqrt(x).view(np.uint32))))


if __name__ == "__main__":
    main()
