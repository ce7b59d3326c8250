#!/usr/bin/env python3
"""Writes tests/golden/sqrt_amd_box.npz: 100,000 fp32 inputs in [1, 4) (uint32 bit patterns, seeded sample) and the
torch.sqrt results of the GPU box's AMD EPYC 9575F host for them (uint32), from that host's run of
tools/sqrt_box_kernels.py (session r03_s12): its sse2_misses_1_4.npz lists, for every fp32 in [1, 4), the inputs
where torch.sqrt differed from oracle_sqrt_mkl_sse2 and torch's bits there; everywhere else torch equalled it.

  python tests/golden/make_sqrt_amd_box.py gpurun_out/r03_s12/sqrt/sse2_misses_1_4.npz
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from oracle import fedavg_oracle as orc

    d = np.load(sys.argv[1], allow_pickle=False)
    bits = np.arange(0x3F800000, 0x40800000, dtype=np.uint32)
    box = orc.sqrt_torch_cpu_sse2(bits.view(np.float32)).view(np.uint32).copy()
    box[d["x"] - 0x3F800000] = d["torch"]
    sel = np.sort(np.random.default_rng(355).choice(bits.size, 100_000, replace=False))
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "sqrt_amd_box.npz"), x=bits[sel], torch_sqrt=box[sel])


if __name__ == "__main__":
    main()
