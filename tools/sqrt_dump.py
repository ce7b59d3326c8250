#!/usr/bin/env python3
"""Dump this host's torch CPU fp32 sqrt over [1, 2) (every mantissa) and [2, 4) (every 4th) for offline analysis
of which sequence it runs (diagnostic; tools/sqrt_probe.py counts candidates, this keeps the raw results).

  python tools/sqrt_dump.py OUT_DIR      writes sqrt_1_2.f32 (2^23 values) and sqrt_2_4_s4.f32 (2^21 values)
"""

import os
import sys

import numpy as np


def main():
    import torch

    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    a = (np.uint32(127 << 23) | np.arange(1 << 23, dtype=np.uint32)).view(np.float32)
    b = (np.uint32(128 << 23) | np.arange(0, 1 << 23, 4, dtype=np.uint32)).view(np.float32)
    torch.from_numpy(a.copy()).sqrt().numpy().tofile(os.path.join(out, "sqrt_1_2.f32"))
    torch.from_numpy(b.copy()).sqrt().numpy().tofile(os.path.join(out, "sqrt_2_4_s4.f32"))
    print("ok", flush=True)


if __name__ == "__main__":
    main()
