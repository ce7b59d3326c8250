"""The kernel's VRSQRT14PS estimate (fedavg_rsqrt14.h, 2 x 32 fixed-point line segments) against the captured
instruction table it replaces (nvflare_amd/data/rsqrt14_avx512.bin, the oracle's and nvflare_amd.torch_sqrt's
table): every one of the 65536 estimates, and the generator reproducing the committed header."""

import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "nvflare_amd", "csrc", "fedavg_rsqrt14.h")


def _array(text, name):
    body = re.search(rf"{name}\[64\] = \{{(.*?)\}};", text, re.S).group(1)
    vals = [int(v) for v in re.findall(r"(\d+)u", body)]
    assert len(vals) == 64
    return np.array(vals, dtype=np.uint64)


def _estimate(base, slope, p, m):
    """fedavg_arith.h sqrt_torch_cpu's y16 in uint32 arithmetic, as the kernel computes it."""
    seg = (p << 5) | (m >> 18)
    prod = (slope[seg] * ((m >> 8) & 1023)) & 0xFFFFFFFF
    return (((base[seg] - prod) & 0xFFFFFFFF) >> 10).astype(np.uint32)


def test_segments_reproduce_every_estimate():
    from nvflare_amd import torch_sqrt

    with open(HEADER) as f:
        text = f.read()
    base, slope = _array(text, "kRsqrt14Base"), _array(text, "kRsqrt14Slope")
    tab = torch_sqrt.table()
    idx = np.arange(65536, dtype=np.uint64)
    p, m = idx >> 15, (idx & 0x7FFF) << 8
    got = _estimate(base, slope, p, m)
    assert np.array_equal(got, tab.astype(np.uint32))
    # the low 8 mantissa bits never matter (the estimate depends on the top 15 only)
    got_hi = _estimate(base, slope, p, m | 0xFF)
    assert np.array_equal(got_hi, got)
    assert np.all(base >= slope * 1023)  # no uint32 wrap in the kernel's subtraction


def test_generator_reproduces_header(tmp_path):
    out = tmp_path / "fedavg_rsqrt14.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_rsqrt14_segments.py"), "--out", str(out)],
                   check=True, capture_output=True)
    with open(HEADER) as f:
        assert out.read_text() == f.read()
