"""The plain kernels' FIN_DIV (torch's ``total.div_(count)``) runs Markstein's correction from the correctly rounded
reciprocal of the launch-constant count instead of a division per element (nvflare_amd/csrc/fedavg_tiles.h
div_const).  Bit-exactness rests on that correction giving the correctly rounded quotient for every pair of
significands (away from underflow / overflow, where the kernel keeps the IEEE division).  The GPU probe
(tools/div_const_probe.py --all, profiles/r04/) checks all 2^23 x 2^23 pairs on the device; this CPU test repeats the
argument on the host with C's fmaf for every dividend significand and 1,536 divisors: the integer weight sums 1..1024
and 512 seeded random significands."""

import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc is absent")
    exe = str(tmp_path_factory.mktemp("divc") / "div_const_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", os.path.join(HERE, "div_const_check.c"), "-o", exe,
                    "-lm"], check=True)
    return exe


def test_every_dividend_significand(checker):
    rng = np.random.default_rng(4)
    divisors = [str(i) for i in range(1, 1025)] + [repr(float(x)) for x in rng.uniform(1.0, 2.0, 512).astype(np.float32)]
    chunks = [divisors[i::8] for i in range(8)]

    def run(ch):
        p = subprocess.run([checker, *ch], capture_output=True, text=True, timeout=600)
        return p.returncode, p.stdout

    with ThreadPoolExecutor(8) as pool:
        outs = list(pool.map(run, chunks))
    bad = [ln for _, out in outs for ln in out.splitlines() if not ln.endswith(" 0")]
    assert all(rc == 0 for rc, _ in outs) and not bad, bad[:10]
    assert sum(len(out.splitlines()) for _, out in outs) == len(divisors)
