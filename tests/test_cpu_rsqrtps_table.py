"""The RSQRTPS table behind FEDAVG_SQRT_TORCH_AMD is THIS host's, captured at run time: the
product's capture (fedavg_host_rsqrtps_table, C-ABI v9; host code, no device) equals the oracle's independent one
(oracle_host_rsqrtps_table) and tools/rsqrtps_dump.c's every-input dump of this CPU; the GPU pool's AMD table
captured in round 3 is a test fixture (tests/golden/rsqrtps_amd_epyc9575f.bin, from profiles/r03/s12/rsqrtps_amd.bin),
equal to the run-time capture on that CPU (checked here when the tests run there, and on the box by
tests/test_gpu_torch_sqrt.py)."""

import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

from nvflare_amd import torch_sqrt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "profiles", "r03", "s12", "rsqrtps_amd.bin")
BOX_CPU = "AMD EPYC 9575F"


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def test_runtime_capture_equals_the_oracle_and_the_dump(oracle, tmp_path):
    tab = torch_sqrt.host_rsqrtps_table()
    assert tab.dtype == np.uint16 and tab.size == 8192 and tab.max() <= 0xFFF
    assert np.array_equal(tab, oracle.rsqrtps_table())
    # a reciprocal square root estimate falls with x across each binade pair: [1, 2) then [2, 4)
    assert np.all(np.diff(tab[:4096].astype(int)) <= 0) and np.all(np.diff(tab[4096:].astype(int)) <= 0)
    if shutil.which("gcc") is None:
        pytest.skip("gcc is absent")
    exe = str(tmp_path / "rsqrtps_dump")
    subprocess.run(["gcc", "-O2", "-msse2", os.path.join(ROOT, "tools", "rsqrtps_dump.c"), "-o", exe], check=True)
    subprocess.run([exe, str(tmp_path / "rsq.bin"), str(tmp_path / "rcp.bin")], check=True, capture_output=True)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_rsqrtps_table

    assert np.array_equal(tab, make_rsqrtps_table.table_from_dump(str(tmp_path / "rsq.bin")))


def test_box_fixture_is_the_round3_dump(oracle):
    box = oracle.rsqrtps_table_box()
    if os.path.exists(DUMP):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import make_rsqrtps_table

        assert np.array_equal(box, make_rsqrtps_table.table_from_dump(DUMP))
    if BOX_CPU in cpu_model():
        assert np.array_equal(torch_sqrt.host_rsqrtps_table(), box)
    else:  # another vendor's estimate: the reason the table is captured at run time
        assert not np.array_equal(torch_sqrt.host_rsqrtps_table(), box) or "AMD" in cpu_model()


def test_restated_sse_sqrt_in_numpy_equals_the_oracle(oracle):
    """torch_sqrt.sqrt_sse_restated (the detection's numpy form) against oracle_sqrt_mkl_rsqrtps, with this host's and
    the box's tables, over every mantissa of [1, 4) sampled, the binade edges, subnormals and specials."""
    rng = np.random.default_rng(5)
    bits = np.concatenate([rng.integers(0, 1 << 32, 400_000, dtype=np.uint64).astype(np.uint32),
                           np.arange(0x3F800000, 0x40800000, 97, dtype=np.uint32),
                           np.array([0, 1, 0x007FFFFF, 0x00800000, 0x7F7FF000, 0x7F7FF001, 0x7F800000, 0xFF800000,
                                     0x7FC00000, 0x80000001, 0xBF800000], np.uint32)])
    x = bits.view(np.float32)
    for tab in (torch_sqrt.host_rsqrtps_table(), oracle.rsqrtps_table_box()):
        got = torch_sqrt.sqrt_sse_restated(x, tab)
        with np.errstate(invalid="ignore"):
            exp = oracle.sqrt_torch_cpu_amd(x, tab)
        same = (got.view(np.uint32) == exp.view(np.uint32)) | (np.isnan(got) & np.isnan(exp))
        assert same.all(), int((~same).sum())
