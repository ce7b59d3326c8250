"""The kernel's AMD-host RSQRTPS table (fedavg_rsqrtps_amd.h, staged in LDS by sqrt_mkl_rsqrtps) against the table
the oracle reads (nvflare_amd/data/rsqrtps_amd.bin) and the box dump both came from (profiles/r03/s12/
rsqrtps_amd.bin, tools/rsqrtps_dump.c): the same 8192 estimates, packed two per word as the kernel reads them."""

import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "nvflare_amd", "csrc", "fedavg_rsqrtps_amd.h")
DUMP = os.path.join(ROOT, "profiles", "r03", "s12", "rsqrtps_amd.bin")


def _header_table():
    with open(HEADER) as f:
        body = re.search(r"kRsqrtpsAmd\[4096\] = \{(.*?)\};", f.read(), re.S).group(1)
    words = np.array([int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", body)], dtype=np.uint32)
    assert words.size == 4096
    tab = np.empty(8192, np.uint16)
    tab[0::2], tab[1::2] = words & 0xFFFF, words >> 16  # low half first, as the kernel's 16-bit LDS read sees it
    return tab


def test_header_equals_the_oracle_table(oracle):
    tab = _header_table()
    assert np.array_equal(tab, oracle.rsqrtps_table())
    assert tab.max() <= 0xFFF
    # a reciprocal square root estimate falls with x across each binade pair: [1, 2) then [2, 4)
    assert np.all(np.diff(tab[:4096].astype(int)) <= 0) and np.all(np.diff(tab[4096:].astype(int)) <= 0)


def test_generator_reproduces_table_and_header(tmp_path):
    if not os.path.exists(DUMP):
        pytest.skip("the box dump is not in this tree")
    out, hdr = tmp_path / "t.bin", tmp_path / "fedavg_rsqrtps_amd.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_rsqrtps_table.py"), DUMP, str(out), "--header",
                    str(hdr)], check=True, capture_output=True, cwd=ROOT)
    assert np.array_equal(np.fromfile(out, dtype=np.uint16), _header_table())
    with open(hdr) as a, open(HEADER) as b:
        assert a.read().split("\n", 1)[1] == b.read().split("\n", 1)[1]  # all but the source path in line 1
