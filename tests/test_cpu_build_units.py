"""tools/build_rev_lib.py's unit list for OTHER revisions' sources: round-4 sources (22c4d2a)
define every fused entry once per (mode, finalisation) source and the 16-bit entries once, so splitting them into
FEDAVG_EPI_PART=1/2 and FEDAVG_NARROW_PART=1/2 objects defined each symbol twice and the shared link failed; the
product's stand-alone server-step unit does not exist there either.  The list must follow what the sources know."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nvflare_amd import _build as B  # noqa: E402

OLD_REV = "22c4d2a"  # round 4's final tree


def _export(rev, dst):
    files = subprocess.run(["git", "-C", ROOT, "ls-tree", "-r", "--name-only", rev, "nvflare_amd/csrc"], check=True,
                           capture_output=True, text=True).stdout.split()
    for f in files:
        blob = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], check=True, capture_output=True).stdout
        out = os.path.join(dst, f)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "wb") as fh:
            fh.write(blob)
    return os.path.join(dst, "nvflare_amd", "csrc")


def _check_unique(units):
    names = [u[1] for u in units]
    assert len(names) == len(set(names)), names
    # one object per (source, flags): no two units compile the same definitions
    keys = [(u[0], tuple(sorted(f for f in u[2] if not f.startswith("-DFEDAVG_EPI_FN2")))) for u in units]
    assert len(keys) == len(set(keys)), keys


def test_units_of_this_tree_are_split():
    units = B.compile_units(B.SOURCES, ab=False, csrc=B.CSRC)
    _check_unique(units)
    assert units == B.compile_units(B.SOURCES, ab=False)
    assert any("-DFEDAVG_EPI_PART=2" in u[2] for u in units) and any("-DFEDAVG_NARROW_PART=2" in u[2] for u in units)


@pytest.mark.parametrize("ab", [True, False])
def test_units_of_round4_sources_are_one_per_source(tmp_path, ab):
    try:
        csrc = _export(OLD_REV, str(tmp_path))
    except (subprocess.CalledProcessError, FileNotFoundError):
        pytest.skip(f"revision {OLD_REV} not in this checkout")
    srcs = [s for s in B.SOURCES if os.path.exists(os.path.join(csrc, s))]
    units = B.compile_units(srcs, ab=ab, csrc=csrc)
    _check_unique(units)
    flags = [f for u in units for f in u[2]]
    assert not any("PART" in f for f in flags), flags
    assert not any(f == "-DFEDAVG_EPI_STEP" for f in flags)
    epi = [u for u in units if u[0] == B.EPI_SOURCE]
    assert len(epi) == len([u for u in (B.EPI_UNITS_AB if ab else B.EPI_UNITS) if u[1] is not None])
