#!/usr/bin/env python3
"""Export a whole earlier revision (its bench.py, package and C-ABI -- an earlier ABI than today's Python binds) into
abtree/<name>/ and build its library there with that revision's own nvflare_amd/_build.py, for same-box comparisons
of a past round's complete tree (round 5's bisect of the fused few-client line ran round 3's 229fc6e this way:
``python abtree/r3/bench.py ...``, profiles/r05/scripts/s4.sh).  abtree/ is git-ignored; its objects are
gpurun-ignored, its library travels.

  python tools/export_rev_tree.py --rev 229fc6e --name r3
"""

import argparse
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rev", required=True)
    ap.add_argument("--name", required=True)
    a = ap.parse_args()
    dst = os.path.join(ROOT, "abtree", a.name)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    os.makedirs(dst)
    archive = subprocess.run(["git", "-C", ROOT, "archive", a.rev], check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", dst], input=archive, check=True)
    for junk in ("profiles",):  # results of that round: not needed to run it
        shutil.rmtree(os.path.join(dst, junk), ignore_errors=True)
    subprocess.run([sys.executable, "-c", "from nvflare_amd import _build; print(_build.build_library(force=True))"],
                   cwd=dst, check=True)


if __name__ == "__main__":
    main()
