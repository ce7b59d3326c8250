#!/usr/bin/env python3
"""Build the HIP library from the sources of another git revision into a side path, for same-box A/B runs
(``NVFLARE_AMD_FEDAVG_LIB=<out> python tools/bench_narrow.py ...`` against the in-tree library).

  python tools/build_rev_lib.py --rev HEAD --out nvflare_amd/lib/ab/libnvflare_amd_fedavg_head.so
  python tools/build_rev_lib.py --rev WORKTREE -D FEDAVG_NARROW_UNROLL=8 --out nvflare_amd/lib/ab/u8.so

The revision's csrc/ and include/ are exported to a temporary directory with ``git show``; the flags and
source list (with the fused kernels' per-unit definitions) are the current nvflare_amd/_build.py's (the A/B
compares kernels, not build settings).  The library is an A/B build (-DFEDAVG_AB): it carries every kernel form,
launch variant, tile width and unroll the sources know, which the product library (nvflare_amd/_build.py) leaves out."""

import argparse
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nvflare_amd import _build as B  # noqa: E402

AB_OBJ = os.path.join(B.PKG, "lib", "obj_ab")  # objects of the last full WORKTREE A/B build (no -D), for --only


def _export(rev: str, path: str, dst: str) -> None:
    files = subprocess.run(["git", "-C", ROOT, "ls-tree", "-r", "--name-only", rev, path], check=True,
                           capture_output=True, text=True).stdout.split()
    for f in files:
        blob = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], check=True, capture_output=True).stdout
        out = os.path.join(dst, f)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "wb") as fh:
            fh.write(blob)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--out", required=True)
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor definitions")
    ap.add_argument("--product", action="store_true",
                    help="a product-sized library (no -DFEDAVG_AB, the product unit list) plus the -D definitions, "
                         "e.g. -D FEDAVG_AB_FEW for the few-client forms' sweep only")
    ap.add_argument("--only", default="",
                    help="with --rev WORKTREE: comma list of sources or object names to compile (with -D); every "
                         "other unit's object is the last full WORKTREE A/B build's (nvflare_amd/lib/obj_ab), or with "
                         "--product the in-tree product build's (nvflare_amd/lib/obj), so a one-unit A/B links in "
                         "minutes")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        if args.rev == "WORKTREE":  # the working tree's sources as they are
            shutil.copytree(os.path.join(ROOT, "nvflare_amd", "csrc"), os.path.join(tmp, "nvflare_amd", "csrc"))
            shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        else:
            _export(args.rev, "nvflare_amd/csrc", tmp)
            _export(args.rev, "include", tmp)
        csrc = os.path.join(tmp, "nvflare_amd", "csrc")
        inc = [f"-I{os.path.join(tmp, 'include')}", f"-I{csrc}"]
        # an A/B library: every kernel form the sources know (-DFEDAVG_AB; ignored by revisions before round 5)
        # the unit list the revision's sources support (round-4 sources define every fused / 16-bit entry
        # once per source, so they must not be split into PART=1 / PART=2 objects)
        units = B.compile_units([s for s in B.SOURCES if os.path.exists(os.path.join(csrc, s))], ab=not args.product,
                                csrc=csrc)
        only = [x for x in args.only.split(",") if x]
        if only and args.rev != "WORKTREE":
            raise SystemExit("--only needs --rev WORKTREE (the reused objects are the working tree's)")
        # --only reuses: the last full WORKTREE A/B build's objects, or with --product the in-tree product build's,
        # or with --product -D ... the last full WORKTREE build's with the same definitions (lib/obj_<defines>)
        reuse = AB_OBJ if not args.product else (
            os.path.join(B.PKG, "lib", "obj_" + "_".join(sorted(args.defines))) if args.defines else B.OBJ_DIR)
        keep = args.rev == "WORKTREE" and not only and (args.product == bool(args.defines))
        if only and not os.path.isdir(reuse):
            raise SystemExit(f"--only reuses the objects of a full build ({reuse}): run one first")
        if only and args.product and not args.defines and B.needs_build():
            raise SystemExit("--only --product reuses the in-tree objects: build the in-tree library first")

        def compile_one(unit):
            src, obj_name, extra = unit
            if only and src not in only and obj_name not in only:  # a source, or one object (fedavg_epi_torch_div.hip.o)
                return os.path.join(reuse, obj_name)
            obj = os.path.join(tmp, obj_name)
            defs = [f"-D{d}" for d in ([] if args.product else ["FEDAVG_AB"]) + args.defines]
            subprocess.run([B.HIPCC, *B.FLAGS, *extra, *defs, *inc, "-c", os.path.join(csrc, src), "-o", obj], check=True)
            if keep:  # for a later --only
                os.makedirs(reuse, exist_ok=True)
                shutil.copy(obj, os.path.join(reuse, obj_name))
            return obj

        with ThreadPoolExecutor(max_workers=min(8, len(units))) as pool:
            objs = list(pool.map(compile_one, units))
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        subprocess.run([B.HIPCC, *B.LINK_FLAGS, *objs, "-o", args.out, "-lpthread"], check=True)
    print(args.out)


if __name__ == "__main__":
    main()
