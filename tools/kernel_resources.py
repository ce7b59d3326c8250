#!/usr/bin/env python3
"""Per-kernel resources of the built HIP library (diagnostic + CPU regression guard): for every in-tree object
under nvflare_amd/lib/obj/, extract the gfx950 code object from its .hip_fatbin section (llvm-objcopy,
clang-offload-bundler) and read the kernels' metadata notes (llvm-readelf --notes): name, VGPR / AGPR / SGPR
counts, scratch bytes per lane (.private_segment_fixed_size) and LDS bytes.

  python tools/kernel_resources.py [--scratch-only]      # one JSON line per kernel
"""

import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "nvflare_amd", "lib", "obj")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernels(obj_path: str):
    """[{name, vgpr, agpr, sgpr, scratch, lds}] of the gfx950 kernels in one host object."""
    with tempfile.TemporaryDirectory() as tmp:
        fat = os.path.join(tmp, "fat.bin")
        co = os.path.join(tmp, "co.elf")
        r = subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", obj_path,
                            os.path.join(tmp, "stripped.o")], capture_output=True, text=True)
        if r.returncode != 0 or not os.path.exists(fat):
            return []
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for block in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        block = ".agpr_count:" + block

        def field(key, default=None):
            m = re.search(rf"\.{key}:\s+(\S+)", block)
            return m.group(1) if m else default

        out.append({"name": field("name"), "vgpr": int(field("vgpr_count", 0)), "agpr": int(field("agpr_count", 0)),
                    "sgpr": int(field("sgpr_count", 0)), "scratch": int(field("private_segment_fixed_size", 0)),
                    "lds": int(field("group_segment_fixed_size", 0))})
    return out


def all_kernels():
    res = []
    for f in sorted(os.listdir(OBJ)) if os.path.isdir(OBJ) else []:
        if f.endswith(".hip.o"):
            for k in kernels(os.path.join(OBJ, f)):
                k["object"] = f
                res.append(k)
    return res


def main():
    scratch_only = "--scratch-only" in sys.argv
    for k in all_kernels():
        if not scratch_only or k["scratch"]:
            print(json.dumps(k))


if __name__ == "__main__":
    main()
