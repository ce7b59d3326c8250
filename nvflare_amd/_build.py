"""Build libnvflare_amd_fedavg.so in-tree with hipcc for gfx950 (no torch, no cmake).

The library lands in nvflare_amd/lib/ so that it travels with the repository snapshot to the GPU box
(git-ignored, not gpurun-ignored)."""

from __future__ import annotations

import os
import re
import subprocess
import time
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB_NAME = "libnvflare_amd_fedavg.so"
LIB_PATH = os.path.join(LIB_DIR, LIB_NAME)
# the fp32 tile kernels are instantiated per arithmetic mode in their own translation units so that the
# objects compile in parallel (one hipcc per source), then link into one shared library; the fused kernels
# (every optimizer kind x launch form) go further: fedavg_epi_inst.hip is compiled once per (mode,
# finalisation), nine objects, the heaviest first in the queue
EPI_SOURCE = "fedavg_epi_inst.hip"
# A/B builds (-DFEDAVG_AB, tools/build_rev_lib.py): every (mode, finalisation) pair.  Product builds: the pairs the
# drop-in's callers produce plus the server step alone (csrc/fedavg_internal.h epi_direct; "step" = -DFEDAVG_EPI_STEP)
EPI_UNITS_AB = [(f"{mode}_{fin}", op, fin_v) for mode, op in (("torch", 1), ("numpy", 0), ("unweighted", 2))
                for fin, fin_v in (("div", 2), ("scale", 1), ("none", 0))]
EPI_UNITS = [u for u in EPI_UNITS_AB if u[0] in ("torch_div", "torch_scale", "numpy_scale", "unweighted_scale",
                                                  "unweighted_div")] + [("step", None, None)]
NARROW_SOURCE = "fedavg_narrow.hip"
SOURCES = [EPI_SOURCE, "fedavg_tiles_numpy.hip", "fedavg_tiles_torch.hip", "fedavg_tiles_unweighted.hip",
           "fedavg_kernels.hip", "fedavg_narrow.hip", "fedavg_dequant.hip", "fedavg_capi.cpp"]
HEADERS = ["fedavg_internal.h", "fedavg_rsqrt14.h", "fedavg_arith.h", "fedavg_tiles.h",
           "fedavg_epi.h"]
OBJ_DIR = os.path.join(PKG, "lib", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

# -ffp-contract=off: the numpy-mode multiply and add must round separately (bit parity with the
# reference); the torch mode uses explicit fma builtins.  No fast-math: IEEE division, denormals kept.
# -pragma-unroll-threshold: the burst epilogue's `#pragma unroll` over its register-held tiles must unroll fully
# (tile m's results live in dd[m]); at LLVM's default threshold the largest epilogue (RMSprop with torch CPU's
# restated sqrt) stayed rolled and dd went to 528 bytes of scratch per lane.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"--offload-arch={ARCH}",
         "-mllvm", "-pragma-unroll-threshold=200000", "-Wall", "-Wno-unused-command-line-argument"]


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(ROOT, "include", "nvflare_amd_fedavg.h"))
    files.append(os.path.abspath(__file__))  # flags and the source list live here
    return files


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def _mentions(csrc: str, src: str, macro: str) -> bool:
    try:
        with open(os.path.join(csrc, src)) as f:
            return macro in f.read()
    except OSError:
        return False


def compile_units(sources=SOURCES, ab=False, csrc=None):
    """(source, object name, extra flags) of every translation unit: the fused kernels' source once per EPI_UNITS
    entry (EPI_UNITS_AB for an A/B build) in two halves by optimizer kind, the 16-bit source once per format, the others
    once each.  ``csrc``: the directory of sources from another revision (tools/build_rev_lib.py): a source that does
    not know a split macro (FEDAVG_EPI_PART, FEDAVG_NARROW_PART -- round 5) is compiled as one unit, and the stand-alone
    server-step unit (FEDAVG_EPI_STEP) is left out where the sources lack it, so no symbol is defined twice."""
    split_epi = csrc is None or _mentions(csrc, EPI_SOURCE, "FEDAVG_EPI_PART")
    split_narrow = csrc is None or _mentions(csrc, NARROW_SOURCE, "FEDAVG_NARROW_PART")
    has_step = csrc is None or _mentions(csrc, EPI_SOURCE, "FEDAVG_EPI_STEP")
    units = []
    for src in sources:
        if src == EPI_SOURCE:  # each (mode, finalisation) pair in two halves (fedavg_epi_inst.hip FEDAVG_EPI_PART)
            for name, op, fin in (EPI_UNITS_AB if ab else EPI_UNITS):
                if op is None:
                    if has_step:
                        units.append((src, f"fedavg_epi_{name}.hip.o", ["-DFEDAVG_EPI_STEP"]))
                    continue
                defs = [f"-DFEDAVG_EPI_OP={op}", f"-DFEDAVG_EPI_FIN={fin}", f"-DFEDAVG_EPI_FN=launch_epi_{name}",
                        f"-DFEDAVG_EPI_FN2=launch_epi_{name}_part2"]
                if not split_epi:
                    units.append((src, f"fedavg_epi_{name}.hip.o", defs))
                    continue
                units += [(src, f"fedavg_epi_{name}.hip.o", defs + ["-DFEDAVG_EPI_PART=1"]),
                          (src, f"fedavg_epi_{name}_part2.hip.o", defs + ["-DFEDAVG_EPI_PART=2"])]
        elif src == NARROW_SOURCE and split_narrow:  # once per 16-bit format (fedavg_narrow.hip FEDAVG_NARROW_PART)
            units += [(src, "fedavg_narrow_bf16.hip.o", ["-DFEDAVG_NARROW_PART=1"]),
                      (src, "fedavg_narrow_f16.hip.o", ["-DFEDAVG_NARROW_PART=2"])]
        else:
            units.append((src, src + ".o", []))
    return units


# every symbol must resolve at link time: a translation unit missing from the link fails the build, not the first
# dlopen on the GPU box
LINK_FLAGS = ["-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,--no-undefined"]


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def unit_deps(src: str) -> list:
    """The source and every local header it includes, transitively (csrc/ and include/), plus this file (flags)."""
    seen, todo = [], [os.path.join(CSRC, src)]
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.append(f)
        with open(f) as fh:
            for name in _INCLUDE.findall(fh.read()):
                for d in (CSRC, os.path.join(ROOT, "include")):
                    cand = os.path.join(d, name)
                    if os.path.exists(cand):
                        todo.append(cand)
                        break
    return seen + [os.path.abspath(__file__)]


def build_library(force: bool = False, verbose: bool = False, jobs: int = 0) -> str:
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(OBJ_DIR, exist_ok=True)
    inc = [f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]

    # the longest units first (the 16-bit and fused units take minutes each, the rest seconds to a minute), so the
    # pool's critical path is one long unit, not a long unit started last
    units = sorted(compile_units(), key=lambda u: 0 if "_part2" in u[1] else 1 if u[0] == EPI_SOURCE else
                   2 if u[0] == NARROW_SOURCE else 3)

    def compile_one(unit) -> str:
        src, obj_name, extra = unit
        obj = os.path.join(OBJ_DIR, obj_name)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(
                os.path.getmtime(f) for f in unit_deps(src)):
            return obj  # up to date: a unit recompiles when its source or a header it includes changed
        cmd = [HIPCC, *FLAGS, *extra, *inc, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        t0 = time.time()
        subprocess.run(cmd, check=True)
        if verbose:
            print(f"{obj_name}: {time.time() - t0:.0f} s", flush=True)
        return obj

    jobs = jobs or min(len(units), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=jobs) as pool:
        objs = list(pool.map(compile_one, units))
    for f in os.listdir(OBJ_DIR):  # objects of units this build no longer has (an earlier unit list)
        if f.endswith(".o") and os.path.join(OBJ_DIR, f) not in objs:
            os.remove(os.path.join(OBJ_DIR, f))
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, *LINK_FLAGS, *objs, "-o", tmp, "-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
