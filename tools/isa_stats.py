#!/usr/bin/env python3
"""Instruction statistics of one kernel in a host object's gfx950 code object (diagnostic for A/Bs): the counts of
the memory, wait, branch and division instructions, and where the waits fall relative to the global loads.

  python tools/isa_stats.py nvflare_amd/lib/obj/fedavg_epi_torch_div.hip.o fedavg_tiles_epi_f32x4ILi1ELi2ELb0ELi515ELb1E
  python tools/isa_stats.py OBJ PATTERN --dump out.s      # also write the kernel's disassembly
"""

import argparse
import collections
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
KEYS = ["global_load_dwordx4", "global_store_dwordx4", "global_load_dword", "ds_read_u16", "ds_read_b128",
        "ds_write_b128", "s_waitcnt", "s_cbranch_execz", "s_cbranch_execnz", "s_cbranch_scc0", "s_cbranch_scc1",
        "s_cbranch_vccnz", "s_cbranch_vccz", "s_branch", "v_div_scale_f32", "v_div_fixup_f32", "v_rcp_f32",
        "v_sqrt_f32", "v_fma_f32", "v_cndmask_b32_e64", "v_cndmask_b32_e32", "s_and_saveexec_b64",
        "scratch_store_dword", "scratch_store_dwordx4", "scratch_load_dword", "scratch_load_dwordx4"]


def disasm(obj: str, tmp: str) -> str:
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "co.elf")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", obj,
                    os.path.join(tmp, "s.o")], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--targets={TARGET}", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True, capture_output=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                          text=True).stdout


def kernel_body(text: str, pattern: str) -> tuple:
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^[0-9a-f]+ <([^>]+)>:$", text, re.M)]
    for i, (pos, name) in enumerate(heads):
        if pattern in name and not name.endswith(".kd"):
            end = heads[i + 1][0] if i + 1 < len(heads) else len(text)
            return name, text[pos:end]
    raise SystemExit(f"no kernel matching {pattern}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("pattern")
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        name, body = kernel_body(disasm(a.obj, tmp), a.pattern)
    if a.dump:
        with open(a.dump, "w") as f:
            f.write(body)
    c = collections.Counter()
    n = 0
    top = {"v": -1, "a": -1}  # the highest VGPR / AGPR index the kernel names (register pressure; spills show above)
    for m in re.finditer(r"\b([va])(?:(\d+)\b|\[\d+:(\d+)\])", body):
        top[m.group(1)] = max(top[m.group(1)], int(m.group(2) or m.group(3)))
    for line in body.splitlines():
        m = re.match(r"\s+(\w+)", line.split("//")[0])
        if m:
            c[m.group(1)] += 1
            n += 1
    print(name)
    print("instructions", n)
    print("vgprs", top["v"] + 1, "agprs", top["a"] + 1)
    for k in KEYS:
        if c[k]:
            print(f"{k:24s} {c[k]}")


if __name__ == "__main__":
    main()
