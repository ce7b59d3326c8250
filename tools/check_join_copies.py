"""Scan gfx950 assembly (hipcc --save-temps .s, or llvm-objdump -d of a code object) for the miscompile round 6 hit in
the LDS-DMA fused form (fedavg_arith.h wave_any): a VALU write placed in a divergent branch's join block BEFORE the
block's exec restore (s_or_b64 exec, exec, s[..]) whose destination register is written nowhere else in the kernel --
the lanes that skipped the branch then never receive the value.  A heuristic, not a proof: it flags the pattern in its
simplest (and observed) form.

usage: python tools/check_join_copies.py FILE.s|LIB.so [...]   (exit 1 when any kernel is flagged)
"""
import re
import subprocess
import sys
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"
_REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")


def _regs(operand):
    out = []
    for m in _REG.finditer(operand):
        if m.group(1):
            out.append(f"{m.group(1)}{m.group(2)}")
        else:
            out += [f"{m.group(3)}{i}" for i in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out


_LOADS = ("global_load", "ds_read", "buffer_load", "scratch_load", "flat_load", "global_atomic", "ds_bpermute",
          "ds_permute", "ds_swizzle")


def _dest(line, loads=False):
    """Destination VGPR/AGPR names of a VALU instruction (first operand), or [] (loads too with loads=True)."""
    t = line.strip().split(None, 1)
    if len(t) < 2:
        return []
    if loads and t[0].startswith(_LOADS) and "_lds" not in t[0]:
        return _regs(t[1].split(",")[0])
    if not t[0].startswith("v_") or t[0].startswith(("v_cmp", "v_writelane", "v_readlane", "v_readfirstlane")):
        return []
    return _regs(t[1].split(",")[0])


def kernels_from_asm(text):
    for m in re.finditer(r"^(_Z\S+|[A-Za-z_]\w*):[^\n]*\n(.*?)\n\ts_endpgm", text, re.S | re.M):
        yield m.group(1), m.group(2).split("\n")


def code_objects(path):
    """The gfx950 code objects in a host .so's .hip_fatbin section: one clang offload bundle per linked object file,
    concatenated (magic, bundle count, then (offset, size, triple length, triple) per entry, offsets from the magic)."""
    import os
    import struct
    import tempfile

    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    pos = data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(magic))[0]
        q = pos + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple and size:
                yield data[pos + off:pos + off + size]
        pos = data.find(magic, pos + len(magic))


def _kernels_of_code_object(co):
    """(name, lines) per kernel of one code object, with a label line inserted at every branch target (objdump prints
    none): "L<addr>:"."""
    import os
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "co.o")
        open(f, "wb").write(co)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f], capture_output=True, text=True).stdout
    out = []
    for name, start, insts in _functions(dis):
        targets = set()
        for _, text, cmt in insts:
            m = re.search(r"<.*\+0x([0-9a-f]+)>", cmt)
            if text.startswith(("s_cbranch", "s_branch")) and m:
                targets.add(start + int(m.group(1), 16))
        lines = []
        for addr, text, _ in insts:
            if addr in targets:
                lines.append(f"L{addr:x}:")
            lines.append(text)
        out.append((name, lines))
    return out


def _check_code_object(co):
    ks = _kernels_of_code_object(co)
    return len(ks), [(name, f) for name, lines in ks for f in [check(name, lines)] if f]


def scan_so(path, jobs=8):
    """(kernels scanned, [(kernel, flagged lines)]) over every gfx950 code object of a host .so, `jobs` at a time."""
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(jobs) as ex:
        res = list(ex.map(_check_code_object, code_objects(path)))
    return sum(n for n, _ in res), [x for _, fl in res for x in fl]


def _functions(dis):
    cur = None
    for line in dis.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            if cur:
                yield cur
            cur = (m.group(2), int(m.group(1), 16), [])
            continue
        if cur is None or "//" not in line:
            continue
        text, cmt = line.split("//", 1)
        a = re.match(r"\s*([0-9A-Fa-f]+):", cmt)
        if text.strip() and a:
            cur[2].append((int(a.group(1), 16), text.strip(), cmt))
    if cur:
        yield cur


def check(name, lines):
    writes = Counter()
    for ln in lines:
        for r in _dest(ln, loads=True):
            writes[r] += 1
    flagged = []
    block = []
    for ln in lines:
        s = ln.strip()
        if re.match(r"^\.?[\w.$]+:", s) or s.startswith("s_cbranch") or s.startswith("s_branch"):
            block = []
            continue
        if re.match(r"s_or_b64\s+exec,\s*exec,", s):
            for b in block:
                d = _dest(b)
                if d and all(writes[r] == 1 for r in d):
                    flagged.append(b.strip())
            block = []
            continue
        block.append(ln)
    return flagged


def main(paths):
    bad = 0
    for p in paths:
        if p.endswith(".s"):
            ks = list(kernels_from_asm(open(p).read()))
            n, flagged = len(ks), [(name, f) for name, lines in ks for f in [check(name, lines)] if f]
        else:
            n, flagged = scan_so(p)
        for name, f in flagged:
            bad += 1
            print(f"{p}: {name[:120]}: {len(f)} join-block write(s) before the exec restore, e.g. {f[:4]}")
        print(f"{p}: {n} kernels scanned")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
