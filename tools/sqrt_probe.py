#!/usr/bin/env python3
"""torch CPU's fp32 sqrt on this host against its restatement (tools/sqrt_probe.c): diagnostic.

Builds tools/sqrt_probe.c, dumps this CPU's VRSQRT14PS table, checks the table-driven restatement against the
instruction, and compares torch.sqrt (the reference's op: torch/optim/adam.py:545 ``exp_avg_sq.sqrt()``) with
  * correctly rounded sqrt (numpy),
  * the restatement from this CPU's table,
  * the restatement from the committed table (nvflare_amd/data/rsqrt14_avx512.bin, captured where the golden
    FedOpt fixtures were generated),
over every mantissa of [1, 4), every subnormal and a sample of every binade.  Prints one JSON line.

  python tools/sqrt_probe.py [--save-table OUT.bin]
"""

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
COMMITTED = os.path.join(ROOT, "nvflare_amd", "data", "rsqrt14_avx512.bin")


def probe_set() -> np.ndarray:
    """The x values of sqrt_probe.c probe_set(), in the same order (uint32 bit patterns)."""
    parts = [np.arange(127 << 23, 129 << 23, dtype=np.uint32), np.arange(1, 1 << 23, dtype=np.uint32)]
    for e in range(1, 255):
        if e in (127, 128):
            continue
        parts.append((np.uint32(e << 23) | np.arange(e % 61, 1 << 23, 61, dtype=np.uint32)).astype(np.uint32))
    parts.append(np.array([0x00000000, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0xBF800000, 0x7F7FFFFF,
                           0x00000001, 0x3F800000, 0x40800000, 0x3E800000, 0x00800000], dtype=np.uint32))
    return np.concatenate(parts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save-table", default=None)
    a = ap.parse_args()
    import torch

    tmp = tempfile.mkdtemp(prefix="sqrt_probe_")
    exe = os.path.join(tmp, "sqrt_probe")
    subprocess.run(["gcc", "-O2", "-mavx512f", "-mfma", "-o", exe, os.path.join(HERE, "sqrt_probe.c"), "-lm"], check=True)
    local_tab = os.path.join(tmp, "table.bin")
    subprocess.run([exe, "table", local_tab], check=True)
    if a.save_table:
        with open(local_tab, "rb") as f, open(a.save_table, "wb") as g:
            g.write(f.read())
    x = probe_set()
    xf = x.view(np.float32)
    with np.errstate(invalid="ignore"):
        t = torch.from_numpy(xf.copy()).sqrt().numpy()
        cr = np.sqrt(xf)
    res = {"host_cpu": _cpu_model(), "torch": torch.__version__, "probe_values": int(x.size),
           "torch_cpu_capability": torch.backends.cpu.get_cpu_capability()}

    def diff(a_, b_):
        same = (a_.view(np.uint32) == b_.view(np.uint32)) | (np.isnan(a_) & np.isnan(b_))
        return int(np.count_nonzero(~same))

    res["torch_vs_correctly_rounded"] = diff(t, cr)
    tables = {"local": local_tab}
    if os.path.exists(COMMITTED):
        tables["committed"] = COMMITTED
    for name, tab in tables.items():
        out = os.path.join(tmp, f"sqrt_{name}.bin")
        p = subprocess.run([exe, "check", tab, out], check=True, capture_output=True, text=True)
        chk = json.loads(p.stdout)
        r = np.fromfile(out, dtype=np.float32)
        assert r.size == x.size
        res[f"torch_vs_restated_{name}_table"] = diff(t, r)
        res[f"{name}_table_restatement_vs_this_cpu_instruction"] = chk
        if name == "local":
            res["breakdown"] = _breakdown(x, xf, t, cr, r)
    # which candidate sequence reproduces this host's torch (tools/sqrt_probe2.c: rsqrt14 / rsqrtps estimates,
    # Newton forms, small-input scaling)
    exe2 = os.path.join(tmp, "sqrt_probe2")
    subprocess.run(["gcc", "-O2", "-mavx512f", "-mavx2", "-mfma", "-o", exe2, os.path.join(HERE, "sqrt_probe2.c"), "-lm"],
                   check=True)
    xin, tin = os.path.join(tmp, "x.bin"), os.path.join(tmp, "torch.bin")
    x.tofile(xin)
    t.tofile(tin)
    p2 = subprocess.run([exe2, xin, tin], check=True, capture_output=True, text=True)
    res["candidates"] = json.loads(p2.stdout)
    with open(local_tab, "rb") as f:
        lt = f.read()
    res["local_table_sha256"] = hashlib.sha256(lt).hexdigest()
    if os.path.exists(COMMITTED):
        with open(COMMITTED, "rb") as f:
            ct = f.read()
        res["committed_table_sha256"] = hashlib.sha256(ct).hexdigest()
        res["local_table_equals_committed"] = lt == ct
    print(json.dumps(res), flush=True)


def _breakdown(x, xf, t, cr, r):
    """Where torch differs from the correctly rounded and the restated sqrt, by input class, with samples."""
    tb, cb, rb = t.view(np.uint32), cr.view(np.uint32), r.view(np.uint32)
    fin = np.isfinite(xf) & (xf > 0)
    classes = {"subnormal": fin & (x < 0x00800000), "normal_lt_2m96": fin & (x >= 0x00800000) & (xf < 2.0 ** -96),
               "normal_ge_2m96": fin & (xf >= 2.0 ** -96), "one_to_four": fin & (xf >= 1.0) & (xf < 4.0)}
    out = {}
    for name, sel in classes.items():
        n = int(np.count_nonzero(sel))
        d_cr = sel & (tb != cb)
        d_r = sel & (tb != rb)
        e = {"n": n, "vs_cr": int(np.count_nonzero(d_cr)), "vs_restated": int(np.count_nonzero(d_r)),
             "torch_zero": int(np.count_nonzero(sel & (tb == 0)))}
        # signed ulp distance torch - correctly rounded, histogram
        ulp = tb[sel].astype(np.int64) - cb[sel].astype(np.int64)
        vals, cnt = np.unique(np.clip(ulp, -4, 4), return_counts=True)
        e["ulp_vs_cr"] = {int(v): int(c) for v, c in zip(vals, cnt)}
        idx = np.flatnonzero(d_r)[:12]
        e["samples"] = [[f"{int(x[i]):08x}", f"{int(tb[i]):08x}", f"{int(cb[i]):08x}", f"{int(rb[i]):08x}"] for i in idx]
        out[name] = e
    return out


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    sys.exit(main())
