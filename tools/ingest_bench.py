#!/usr/bin/env python3
"""Accept-side cost of decoding client payloads (row f2): reference decoders vs zero-copy ingest.

For K clients x P fp32 params (one key), measures the time from serialized bytes (or a disk-offloaded
safetensors file) to "staged in HBM" through WeightedAggregationHelper.add:
  npy_ref     np.load(BytesIO(data)) (numpy_decomposers.py:105-107) then add
  npy_view    nvflare_amd.ingest.recompose_npy (view over the bytes) then add
  st_ref      safetensors.torch.load(data) (app_opt/pt/decomposers.py:127-132) then add
  st_view     recompose_safetensors then add
  lazy_ref    _LazyRef.materialize() (lazy_tensor_dict.py:73-77) then add     (files in the page cache)
  lazy_mmap   the helper maps the file and stages from the mmap (MappedTensor)

  python tools/ingest_bench.py [--clients 8 --params 125e6 --dir /tmp/ingest_bench]
"""

import argparse
import io
import json
import os
import shutil
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class LazyRefLike:
    def __init__(self, file_path, key):
        self.file_path = file_path
        self.key = key

    def materialize(self):
        from safetensors import safe_open

        with safe_open(self.file_path, framework="pt") as f:
            return f.get_tensor(self.key)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=float, default=125e6)
    ap.add_argument("--dir", default="/tmp/ingest_bench")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    from safetensors.torch import load, save, save_file

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper
    from nvflare_amd.ingest import recompose_npy, recompose_safetensors

    K, P = args.clients, int(args.params)
    rng = np.random.default_rng(0)
    base = rng.standard_normal(P, dtype=np.float32)
    npy, st, files = [], [], []
    os.makedirs(args.dir, exist_ok=True)
    for k in range(K):
        a = base * np.float32(1 + 0.01 * k)
        s = io.BytesIO()
        np.save(s, a, allow_pickle=False)
        npy.append(s.getvalue())
        st.append(save({"t": torch.from_numpy(a)}))
        path = os.path.join(args.dir, f"c{k}.safetensors")
        save_file({"w": torch.from_numpy(a)}, path)
        files.append(path)
    del base, a
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    h = WeightedAggregationHelper()
    modes = {
        "npy_ref": lambda k: {"w": np.load(io.BytesIO(npy[k]), allow_pickle=False)},
        "npy_view": lambda k: {"w": recompose_npy(npy[k])},
        "st_ref": lambda k: {"w": load(st[k])["t"]},
        "st_view": lambda k: {"w": recompose_safetensors(st[k])["t"]},
        "lazy_ref": lambda k: {"w": LazyRefLike(files[k], "w").materialize()},
        "lazy_mmap": lambda k: {"w": LazyRefLike(files[k], "w")},
    }
    res = {m: [] for m in modes}
    for r in range(args.rounds):
        for m, fn in modes.items():
            t0 = time.perf_counter()
            for k in range(K):
                h.add(fn(k), ws[k], f"s{k}", r)
            h.engine.ctx.sync()
            t1 = time.perf_counter()
            h.get_result()
            res[m].append(t1 - t0)
    for m, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        print(json.dumps({"tool": "ingest_bench", "mode": m, "clients": K, "params": P, "accept_s": round(t, 4),
                          "GBs_into_hbm": round(4.0 * K * P / t / 1e9, 2)}), flush=True)
    shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
