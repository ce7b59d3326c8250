"""Diagnostic: fp32 device tensors, drop-in vs torch-ROCm, the test_device_tensors_match_torch_rocm draw."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper  # noqa: E402
from oracle import fedavg_oracle as orc  # noqa: E402

rng = np.random.default_rng(5)
dt = torch.float32
sizes = {"a": (4097 * 3 + 5,), "b": (33, 7), "c": (), "d": (3072,), "e": (2048,)}
for K in (6, 130):
    clients = []
    for _ in range(K):
        c = {}
        for k, s in sizes.items():
            x = torch.from_numpy(np.asarray(rng.standard_normal(s) * 20, dtype=np.float32))
            c[k] = x.to(dt).to("cuda:0")
        clients.append(c)
    ws = [float(rng.random() * 4 + 0.05) for _ in range(K)]
    h = WeightedAggregationHelper()
    for k, (c, w) in enumerate(zip(clients, ws)):
        h.add(c, w, f"s{k}", 0)
    out = h.get_result()
    cnt = 0.0
    for w in ws:
        cnt += w
    for key in sizes:
        tot = clients[0][key].mul(ws[0])
        for c, w in zip(clients[1:], ws[1:]):
            tot.add_(c[key], alpha=w)
        pre = tot.clone()
        exp = tot.div_(cnt).cpu().numpy().reshape(-1)
        got = out[key].cpu().numpy().reshape(-1)
        d = np.nonzero(got != exp)[0]
        p = pre.cpu().numpy().reshape(-1)
        print(K, key, "diffs", d.size, "count", repr(cnt), "f32(count)", repr(float(np.float32(cnt))))
        s32 = np.float32(1.0) / np.float32(cnt)
        s64 = np.float32(1.0 / cnt)
        for i in d[:4]:
            print("   ", i, "got", repr(got[i]), "exp", repr(exp[i]), "pre", repr(p[i]), "pre*s32", repr(p[i] * s32),
                  "pre*s64", repr(p[i] * s64), "pre/f32c", repr(p[i] / np.float32(cnt)))
