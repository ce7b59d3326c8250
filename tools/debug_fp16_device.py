"""Diagnostic: fp16 device-tensor aggregation, torch-ROCm vs the drop-in vs a host model of both roundings."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper  # noqa: E402


def r16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


rng = np.random.default_rng(5)
dt = torch.float16
for K in (6, 127, 128, 129, 130):
    clients = [torch.from_numpy(np.asarray(rng.standard_normal((33, 7)) * 20, dtype=np.float32)).to(dt).to("cuda:0")
               for _ in range(K)]
    ws = [float(rng.random() * 4 + 0.05) for _ in range(K)]
    h = WeightedAggregationHelper()
    for k, (c, w) in enumerate(zip(clients, ws)):
        h.add({"b": c}, w, f"s{k}", 0)
    got = h.get_result()["b"].float().cpu().numpy().reshape(-1)
    tot = clients[0].mul(ws[0])
    steps_ref = []
    for c, w in zip(clients[1:], ws[1:]):
        tot.add_(c, alpha=w)
    cnt = sum(ws)
    pre_ref = tot.float().cpu().numpy().reshape(-1)
    exp = tot.clone().div_(cnt).float().cpu().numpy().reshape(-1)
    vs = [c.float().cpu().numpy().reshape(-1).astype(np.float64) for c in clients]
    t = r16(vs[0] * np.float64(np.float32(ws[0])))
    for v, w in zip(vs[1:], ws[1:]):
        t = r16((v * np.float64(np.float32(w)) + t.astype(np.float64)).astype(np.float32))
    model_pre = t
    model = r16(t * np.float32(np.float32(1.0) / np.float32(cnt)))
    t1 = r16(vs[0] * np.float64(np.float32(ws[0])))
    for v, w in zip(vs[1:], ws[1:]):  # one rounding: the exact fma straight to fp16 (v_fma_mixlo_f16)
        t1 = (v * np.float64(np.float32(w)) + t1.astype(np.float64)).astype(np.float16).astype(np.float32)
    print("   single-rounding model: pre_ref!=single", int((pre_ref != t1).sum()))
    print("K", K, "got!=exp", int((got != exp).sum()), "pre_ref!=model_pre", int((pre_ref != model_pre).sum()),
          "got!=model", int((got != model).sum()), "exp!=model", int((exp != model).sum()))
    for i in np.nonzero(got != exp)[0][:3]:
        print("  ", i, "got", got[i], "exp", exp[i], "model", model[i], "pre_ref", pre_ref[i], "model_pre", model_pre[i])
