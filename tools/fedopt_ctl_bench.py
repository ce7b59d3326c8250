#!/usr/bin/env python3
"""Round-end latency of the FedAvg-workflow FedOpt controller through the drop-ins, eager vs deferred (fused).

FedAvg's round (fedavg.py:200-240): every client result -> aggregator.accept_model (H2D staging), then
aggregator.aggregate_model() and the FedOpt controller's update_model() (fedopt_ctl.py:141-176: server step,
new global params to numpy).  Eager: aggregate_model() finalises on the device and returns host arrays, and
update_model copies them back and steps with K = 0.  Deferred (DeviceFedAvgModelAggregator(defer_result=True)):
the aggregate stays in HBM and update_model aggregates and steps in one launch per run.

  python tools/fedopt_ctl_bench.py [--clients 8 --params 125e6 --opt adam --rounds 4] [--defer]
"""

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=float, default=125e6)
    ap.add_argument("--opt", choices=["adam", "sgd"], default="adam")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--defer", action="store_true")
    args = ap.parse_args()
    import torch

    from nvflare_amd.app_common.aggregators import DeviceFedAvgModelAggregator
    from nvflare_amd.app_opt.pt.fedopt_ctl import DeviceFedOptUpdate
    from nvflare_amd.compat import FLMetaKey, FLModel

    K, P = args.clients, int(args.params)
    torch.manual_seed(0)

    class Flat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.randn(P) * 0.02)

    model = Flat().to("cuda:0")
    ctl = object.__new__(DeviceFedOptUpdate)  # the attributes the reference controller sets in run()
    ctl.device = torch.device("cuda:0")
    ctl.torch_model = model
    ctl.optimizer = (torch.optim.Adam(model.parameters(), lr=1e-3) if args.opt == "adam"
                     else torch.optim.SGD(model.parameters(), lr=1.0, momentum=0.9))
    ctl.lr_scheduler = None
    ctl.current_round = 0
    ctl.info = lambda msg: None
    agg = DeviceFedAvgModelAggregator(device=0, defer_result=args.defer)
    rng = np.random.default_rng(1)
    diffs = [{"w": (rng.standard_normal(P) * 0.01).astype(np.float32)} for _ in range(K)]
    g = FLModel(params={"w": model.w.detach().cpu().numpy().copy()})
    res = []
    for rnd in range(args.rounds):
        agg.reset_stats()
        t0 = time.perf_counter()
        for c in range(K):
            m = FLModel(params=diffs[c], current_round=rnd, meta={FLMetaKey.NUM_STEPS_CURRENT_ROUND: 1 + c,
                                                                  "client_name": f"site-{c}"})
            agg.accept_model(m)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        out = agg.aggregate_model()
        t2 = time.perf_counter()
        g = ctl.update_model(g, out)
        t3 = time.perf_counter()
        res.append({"round": rnd, "accept_s": round(t1 - t0, 4), "aggregate_s": round(t2 - t1, 4),
                    "update_model_s": round(t3 - t2, 4), "round_end_s": round(t3 - t1, 4)})
        print(json.dumps(res[-1]), flush=True)
    tail = res[1:] or res
    print(json.dumps({"tool": "fedopt_ctl_bench", "defer": args.defer, "clients": K, "params": P, "opt": args.opt,
                      "round_end_s_median": round(statistics.median(r["round_end_s"] for r in tail), 4),
                      "aggregate_s_median": round(statistics.median(r["aggregate_s"] for r in tail), 4),
                      "update_model_s_median": round(statistics.median(r["update_model_s"] for r in tail), 4),
                      "note": "round_end = aggregate_model() + update_model() (incl. the D2H of the new global params)"}))


if __name__ == "__main__":
    main()
