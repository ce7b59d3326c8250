#!/usr/bin/env python3
"""Round-end latency of a scatter-and-gather FedOpt job through the drop-ins, eager vs deferred (fused).

ScatterAndGather's round (scatter_and_gather.py:224-349): every client result -> aggregator.accept
(H2D staging), then aggregator.aggregate() and shareable_gen.shareable_to_learnable() (FedOpt server step,
app_opt/pt/fedopt.py:184-270), then aggregator.reset().  Eager: aggregate() finalises on the device and
returns host arrays (D2H), the generator copies them back (H2D) and steps with K = 0.  Deferred
(--defer, InTimeAccumulateWeightedAggregator(defer_result=True)): aggregate() returns DeferredAggregate
values and the generator runs the K-client aggregation and the optimizer step in one launch.

  python tools/sag_fedopt_bench.py [--clients 8 --params 125e6 --keys 1 --opt adam --rounds 4] [--defer]

Prints one JSON line per round and a summary line (medians over rounds after the first).
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
    ap.add_argument("--keys", type=int, default=1)
    ap.add_argument("--opt", choices=["adam", "sgd"], default="adam")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--defer", action="store_true")
    ap.add_argument("--profile", action="store_true", help="cProfile the last round's aggregate + server step (stderr)")
    args = ap.parse_args()
    import torch

    from nvflare_amd.app_common.aggregators import InTimeAccumulateWeightedAggregator
    from nvflare_amd.app_opt.pt import PTFedOptModelShareableGenerator
    from nvflare_amd.compat import (DXO, AppConstants, DataKind, EventType, FLContext, MetaKey, ModelLearnableKey,
                                    ReservedKey, make_model_learnable)

    K, P = args.clients, int(args.params)
    sizes = np.full(args.keys, P // args.keys)
    sizes[-1] += P - sizes.sum()
    torch.manual_seed(0)

    class Flat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.layers = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(int(n)) * 0.02) for n in sizes])

    model = Flat()
    opt = ({"path": "torch.optim.Adam", "args": {"lr": 1e-3}} if args.opt == "adam"
           else {"path": "torch.optim.SGD", "args": {"lr": 1.0, "momentum": 0.9}})
    gen = PTFedOptModelShareableGenerator(optimizer_args=opt, source_model=model, device=0)
    fl_ctx = FLContext()
    gen.handle_event(EventType.START_RUN, fl_ctx)
    agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF, defer_result=args.defer)
    agg.handle_event(EventType.START_RUN, fl_ctx)
    names = [f"layers.{j}" for j in range(args.keys)]
    rng = np.random.default_rng(1)
    base = (rng.standard_normal(P, dtype=np.float32) * np.float32(1e-3))
    clients = []
    for k in range(K):
        flat = base * np.float32(1.0 + 0.01 * k)
        parts, off = {}, 0
        for name, n in zip(names, sizes):
            parts[name] = flat[off: off + int(n)]
            off += int(n)
        clients.append(parts)
    weights = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    rows = []
    for rnd in range(args.rounds):
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=True)
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(weights, {}), private=True, sticky=True)
        t0 = time.perf_counter()
        for k in range(K):
            s = DXO(DataKind.WEIGHT_DIFF, data=clients[k], meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1 + (37 * k) % 100}
                    ).to_shareable()
            s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
            s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
            assert agg.accept(s, fl_ctx)
        prof = None
        if args.profile and rnd == args.rounds - 1:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        t1 = time.perf_counter()
        aggr = agg.aggregate(fl_ctx)
        t2 = time.perf_counter()
        learnable = gen.shareable_to_learnable(aggr, fl_ctx)
        t3 = time.perf_counter()
        if prof is not None:
            import pstats

            prof.disable()
            pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
        agg.reset(fl_ctx)
        weights = learnable[ModelLearnableKey.WEIGHTS]
        row = {"round": rnd, "accept_s": round(t1 - t0, 4), "aggregate_s": round(t2 - t1, 4),
               "server_step_s": round(t3 - t2, 4), "round_end_s": round(t3 - t1, 4),
               "h2d_GBs": round(4.0 * K * P / (t1 - t0) / 1e9, 2)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    tail = rows[1:] or rows
    summary = {
        "tool": "sag_fedopt_bench", "defer": args.defer, "clients": K, "params": P, "keys": args.keys, "opt": args.opt,
        "round_end_s_median": statistics.median(r["round_end_s"] for r in tail),
        "aggregate_s_median": statistics.median(r["aggregate_s"] for r in tail),
        "server_step_s_median": statistics.median(r["server_step_s"] for r in tail),
        "accept_s_median": statistics.median(r["accept_s"] for r in tail),
        "note": "round_end = aggregate() + shareable_to_learnable() (incl. D2H of the returned host weights)",
    }
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
