#!/usr/bin/env python3
"""Round-end latency of get_result() for host-container results: one-shot (all launches, then one D2H)
vs pipelined egress (launches split at EGRESS_CHUNK, each finished chunk's D2H overlapping the rest).

  python tools/result_latency.py [--clients 8 --params 1e9 --rounds 3]
  python tools/result_latency.py --devices 8    # parameter buckets over 8 engines (all on device 0):
                                                # direct egress into one host array vs per-key concatenation
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=float, default=1e9)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--devices", type=int, default=1, help="parameter buckets (engines), all on device 0")
    args = ap.parse_args()
    import nvflare_amd.engine as E
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    K, P = args.clients, int(args.params)
    base = np.ones(P, dtype=np.float32)
    base[::7] = 0.5
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    default_chunk = E.EGRESS_CHUNK
    from nvflare_amd.sharding import ShardedFedAvg

    h = WeightedAggregationHelper(devices=[0] * args.devices if args.devices > 1 else None)
    if args.devices > 1:
        modes = (("direct", default_chunk), ("concat", default_chunk), ("direct", default_chunk), ("concat", default_chunk))
    else:
        modes = (("one_shot", 1 << 50), ("pipelined", default_chunk), ("one_shot", 1 << 50), ("pipelined", default_chunk))
    for mode, chunk in modes:
        E.EGRESS_CHUNK = chunk
        ShardedFedAvg.direct_egress = mode != "concat"
        ts = []
        for r in range(args.rounds):
            for k in range(K):
                h.add({"w": base}, ws[k], f"s{k}", r)
            for e in getattr(h.engine, "engines", [h.engine]):
                e.ctx.sync()
            t0 = time.perf_counter()
            out = h.get_result()
            ts.append(time.perf_counter() - t0)
            del out
        t = sorted(ts)[len(ts) // 2]
        print(json.dumps({"tool": "result_latency", "mode": mode, "clients": K, "params": P, "buckets": args.devices,
                          "egress_chunk_MiB": chunk >> 20 if chunk < (1 << 40) else None,
                          "get_result_ms": round(t * 1e3, 2), "result_GB": round(4 * P / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
