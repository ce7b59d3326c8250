#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel + memory-copy trace database (rocpd sqlite, ``--kernel-trace --memory-copy-trace``)
of a host-resident aggregation round (bench.py ``--also 2h``): per round, the client H2D DMAs, the aggregation kernels,
the result D2H and the gap to the next round, as JSON.  A round is delimited by its result D2H (the longest blit
kernel / copy after the aggregation kernels).

  python tools/trace_summary.py gpurun_out/r04_s3/trace2h/trace_results.db > profiles/r04/s3/trace2h_summary.json
"""

import json
import sqlite3
import statistics
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    ks = list(db.execute("select name, start, end from kernels order by start"))
    cs = list(db.execute("select name, start, end, size from memory_copies order by start"))
    ev = sorted([("K", n, s, e, 0) for n, s, e in ks] + [("C", n, s, e, z) for n, s, e, z in cs], key=lambda x: x[2])
    rounds, h2d = [], []
    agg = []
    for i, (kind, name, s, e, size) in enumerate(ev):
        if kind == "C" and size:
            h2d.append((s, e, size))
        elif kind == "K" and "fedavg" in name:
            agg.append((s, e))
        elif kind == "K" and "copyBuffer" in name and e - s > 1e6 and agg:
            nxt = ev[i + 1][2] if i + 1 < len(ev) else None
            rounds.append({"h2d_ms": round(sum(b - a for a, b, _ in h2d) / 1e6, 3),
                           "h2d_GBps": round(sum(z for *_, z in h2d) / max(sum(b - a for a, b, _ in h2d), 1), 2),
                           "h2d_bytes": int(sum(z for *_, z in h2d)),
                           "kernels": len(agg), "kernel_ms": round((agg[-1][1] - agg[0][0]) / 1e6, 3),
                           "kernels_end_to_d2h_start_ms": round((s - agg[-1][1]) / 1e6, 3),
                           "d2h_ms": round((e - s) / 1e6, 3),
                           "gap_to_next_ms": round((nxt - e) / 1e6, 3) if nxt else None})
            h2d, agg = [], []
    d2h = [r["d2h_ms"] for r in rounds]
    # the first round also holds the kernels of the workload traced before it (bench.py's main entry)
    print(json.dumps({"trace": sys.argv[1], "rounds": rounds,
                      "median": {k: statistics.median(r[k] for r in rounds) for k in
                                 ("h2d_ms", "h2d_GBps", "kernel_ms", "kernels_end_to_d2h_start_ms", "d2h_ms")},
                      "rounds_with_a_host_stall_over_5ms": sum(r["kernels_end_to_d2h_start_ms"] > 5 for r in rounds[1:]),
                      "d2h_GBps_median": round(500e6 / (statistics.median(d2h) * 1e6), 2) if d2h else None},
                     indent=1))


if __name__ == "__main__":
    main()
