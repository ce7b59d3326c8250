#!/usr/bin/env python3
"""Per-kernel launch durations and the idle gaps between back-to-back launches, from a rocprofv3 --kernel-trace csv
(diagnostic).  A gap is measured from the previous dispatch's end to this one's start when both run the same
kernel on the same queue (a series of burst launches); the first launch of each series has no gap.

  python tools/launch_gaps.py gpurun_out/r04_s5/gap_lib/lib_kernel_trace.csv [--match burst]
"""

import argparse
import csv
import json
import statistics


def summarize(path, match=""):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if match and match not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                         int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
    rows.sort()
    per = {}
    prev = {}
    for start, end, name, queue, blocks in rows:
        d = per.setdefault(name, {"durations_us": [], "gaps_us": [], "blocks": set()})
        d["durations_us"].append((end - start) / 1e3)
        d["blocks"].add(blocks)
        p = prev.get(queue)
        if p is not None and p[2] == name and start >= p[1]:
            d["gaps_us"].append((start - p[1]) / 1e3)
        prev[queue] = (start, end, name)
    out = []
    for name, d in per.items():
        dur, gaps = d["durations_us"], d["gaps_us"]
        out.append({"kernel": name[:160], "launches": len(dur), "blocks": sorted(d["blocks"])[:6],
                    "duration_us_median": round(statistics.median(dur), 2),
                    "duration_us_mean": round(statistics.fmean(dur), 2),
                    "gap_us_median": round(statistics.median(gaps), 2) if gaps else None,
                    "gap_us_mean": round(statistics.fmean(gaps), 2) if gaps else None,
                    "gap_share": round(sum(gaps) / (sum(gaps) + sum(dur)), 4) if gaps else None})
    return sorted(out, key=lambda x: -x["launches"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for rec in summarize(a.trace, a.match):
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
