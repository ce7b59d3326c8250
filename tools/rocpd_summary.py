"""rocprofv3's SQLite output (``*_results.db``, the rocpd schema ROCm 7.2 writes by default) into the CSV files the rest
of the tooling reads:

  --stats OUT.csv        per-kernel statistics in the ``--stats`` kernel_stats.csv format (Name, Calls, TotalDurationNs,
                         AverageNs, Percentage, MinNs, MaxNs, StdDev) from the kernel-dispatch view
  --durations OUT.json   every dispatch's duration (ns) of the kernels whose name contains --kernel, in dispatch order
                         (per-launch distributions: VERDICT r05 item 3)
  --pmc OUT.csv          counter values per dispatch in the pmc_counter_collection.csv columns tools/pmc_traffic.py reads
                         (Kernel_Name, Counter_Name, Counter_Value)

  python tools/rocpd_summary.py gpurun_out/x/rp/k2_results.db --stats profiles/r06/s1/adam_k2_kernel_stats.csv
"""

import argparse
import csv
import json
import math
import sqlite3


def kernel_rows(db):
    c = sqlite3.connect(db)
    return [(name, int(dur)) for name, dur in c.execute("select name, duration from kernels order by start")]


def stats(db, out):
    by = {}
    for name, dur in kernel_rows(db):
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values()) or 1
    rows = []
    for name, v in by.items():
        avg = sum(v) / len(v)
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / len(v))
        rows.append([name, len(v), sum(v), avg, 100.0 * sum(v) / total, min(v), max(v), sd])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 6), round(r[4], 2), r[5], r[6], round(r[7], 6)])
    return rows


def durations(db, kernel, out):
    d = [dur for name, dur in kernel_rows(db) if kernel in name]
    with open(out, "w") as f:
        json.dump({"kernel": kernel, "durations_ns": d, "calls": len(d)}, f)
    return d


def pmc(db, out):
    c = sqlite3.connect(db)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for row in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection "
                             "order by dispatch_id"):
            w.writerow(row)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--stats")
    ap.add_argument("--durations")
    ap.add_argument("--kernel", default="fedavg_tiles")
    ap.add_argument("--pmc")
    a = ap.parse_args()
    if a.stats:
        for r in stats(a.db, a.stats)[:4]:
            print(f"{r[1]:6d} x {r[3] / 1e3:10.2f} us  {r[0][:110]}")
    if a.durations:
        d = durations(a.db, a.kernel, a.durations)
        print(f"{len(d)} dispatches of *{a.kernel}*")
    if a.pmc:
        pmc(a.db, a.pmc)


if __name__ == "__main__":
    main()
