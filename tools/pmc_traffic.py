"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into a per-launch HBM-traffic record in
profiles/pmc_traffic.json (read by bench.py for its roofline.traffic field).

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE counts half the bytes of a
16-B/lane streaming read -> read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for 16-B/lane
streaming stores.  --aggregations N turns per-launch values into per-aggregation sums (burst kernel).

  python tools/pmc_traffic.py --fetch F.csv --write W.csv --kernel fedavg_tiles_epi \
      --config '{"clients":64,"params":1000000000,"tile":4096,"mode":"torch","epilogue":"adam"}' \
      --alg-bytes 280e9 --command "python bench.py --epilogue adam ..."
"""

import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def per_launch(path, kernel, counter, aggregations=0):
    """Mean counter value per launch of `kernel`, or, with `aggregations`, the sum over all its launches
    divided by the number of aggregations the profiled command ran (the burst kernel issues many launches
    per aggregation; their sizes differ at the end of a range)."""
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel {kernel!r} in {path}")
    if aggregations:
        return sum(vals) / aggregations, len(vals), None
    return sum(vals) / len(vals), len(vals), None


def kernel_name(path, kernel):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                return row["Kernel_Name"]
    return kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--config", required=True, help="JSON: clients, params, tile, mode, epilogue")
    ap.add_argument("--alg-bytes", type=float, required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--source", default="")
    ap.add_argument("--aggregations", type=int, default=0,
                    help="aggregations the profiled command ran (warmup + steps): traffic per aggregation = sum over "
                         "all launches / this (for kernels that issue several launches per aggregation)")
    a = ap.parse_args()
    fetch_kb, nf, _ = per_launch(a.fetch, a.kernel, "FETCH_SIZE", a.aggregations)
    write_kb, nw, _ = per_launch(a.write, a.kernel, "WRITE_SIZE", a.aggregations)
    read_b = 2.0 * fetch_kb * 1024
    write_b = write_kb * 1024
    rec = {
        "kernel": kernel_name(a.fetch, a.kernel),
        "config": json.loads(a.config),
        "command": a.command,
        "source": a.source or f"{a.fetch}, {a.write}",
        "launches_averaged": [nf, nw],
        "per": f"aggregation ({a.aggregations} in the profiled command, {nf // max(a.aggregations, 1)} launches each)"
               if a.aggregations else "launch",
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "read_bytes": int(read_b),
        "write_bytes": int(write_b),
        "bytes_per_launch": int(read_b + write_b),
        "algorithmic_bytes_per_launch": int(a.alg_bytes),
    }
    try:
        with open(OUT) as f:
            db = json.load(f)
    except (OSError, ValueError):
        db = {}
    records = [r for r in db.get("records", []) if r.get("config") != rec["config"]]
    records.append(rec)
    db["records"] = records
    with open(OUT, "w") as f:
        json.dump(db, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
