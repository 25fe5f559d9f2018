#!/usr/bin/env python3
"""Turn rocprofv3 --pmc pass CSVs into the per-launch HBM traffic record that
bench.py reports as roofline.traffic.

    python scripts/traffic_json.py <pmc_dir> <kernel-substring> <out.json> [launch-desc] [--per-kernel]

The record is merged into <out.json>'s "records" list (a record of the same kernel is
replaced).  --per-kernel: one record per kernel whose name contains the substring.

gfx950 corrections (MI355X_MICROARCH.md HBM/rocprofv3 section, calibrated in
profiles/r01/calib_*.csv): FETCH_SIZE reports half the bytes of wide streaming
reads -> x2; WRITE_SIZE reads the bytes exactly.  Both counters are KB."""
import csv
import glob
import json
import os
import sys


def per_dispatch(pmc_dir, kernel):
    vals = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            if kernel not in row["Kernel_Name"]:
                continue
            key = (row["Counter_Name"], row["Dispatch_Id"], f)
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (name, _, _), v in vals.items():
        out.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}


def kernel_names(pmc_dir, sub):
    names = set()
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if sub in row["Kernel_Name"] and "mipx" in row["Kernel_Name"]:
                names.add(row["Kernel_Name"])
    return sorted(names)


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void mipx::", "").split("(")[0]


def record(pmc_dir, kernel, desc):
    c = per_dispatch(pmc_dir, kernel)
    fetch = c["FETCH_SIZE"] * 1024 * 2
    write = c["WRITE_SIZE"] * 1024
    rec = {"kernel": short(kernel), "launch": desc, "fetch_size_kb_raw": c["FETCH_SIZE"],
           "write_size_kb_raw": c["WRITE_SIZE"], "fetch_bytes_corrected": fetch, "write_bytes": write,
           "traffic_bytes": fetch + write,
           "correction": "FETCH_SIZE x 2, WRITE_SIZE x 1 (gfx950, profiles/r01/calib_*.csv)",
           "counters": c}
    alg = os.environ.get("ALG_BYTES")
    if alg:
        rec["alg_bytes"] = int(alg)
        rec["traffic_over_alg"] = (fetch + write) / int(alg)
    return rec


def main():
    args = [a for a in sys.argv[1:] if a != "--per-kernel"]
    pmc_dir, kernel, dst = args[:3]
    desc = args[3] if len(args) > 3 else ""
    names = kernel_names(pmc_dir, kernel) if "--per-kernel" in sys.argv else [kernel]
    recs = []
    if os.path.exists(dst):
        with open(dst) as f:
            old = json.load(f)
        recs = old.get("records", [old])
    for name in names:
        rec = record(pmc_dir, name, desc)
        recs = [r for r in recs if r.get("kernel") != rec["kernel"]] + [rec]
        print(json.dumps({k: rec[k] for k in rec if k != "counters"}))
    with open(dst, "w") as f:
        json.dump({"records": recs}, f, indent=1)


if __name__ == "__main__":
    main()
