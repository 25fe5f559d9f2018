#!/usr/bin/env python3
"""Turn rocprofv3 --pmc pass CSVs into the per-launch HBM traffic record that
bench.py reports as roofline.traffic.

    python scripts/traffic_json.py <pmc_dir> <kernel-substring> <out.json> [launch-desc]

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


def main():
    pmc_dir, kernel, dst = sys.argv[1:4]
    desc = sys.argv[4] if len(sys.argv) > 4 else ""
    c = per_dispatch(pmc_dir, kernel)
    fetch = c["FETCH_SIZE"] * 1024 * 2
    write = c["WRITE_SIZE"] * 1024
    rec = {"kernel": kernel, "launch": desc, "fetch_size_kb_raw": c["FETCH_SIZE"],
           "write_size_kb_raw": c["WRITE_SIZE"], "fetch_bytes_corrected": fetch, "write_bytes": write,
           "traffic_bytes": fetch + write,
           "correction": "FETCH_SIZE x 2, WRITE_SIZE x 1 (gfx950, profiles/r01/calib_*.csv)",
           "counters": c}
    alg = os.environ.get("ALG_BYTES")
    if alg:
        rec["alg_bytes"] = int(alg)
        rec["traffic_over_alg"] = (fetch + write) / int(alg)
    with open(dst, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in rec if k != "counters"}))


if __name__ == "__main__":
    main()
