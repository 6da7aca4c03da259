"""Summarise tools/pmc.sh output: per-dispatch mean of every counter for one kernel.

Usage: python tools/summarize_pmc.py gpurun_out/pmc [kernel-substring]
FETCH_SIZE is doubled (gfx950 reports 1/2 of a wide streaming read, MI355X_MICROARCH.md §HBM);
sizes are KB in rocprofv3 -> bytes = value * 1024.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "cost_volume_gather_kernel"
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        per = defaultdict(lambda: defaultdict(float))
        for r in rows:
            if pat not in r.get("Kernel_Name", ""):
                continue
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for name, d in per.items():
            vals = list(d.values())
            acc[name].append(sum(vals) / len(vals))
    out = {k: sum(v) / len(v) for k, v in sorted(acc.items())}
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_corrected" in out and "hbm_write_bytes" in out:
        out["hbm_bytes_per_launch"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
