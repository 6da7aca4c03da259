"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace: separates launches of one kernel
at different configurations (e.g. the cfg2 fused kernel inside the bench's timed steps from its cfg5
launches), which rocprofv3's --stats merges.

Usage: python tools/trace_by_grid.py <run_kernel_trace.csv> [kernel-substring ...]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    acc = defaultdict(list)
    order = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if pats and not any(p in name for p in pats):
            continue
        key = (name, int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
        if key not in acc:
            order.append(key)
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = []
    for key in order:
        d = sorted(acc[key])
        out.append({"kernel": key[0][:120], "grid_x": key[1], "calls": len(d),
                    "avg_ms": sum(d) / len(d), "median_ms": d[len(d) // 2], "min_ms": d[0], "max_ms": d[-1]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
