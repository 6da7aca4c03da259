"""Print a rocprofv3 run_kernel_stats.csv as per-step milliseconds: python tools/kstats.py <csv> [steps] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel time %.2f ms in all, %.3f ms per step (%g steps)" % (tot / 1e6, tot / 1e6 / steps, steps))
for r in rows[:top]:
    n = r["Name"].replace("void mvs::(anonymous namespace)::", "").replace("_ZN3mvs12_GLOBAL__N_1", "")[:78]
    print("%-80s %5s calls %8.3f ms/step  avg %7.3f ms" % (n, r["Calls"], float(r["TotalDurationNs"]) / 1e6 / steps,
                                                          float(r["AverageNs"]) / 1e6))
