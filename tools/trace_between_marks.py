"""Per-kernel totals of a rocprofv3 kernel trace (run_kernel_trace.csv) between the last two marker
launches (torch.cumprod's rocprim single_scan_kernel): the timed step of
tools/train_step_prof.py under MVS_TRAIN_MARK=1.  Usage: python tools/trace_between_marks.py TRACE [N]"""
import collections
import csv
import sys

MARK = "single_scan_kernel"   # torch.cumprod of one element (rocprim scan)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if MARK in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("fewer than two marks")
    a, b = marks[-2], marks[-1]
    sel = rows[a + 1:b]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += d
        agg[r["Kernel_Name"]][1] += 1
    tot = sum(v[0] for v in agg.values())
    span = int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"])
    print("step: %d kernels, %.1f ms of kernel time, %.1f ms wall between marks" % (len(sel), tot / 1e6, span / 1e6))
    for name, (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print("%5.1f%% %9.2f ms %5d calls  %s" % (100.0 * d / tot, d / 1e6, n, name[:110]))


if __name__ == "__main__":
    main()
