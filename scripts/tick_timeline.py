"""Per-tick kernel timeline from a rocprofv3 kernel trace: each kernel's duration and the idle gap
before it, so a small shape's tick can be split into kernel time and launch gaps.

usage: python scripts/tick_timeline.py KERNEL_TRACE.csv SKIP_TICKS N_TICKS
A tick starts at a control launch (control_kernel / control_fast_kernel / control_fastfb_kernel /
control_resident_kernel); control_slow_kernel belongs to the tick it follows.
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("rg::", "")
    return n.split("<")[0]


def main():
    path, skip, count = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ticks = []
    for r in rows:
        if r[2].startswith("control_") and r[2] != "control_slow_kernel":
            ticks.append([r])
        elif ticks:
            ticks[-1].append(r)
    win = ticks[skip:skip + count]
    if len(win) < 2:
        sys.exit(f"only {len(ticks)} ticks in the trace")
    dur, gap = defaultdict(list), defaultdict(list)
    periods = []
    for i, t in enumerate(win):
        prev_end = win[i - 1][-1][1] if i else None
        for s, e, n in t:
            dur[n].append(e - s)
            if prev_end is not None:
                gap[n].append(s - prev_end)
            prev_end = e
        if i:
            periods.append(t[0][0] - win[i - 1][0][0])
    print(f"ticks {skip}..{skip + len(win) - 1}: period {sum(periods) / len(periods) / 1e3:.2f} us")
    for n in dur:
        g = gap[n]
        print(f"  {n:32s} {sum(dur[n]) / len(dur[n]) / 1e3:8.2f} us   gap before {sum(g) / max(len(g), 1) / 1e3:6.2f} us"
              f"   launches {len(dur[n])}")


if __name__ == "__main__":
    main()
