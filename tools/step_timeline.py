#!/usr/bin/env python3
"""One step's kernel timeline from a rocprofv3 --kernel-trace csv: start offset, duration and
the gap before each kernel, for the shortest complete step (steps open with FIRST, a
kernel-name substring).   python tools/step_timeline.py <trace dir> [FIRST]"""
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_oceanic_phys"
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mgcm::", ""))
                   for r in csv.DictReader(open(f))), key=lambda x: x[0])
    opens = [n for n, r in enumerate(rows) if first in r[2]]
    if len(opens) < 3:
        print("fewer than 3 steps found"); return
    # the shortest complete step (graph replays; bench.py's eager per-kernel timing pass
    # synchronises around every launch)
    spans = [(rows[opens[n + 1]][0] - rows[opens[n]][0], opens[n], opens[n + 1]) for n in range(len(opens) - 1)]
    _, a, b = min(spans)
    t0, prev = rows[a][0], rows[a][0]
    busy = 0
    for s, e, name in rows[a:b]:
        print("%9.2f %8.2f %7.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, name[:70]))
        prev = max(prev, e)
        busy += e - s
    print("step %.2f us, kernel time %.2f us (%d kernels)" % ((rows[b][0] - t0) / 1e3, busy / 1e3, b - a))


if __name__ == "__main__":
    main()
