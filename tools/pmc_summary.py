#!/usr/bin/env python3
"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into a per-kernel HBM
traffic summary (JSON), corrected as /opt/skills/guides/MI355X_MICROARCH.md
(HBM section) prescribes: counters are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads, so it is doubled.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch, write, out = sys.argv[1:4]
    fe, wr = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f_raw = fe.get(k, (0.0, 0))[0]
        w = wr.get(k, (0.0, 0))[0]
        res[k] = {"fetch_bytes_raw": f_raw, "fetch_bytes_corrected": 2.0 * f_raw, "write_bytes": w,
                  "hbm_bytes_per_launch": 2.0 * f_raw + w, "dispatches": fe.get(k, (0, 0))[1]}
    json.dump({"note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, bytes per dispatch; "
                       "Infinity-Cache hits are counted by these counters", "kernels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
