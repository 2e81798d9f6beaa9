#!/usr/bin/env python3
"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into a per-kernel HBM
traffic summary (JSON).  Counters are in KiB.  MI355X_MICROARCH.md (HBM section)
calibrates FETCH_SIZE only for 16-B-per-lane streams (it reads half the bytes);
the stencil kernels load and store 8 B per lane, so the factor is measured on
our own pattern: tools/pmc_calib (a copy of a known byte count, 8 B per lane)
profiled in the same passes gives bytes / counter for reads and for writes.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [CALIB_FETCH_DIR CALIB_WRITE_DIR]
"""
import collections
import csv
import glob
import json
import os
import sys

CALIB_KERNEL = "k_calib_copy8"
CALIB_BYTES = (96 << 20) * 8      # tools/pmc_calib.hip: bytes read (and written) per dispatch


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def calib_factor(d, counter):
    for k, (v, _) in per_kernel(d, counter).items():
        if CALIB_KERNEL in k and v > 0:
            return CALIB_BYTES / v
    return None


def main():
    fetch, write, out = sys.argv[1:4]
    ffac, wfac, src = 2.0, 1.0, "MI355X_MICROARCH.md 16-B-per-lane factors (FETCH x2, WRITE x1)"
    if len(sys.argv) > 5:
        cf, cw = calib_factor(sys.argv[4], "FETCH_SIZE"), calib_factor(sys.argv[5], "WRITE_SIZE")
        if cf and cw:
            ffac, wfac = cf, cw
            src = "measured on tools/pmc_calib (8-B-per-lane fp64 copy of %d B): FETCH x%.3f, WRITE x%.3f" % (
                CALIB_BYTES, cf, cw)
    fe, wr = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f_raw = fe.get(k, (0.0, 0))[0]
        w_raw = wr.get(k, (0.0, 0))[0]
        res[k] = {"fetch_bytes_raw": f_raw, "fetch_bytes_corrected": ffac * f_raw, "write_bytes_raw": w_raw,
                  "write_bytes_corrected": wfac * w_raw, "hbm_bytes_per_launch": ffac * f_raw + wfac * w_raw,
                  "dispatches": fe.get(k, (0, 0))[1]}
    json.dump({"note": "bytes per dispatch; correction: " + src + "; Infinity-Cache hits are counted by these "
                       "counters (memory-side L2 requests)", "fetch_factor": ffac, "write_factor": wfac,
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
