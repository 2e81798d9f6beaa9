#!/usr/bin/env python3
"""Per-kernel means of the SQ counters of one rocprofv3 --pmc pass (tools/sq_counters.sh):
VALU instructions per wave, VALU-active and wait fractions of the wave cycles."""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("mgcm::", "").replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    if any("SQ_LDS_BANK_CONFLICT" in c for c in acc.values()):
        print("%-36s %8s %9s %9s %9s %8s %8s %8s" % ("kernel", "waves", "valu/wv", "salu/wv", "ldsconf/wv", "lds%", "any%", "waitany%"))
        for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            w = max(c.get("SQ_WAVES", 1), 1)
            wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
            print("%-36s %8d %9.1f %9.1f %9.1f %8.1f %8.1f %8.1f" % (
                k[:36], w / max(n[(k, "SQ_WAVES")], 1), c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_SALU", 0) / w,
                c.get("SQ_LDS_BANK_CONFLICT", 0) / w, 100 * c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * c.get("SQ_WAIT_ANY", 0) / wc))
        return
    print("%-36s %8s %9s %9s %8s %8s %9s %9s" % ("kernel", "waves", "valu/wv", "vmem/wv", "lds/wv", "valu%", "wait%", "busycyc"))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
        w = max(c.get("SQ_WAVES", 1), 1)
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        print("%-36s %8d %9.1f %9.1f %8.1f %8.1f %9.1f %9.0f" % (
            k[:36], w / max(n[(k, "SQ_WAVES")], 1), c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_VMEM_RD", 0) / w,
            c.get("SQ_INSTS_LDS", 0) / w, 100 * c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            100 * c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_BUSY_CYCLES", 0) / max(n[(k, "SQ_BUSY_CYCLES")], 1)))


if __name__ == "__main__":
    main()
