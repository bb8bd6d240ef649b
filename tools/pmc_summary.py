#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: counters of the last dispatch of each decode kernel."""
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if "decode_family" in r["Kernel_Name"] or "decode_" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("<")[1].split(">")[0] if "<" in r["Kernel_Name"] else r["Kernel_Name"][:40]
            agg.setdefault(k, {}).setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    print("==", f)
    for k, d in agg.items():
        last = d[max(d)]
        print("  kernel", k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(last.items())))
