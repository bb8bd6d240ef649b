#!/usr/bin/env python3
"""Per-op instruction counts from the opinst step (gpurun_out/opinst + gpurun_out/opinst.log)."""
import collections
import csv
import glob
import re

rows = list(csv.DictReader(open(glob.glob("gpurun_out/opinst/**/run_counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "covt::" not in r["Kernel_Name"]:
        continue
    agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
disp = sorted(agg)[4:]  # the first four decode dispatches are the warmup launch
jobs = [l for l in open("gpurun_out/opinst.log") if l.startswith("dispatch")]
print("%-14s %9s %11s %8s %8s %8s %8s %9s" % ("op", "streams", "values", "VALU/v", "SALU/v", "LDS/v", "B/v", "ms"))
for d, line in zip(disp, jobs):
    m = re.search(r"op (\S+)\s+streams\s+(\d+) values\s+(\d+) bytes\s+(\d+)", line)
    op, ns, v, b = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4))
    c = agg[d]
    ms = c["GRBM_GUI_ACTIVE"] / 8 / 2.4e6
    print("%-14s %9d %11d %8.3f %8.3f %8.3f %8.2f %9.3f" % (op, ns, v, c["SQ_INSTS_VALU"] / max(v, 1),
          c["SQ_INSTS_SALU"] / max(v, 1), c["SQ_INSTS_LDS"] / max(v, 1), b / max(v, 1), ms))
