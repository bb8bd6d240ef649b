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
        g = last.get("GRBM_GUI_ACTIVE")
        if g:  # derived utilisations (rocprofv3 metric definitions; CU_NUM = 256 on MI355X)
            cu = 256.0
            d = []
            if "SQ_ACTIVE_INST_VALU" in last:
                d.append("VALUBusy=%.1f%%" % (100 * last["SQ_ACTIVE_INST_VALU"] / cu / g))
            if "SQ_INST_CYCLES_SALU" in last:
                d.append("SALUBusy=%.1f%%" % (100 * last["SQ_INST_CYCLES_SALU"] / cu / g))
            if "SQ_ACTIVE_INST_LDS" in last:
                d.append("LDSBusy=%.1f%%" % (100 * last["SQ_ACTIVE_INST_LDS"] / cu / g))
            if "SQ_WAVE_CYCLES" in last:
                d.append("Occupancy=%.1f waves/SIMD" % (4 * last["SQ_WAVE_CYCLES"] / g / cu / 4))
            if "SQ_BUSY_CU_CYCLES" in last:
                d.append("CUbusy=%.1f%%" % (100 * 4 * last["SQ_BUSY_CU_CYCLES"] / cu / g))
            if "SQ_WAIT_INST_ANY" in last and "SQ_WAVE_CYCLES" in last:
                d.append("wait-issue/wave=%.1f%%" % (100 * last["SQ_WAIT_INST_ANY"] / last["SQ_WAVE_CYCLES"]))
            print("    derived:", " ".join(d), " GPU cycles=%.3g" % g)
