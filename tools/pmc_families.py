#!/usr/bin/env python3
"""Per-family SQ counter summary (re-collect the family counters on the current kernels).

Reads the rocprofv3 --pmc CSVs of `tools/gpu_session.sh sq_families` (gpurun_out/sqi_<family>: instruction
counts, gpurun_out/sqw_<family>: wave-cycle counters; each family decoded alone by tools/family_run.py, last
dispatch of its decode kernel) and prints counts and rates per CU per cycle (256 CUs, cycles = GRBM_GUI_ACTIVE /
8 XCDs).  Reference issue ceilings (profiles/r03/issue_rates.txt): ~1.46 VALU, ~0.75 SALU and ~1.35-1.6 VALU +
SALU wave-instructions per CU per cycle.
usage: pmc_families.py [gpurun_out] [suffix]"""
import csv
import os
import sys

CUS, XCDS, SIMDS = 256.0, 8.0, 1024.0


def last_dispatch(path):
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return None
    by = {}
    for r in csv.DictReader(open(f)):
        if "decode_family_kernel" not in r["Kernel_Name"]:
            continue
        by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return by[max(by)] if by else None


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    sfx = sys.argv[2] if len(sys.argv) > 2 else ""
    for fam in ("fastpfor", "varint", "rle", "lane"):
        a = last_dispatch(os.path.join(root, "sqi_%s%s" % (fam, sfx)))
        b = last_dispatch(os.path.join(root, "sqw_%s%s" % (fam, sfx)))
        if a is None:
            continue
        cyc = a["GRBM_GUI_ACTIVE"] / XCDS
        print("%s family alone (config-5 Id/Geometry plan%s)" % (fam, ", property plan" if sfx else ""))
        print("  cycles (GRBM_GUI_ACTIVE / 8 XCDs): %.3g  = %.3f ms at 2.4 GHz" % (cyc, cyc / 2.4e6))
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_BRANCH"):
            if k in a:
                print("  %-18s %.4g  = %.3f per CU per cycle" % (k, a[k], a[k] / CUS / cyc))
        if "SQ_INSTS_VALU" in a and "SQ_INSTS_SALU" in a:
            print("  VALU + SALU        %.3f per CU per cycle" % ((a["SQ_INSTS_VALU"] + a["SQ_INSTS_SALU"]) / CUS / cyc))
        if "SQ_WAVES" in a:
            print("  SQ_WAVES           %.4g" % a["SQ_WAVES"])
        if b:
            cb = b["GRBM_GUI_ACTIVE"] / XCDS
            wc = b.get("SQ_WAVE_CYCLES", 0.0)
            if wc:
                print("  waves resident per SIMD (SQ_WAVE_CYCLES x4 / 1024 SIMDs / cycles): %.2f" % (4 * wc / SIMDS / cb))
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if k in b:
                        print("  %-18s %.1f %% of wave cycles" % (k, 100 * b[k] / wc))
            for k in ("SQ_ACTIVE_INST_VALU", "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_LDS"):
                if k in b:
                    print("  %-18s %.4g quad-cycles = %.3f per CU per cycle (x4 cycles)" % (k, b[k], 4 * b[k] / CUS / cb))
        print()


if __name__ == "__main__":
    main()
