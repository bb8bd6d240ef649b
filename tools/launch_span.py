#!/usr/bin/env python3
"""Duration of each grouped decode launch from a rocprofv3 kernel trace.

The bench's `kernel_ms` times one grouped launch with HIP events: the three decode_family_kernel
instantiations and decode_lane_kernel run concurrently on forked streams between a fork and a join
event.  rocprofv3's per-kernel averages therefore do not add up to it; this groups the trace's
decode dispatches four at a time (in dispatch order) and reports each launch's span, first start to
last end, per launch size (the lane kernel's grid tells the plans apart).

usage: launch_span.py gpurun_out/prof/run_kernel_trace.csv"""
import collections
import csv
import sys

DECODE = ("decode_family_kernel<0", "decode_family_kernel<1", "decode_family_kernel<2", "decode_lane_kernel")  # (<FAM, FS>)


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if any(k in r["Kernel_Name"] for k in DECODE)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    spans = collections.defaultdict(list)
    i = 0
    while i + 4 <= len(rows):
        grp = rows[i:i + 4]
        kinds = sorted(next(k for k in DECODE if k in r["Kernel_Name"]) for r in grp)
        if kinds != sorted(DECODE):
            i += 1
            continue
        lane = next(r for r in grp if "decode_lane_kernel" in r["Kernel_Name"])
        t0 = min(int(r["Start_Timestamp"]) for r in grp)
        t1 = max(int(r["End_Timestamp"]) for r in grp)
        spans[int(lane["Grid_Size_X"]) // 256].append((t1 - t0) / 1e6)
        i += 4
    print("grouped decode launches (fork/join of decode_family_kernel<0,1,2> + decode_lane_kernel):")
    for lane_wgs, v in sorted(spans.items()):
        v = sorted(v)
        print("  lane grid %8d WGs: %3d launches  span mean %.3f ms  median %.3f ms  min %.3f  max %.3f"
              % (lane_wgs, len(v), sum(v) / len(v), v[len(v) // 2], v[0], v[-1]))


if __name__ == "__main__":
    main()
