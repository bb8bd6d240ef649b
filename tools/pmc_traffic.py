#!/usr/bin/env python3
"""HBM traffic per decode launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs).

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
1/2 of the bytes of wide coalesced streaming reads (16 B/lane loads), so the read side is doubled.
A grouped launch = one dispatch per kernel family (RLE, varint, FastPFOR, lane); traffic per launch
sums the last launch's four dispatches.  Writes profiles/pmc_traffic.json for bench.py."""
import csv
import json
import os
import sys


def last_launch(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if ("decode_family" in r["Kernel_Name"] or
                                                        "decode_lane" in r["Kernel_Name"])
            and r["Counter_Name"] == counter]
    by = {}
    for r in rows:
        k = r["Kernel_Name"]
        fam = k.split("<")[1].split(">")[0].split(",")[0] if "decode_family" in k else "lane"  # (<FAM, FS>: the family)
        by.setdefault(fam, []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {f: sorted(v)[-1][1] for f, v in by.items()}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    fetch = last_launch(os.path.join(out, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = last_launch(os.path.join(out, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fb = sum(fetch.values()) * 1024 * 2  # gfx950 FETCH_SIZE under-count correction
    wb = sum(write.values()) * 1024
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    res = {"tiles": 10000, "n_gpus": 1, "kernel_sources_sha256": bench.kernel_sources_sha256(),
           "fetch_kib_raw": fetch, "write_kib_raw": write,
           "read_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as is; KiB -> bytes"}
    os.makedirs("profiles", exist_ok=True)
    with open(os.path.join("profiles", "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
