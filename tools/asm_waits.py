#!/usr/bin/env python3
"""The vmcnt wait in front of each use of a pattern in a kernel's assembly (the FastPFOR window stage reads the
in-flight window through a DPP `wave_shl:1`): `s_waitcnt vmcnt(0)` there means the wait also drains the stores
and loads issued after the window request.
usage: asm_waits.py kernel.s [regex]      (kernel.s: hipcc --cuda-device-only -S, one kernel's lines)"""
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "wave_shl:1")
    for i, ln in enumerate(lines):
        if not pat.search(ln):
            continue
        wait = None
        for j in range(i - 1, max(0, i - 40), -1):
            if "s_waitcnt" in lines[j] and "vmcnt" in lines[j]:
                wait = (j + 1, lines[j].strip())
                break
        label = None
        for j in range(i - 1, max(0, i - 400), -1):
            if lines[j].startswith(".LBB") or lines[j].startswith("; %bb"):
                label = lines[j].split(":")[0].strip()
                break
        print(i + 1, ln.strip()[:60], "| wait:", wait, "|", label)


if __name__ == "__main__":
    main()
