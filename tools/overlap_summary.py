#!/usr/bin/env python3
"""Summarise a rocprofv3 trace (--kernel-trace --memory-copy-trace,
--output-format csv) of tools/rb_overlap_trace.py: how much of the halo
copies' time runs while a k_rb1 launch is executing.

usage: python tools/overlap_summary.py DIR [label]  -> one JSON line
Halo copies are the device-to-device entries of the memory-copy trace and
the runtime's blit kernels (__amd_rocclr_copyBuffer*) of the kernel trace."""
import csv
import glob
import json
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(a, b, u):
    t = 0
    for x, y in u:
        if y <= a:
            continue
        if x >= b:
            break
        t += min(b, y) - max(a, x)
    return t


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else d
    kern = rows(f"{d}/**/*kernel_trace.csv")
    copies = rows(f"{d}/**/*memory_copy_trace.csv")
    rb = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern
          if "k_rb1" in r["Kernel_Name"]]
    halo = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern
            if "copyBuffer" in r["Kernel_Name"]]
    halo += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in copies
             if "DEVICE_TO_DEVICE" in r.get("Direction", "")]
    u = union(rb)
    tot = sum(b - a for a, b in halo)
    ov = sum(overlap(a, b, u) for a, b in halo)
    rb_busy = sum(b - a for a, b in u)
    print(json.dumps({"trace": label, "k_rb1_launches": len(rb), "halo_copies": len(halo),
                      "halo_copy_us": round(tot / 1e3, 1),
                      "halo_copy_us_during_k_rb1": round(ov / 1e3, 1),
                      "frac_overlapped": round(ov / tot, 3) if tot else None,
                      "k_rb1_busy_us": round(rb_busy / 1e3, 1)}))


if __name__ == "__main__":
    main()
