#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (--kernel-trace --memory-copy-trace,
--output-format csv) of tools/rb_overlap_trace.py: for the in-process slab
group's RB-SOR iterations, how much of the halo copies' execution runs while
a k_rb1 launch executes, and the iteration period.

usage: python tools/overlap_summary.py DIR [label]  -> one JSON line
Halo copies are the runtime's blit kernels (__amd_rocclr_copyBuffer) that
start after the first k_rb1 launch (the setup's uploads come before). The
iteration period is the spacing of one stream's k_rb_edge_r launches."""
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
    out = []
    for a, b in sorted(iv):
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
    iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    rb = [r for r in kern if "k_rb1" in r["Kernel_Name"]]
    t0 = min(iv(r)[0] for r in rb)
    rb_streams = {r["Stream_Id"] for r in rb}
    halo = [iv(r) for r in kern if "copyBuffer" in r["Kernel_Name"] and iv(r)[0] >= t0]
    side = [iv(r) for r in kern if "copyBuffer" in r["Kernel_Name"] and iv(r)[0] >= t0
            and r["Stream_Id"] not in rb_streams]
    u = union([iv(r) for r in rb])
    tot = sum(b - a for a, b in halo)
    ov = sum(overlap(a, b, u) for a, b in halo)
    s0 = sorted(rb_streams)[0]
    er = sorted(iv(r)[0] for r in kern if "k_rb_edge_r" in r["Kernel_Name"]
                and r["Stream_Id"] == s0)
    per = [(b - a) / 1e3 for a, b in zip(er, er[1:])]
    per.sort()
    print(json.dumps({"trace": label, "k_rb1_launches": len(rb), "halo_copies": len(halo),
                      "halo_copies_on_side_streams": len(side),
                      "halo_copy_us": round(tot / 1e3, 1),
                      "halo_copy_us_during_k_rb1": round(ov / 1e3, 1),
                      "frac_overlapped": round(ov / tot, 3) if tot else None,
                      "iteration_period_us_median": round(per[len(per) // 2], 1) if per else None,
                      "k_rb1_busy_us": round(sum(b - a for a, b in u) / 1e3, 1)}))


if __name__ == "__main__":
    main()
