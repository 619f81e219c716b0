#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per-kernel call count / average duration
from the kernel-trace stats, and per-dispatch FETCH_SIZE / WRITE_SIZE (KB)
averaged per kernel from separate PMC passes.

HBM traffic per launch follows MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads, so
traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes).

usage: prof_summary.py <prof_dir> [--cells N] [--json out.json]
  <prof_dir>/trace/run_kernel_stats.csv, <prof_dir>/fetch/run_counter_collection.csv,
  <prof_dir>/write/run_counter_collection.csv (the PMC files are optional)
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def stats(path: Path):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            out[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3,
                                       float(row["TotalDurationNs"]) / 1e6)
    return out


def pmc(path: Path):
    """Mean counter value per kernel over the dispatches that did work: CG
    sweeps launched ahead of the host's convergence poll return at once after
    convergence and report ~0; they are left out (< 1 % of the kernel's max)."""
    acc = defaultdict(list)
    if not path.exists():
        return {}
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    out = {}
    for k, v in acc.items():
        big = [x for x in v if x > 0.01 * max(v)] or v
        out[k] = sum(big) / len(big)
    return out


def trace_real(path: Path):
    """Mean duration (us) per kernel over dispatches longer than 1 % of the
    kernel's longest (the same no-op filter), from the kernel trace."""
    acc = defaultdict(list)
    if not path.exists():
        return {}
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    out = {}
    for k, v in acc.items():
        big = [x for x in v if x > 0.01 * max(v)] or v
        out[k] = (len(big), sum(big) / len(big))
    return out


def main():
    d = Path(sys.argv[1])
    cells = None
    if "--cells" in sys.argv:
        cells = float(sys.argv[sys.argv.index("--cells") + 1])
    st = stats(d / "trace" / "run_kernel_stats.csv")
    real = trace_real(d / "trace" / "run_kernel_trace.csv")
    fe = pmc(d / "fetch" / "run_counter_collection.csv")
    wr = pmc(d / "write" / "run_counter_collection.csv")
    print(f"{'kernel':34s} {'calls':>6s} {'avg_us':>10s} {'work_n':>6s} {'work_us':>10s} "
          f"{'total_ms':>10s} {'FETCH_KB':>12s} {'WRITE_KB':>12s}"
          + ("  B/cell(2*fetch,write)" if cells else ""))
    for k, (n, avg, tot) in sorted(st.items(), key=lambda kv: -kv[1][2]):
        f = fe.get(k)
        w = wr.get(k)
        rn, ravg = real.get(k, (n, avg))
        line = f"{k:34s} {n:6d} {avg:10.2f} {rn:6d} {ravg:10.2f} {tot:10.2f} " \
               f"{(f'{f:12.0f}' if f is not None else ' ' * 12)} " \
               f"{(f'{w:12.0f}' if w is not None else ' ' * 12)}"
        if cells and (f is not None or w is not None):
            fb = 2 * f * 1024 / cells if f is not None else float("nan")
            wb = w * 1024 / cells if w is not None else float("nan")
            line += f"  {fb:6.2f},{wb:6.2f}"
        print(line)
    if "--json" in sys.argv:
        import json
        out = {}
        for k, (n, avg, tot) in st.items():
            f, w = fe.get(k), wr.get(k)
            rn, ravg = real.get(k, (n, avg))
            rec = {"calls": n, "avg_us": avg, "working_calls": rn, "working_avg_us": ravg}
            if f is not None and w is not None:
                rec["fetch_size_kb"] = f
                rec["write_size_kb"] = w
                rec["hbm_bytes_per_launch"] = (2.0 * f + w) * 1024.0
                if cells:
                    rec["hbm_bytes_per_cell"] = rec["hbm_bytes_per_launch"] / cells
            out[k] = rec
        sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
        from cfd_amd._native import HIP_LIB, kernel_source_sha
        from cfd_amd._sha import device_code_sha
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump({"source": str(d), "correction": "2*FETCH_SIZE + WRITE_SIZE",
                       "source_sha": kernel_source_sha(),
                       "device_sha": device_code_sha(HIP_LIB),
                       "cells_per_launch": cells, "kernels": out}, fh, indent=1)


if __name__ == "__main__":
    main()
